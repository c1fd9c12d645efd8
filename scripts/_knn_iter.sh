# GPU box: kNN parity subset, phase trace, then the C2 / C5 bench lines and a kernel-stats profile
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "${K:-knn or c2 or c5 or merge or smoke or incremental or threads or multirank}" > gpurun_out/knn_tests.log 2>&1 \
  || { tail -40 gpurun_out/knn_tests.log; exit 1; }
tail -2 gpurun_out/knn_tests.log
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 0 > gpurun_out/tr_c2.log 2>&1
timeout -k 10 120 python scripts/trace_pass.py 25000000 100 0.05 1000 0 > gpurun_out/tr_c5.log 2>&1
python scripts/show_trace.py gpurun_out/tr_c2.log 2>/dev/null | head -20 || true
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line > gpurun_out/b_knn_$i.log 2>&1
  grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*' gpurun_out/b_knn_$i.log | tr '\n' ' '; echo
done
timeout -k 10 200 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-cells-line > gpurun_out/b_c5.log 2>&1
grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*' gpurun_out/b_c5.log | tr '\n' ' '; echo
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_knn -o knn -- python $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line > $GRAFT_REPO_ROOT/gpurun_out/prof_knn.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/prof_knn -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -4 {}'
