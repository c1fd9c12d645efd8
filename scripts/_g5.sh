# GPU box: join binning v2 (16-B records) + direct ALL-pair stores -- parity, bench, kernel stats;
# kNN bench after the final revert.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g5
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_multirank.py tests/test_gpu_threads.py \
    -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "join" > gpurun_out/g5/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -30 gpurun_out/g5/pytest.log; exit 1; }
tail -1 gpurun_out/g5/pytest.log
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
timeout -k 10 300 python -u bench.py --workload join --steps 30 --warmup 3 $B > gpurun_out/g5/bench_join.log 2>&1 || { tail -20 gpurun_out/g5/bench_join.log; exit 2; }
grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/g5/bench_join.log | tr '\n' ' '; echo
timeout -k 10 200 python -u bench.py --workload knn --steps 100 --warmup 5 $B > gpurun_out/g5/bench_knn.log 2>&1 || { tail -20 gpurun_out/g5/bench_knn.log; exit 3; }
grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*' gpurun_out/g5/bench_knn.log | tr '\n' ' '; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g5/prof -o join -- \
    python3 bench.py --workload join --steps 20 --warmup 3 $B > gpurun_out/g5/prof_join.log 2>&1 || { tail -5 gpurun_out/g5/prof_join.log; exit 4; }
python3 scripts/kstats.py gpurun_out/g5/prof/join_kernel_stats.csv | head -16
