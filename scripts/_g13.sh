# GPU box: point-polygon subcells from the cell quotient; join kernels timed one by one -- parity,
# bench lines.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g13
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppoly_ext.py tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_holes.py \
    tests/test_gpu_incremental.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "ppoly or polygon or c4 or hole or join or c3" \
    > gpurun_out/g13/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g13/pytest.log; exit 1; }
tail -1 gpurun_out/g13/pytest.log
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
for wl in ppoly join ppjoin; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 3 $B > gpurun_out/g13/bench_$wl.log 2>&1 || { tail -20 gpurun_out/g13/bench_$wl.log; exit 2; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/g13/bench_$wl.log | tr '\n' ' ')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g13/prof -o ppoly -- \
    python3 bench.py --workload ppoly --steps 12 --warmup 2 $B > gpurun_out/g13/prof_ppoly.log 2>&1 || { tail -5 gpurun_out/g13/prof_ppoly.log; exit 3; }
python3 scripts/kstats.py gpurun_out/g13/prof/ppoly_kernel_stats.csv > gpurun_out/g13/ks.txt; head -4 gpurun_out/g13/ks.txt
