# GPU box: staged range emission (range_fused, knn_pass fused range) -- parity of range / kNN /
# C5 / look-back tests, bench lines for range, c5, knn, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g12
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_lookback.py tests/test_gpu_incremental.py \
    -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "range or knn or c5 or c1 or lookback" \
    > gpurun_out/g12/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g12/pytest.log; exit 1; }
tail -1 gpurun_out/g12/pytest.log
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
for wl in range c5 knn; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 100 --warmup 5 $B > gpurun_out/g12/bench_$wl.log 2>&1 || { tail -20 gpurun_out/g12/bench_$wl.log; exit 2; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/g12/bench_$wl.log | tr '\n' ' ')"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_ingest_traj.py -m gpu -x -q -p no:cacheprovider --timeout 240 \
    --timeout-method thread > gpurun_out/g12/pytest_ingest.log 2>&1 || { echo "ingest pytest failed"; tail -30 gpurun_out/g12/pytest_ingest.log; exit 3; }
tail -1 gpurun_out/g12/pytest_ingest.log
timeout -k 10 300 python -u bench.py --workload ingest --steps 30 --warmup 3 $B > gpurun_out/g12/bench_ingest.log 2>&1 || { tail -20 gpurun_out/g12/bench_ingest.log; exit 4; }
echo "ingest $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/g12/bench_ingest.log | tr '\n' ' ')"
