# GPU box: kNN / C5 parity tests, C2 phase trace, C2 bench line
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_incremental.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "knn or c2 or c5" > gpurun_out/pytest_knn.log 2>&1 || { tail -30 gpurun_out/pytest_knn.log; exit 1; }
tail -1 gpurun_out/pytest_knn.log
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 0 > gpurun_out/tr_c2.log 2>&1
timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1
grep '^{' gpurun_out/bench.log | cut -c1-1000
