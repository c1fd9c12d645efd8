# GPU box: kNN parity tests, then phase traces of the C2 pass (interleaved vs chunk iterations)
# and the default bench line.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "knn or c2" > gpurun_out/pytest_knn.log 2>&1
tail -1 gpurun_out/pytest_knn.log
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 0 > gpurun_out/tr_c2.log 2>&1
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 16 >> gpurun_out/tr_c2.log 2>&1
timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1
grep '^{' gpurun_out/bench.log | cut -c1-900
