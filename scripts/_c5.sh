set -e
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "fused or c5" > gpurun_out/pytest_c5.log 2>&1
tail -1 gpurun_out/pytest_c5.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1
grep '^{' gpurun_out/bench_c5.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o c5 -- python3 bench.py --workload c5 --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/prof/c5.log 2>&1
