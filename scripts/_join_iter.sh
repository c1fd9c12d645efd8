# GPU box: join parity tests, then the C3 bench line with kernel stats
set -e
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "join or c3" > gpurun_out/pytest_join.log 2>&1 || { tail -30 gpurun_out/pytest_join.log; exit 1; }
tail -1 gpurun_out/pytest_join.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o join -- python3 bench.py --workload join --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof/join.log 2>&1
grep '^{' gpurun_out/prof/join.log | cut -c1-200
python3 scripts/kstats.py gpurun_out/prof/join_kernel_stats.csv 2>/dev/null | head -4 || true
