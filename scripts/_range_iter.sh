# GPU box: range / C5 parity tests, C5 phase trace, C5 and range bench lines with kernel stats
set -e
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_incremental.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "range or c5 or c1 or knn" > gpurun_out/pytest_range.log 2>&1 || { tail -30 gpurun_out/pytest_range.log; exit 1; }
tail -1 gpurun_out/pytest_range.log
timeout -k 10 120 python scripts/trace_pass.py 25000000 100 0.05 1000 -1 > gpurun_out/tr_c5.log 2>&1
for WL in c5 range; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $WL -- python3 bench.py --workload $WL --steps 50 --warmup 3 --no-cpu-baseline --no-e2e --no-pipelined > gpurun_out/prof/$WL.log 2>&1
grep '^{' gpurun_out/prof/$WL.log | cut -c1-200
python3 scripts/kstats.py gpurun_out/prof/${WL}_kernel_stats.csv 2>/dev/null | head -3 || true
done
