# GPU box: join / point-polygon parity tests, then C4 and C3 bench lines with kernel stats
set -e
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_holes.py tests/test_gpu_ppoly_ext.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "join or ppoly or c3 or c4 or hole" > gpurun_out/pytest_bin.log 2>&1 || { tail -30 gpurun_out/pytest_bin.log; exit 1; }
tail -1 gpurun_out/pytest_bin.log
for WL in ppoly join; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $WL -- python3 bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof/$WL.log 2>&1
grep '^{' gpurun_out/prof/$WL.log | cut -c1-400
python3 scripts/kstats.py gpurun_out/prof/${WL}_kernel_stats.csv 2>/dev/null | head -8 || true
done
