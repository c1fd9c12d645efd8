# GPU box: point-polygon parity subset, then the C4 / ppjoin bench lines under rocprof kernel stats
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v tests/test_gpu_parity.py tests/test_gpu_holes.py tests/test_gpu_ppoly_ext.py tests/test_gpu_fullscale.py tests/test_gpu_incremental.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K:-ppoly or hole or c4 or cell_class}" > gpurun_out/pytest_pp.log 2>&1 || { tail -30 gpurun_out/pytest_pp.log; exit 1; }
tail -1 gpurun_out/pytest_pp.log
for WL in ${WLS:-ppoly ppjoin}; do
GEOHIP_HOST_PROFILE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $WL -- python3 bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof/$WL.log 2>&1
grep '^{' gpurun_out/prof/$WL.log | cut -c1-300
grep -m1 "cell classes" gpurun_out/prof/$WL.log || true
python3 scripts/kstats.py gpurun_out/prof/${WL}_kernel_stats.csv 2>/dev/null | head -8 || true
done
