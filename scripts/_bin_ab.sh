# GPU box: C4 and C3 bench lines, current library vs scripts/ab/libgeohip_prev.so, alternating (same box)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_holes.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "join or ppoly or c3 or c4 or hole" > gpurun_out/pytest_binab.log 2>&1 || { tail -30 gpurun_out/pytest_binab.log; exit 1; }
tail -1 gpurun_out/pytest_binab.log
for WL in ${WLS:-ppoly join}; do
for r in 1 2; do
for L in spatialflink_amd/libgeohip.so scripts/ab/libgeohip_prev.so; do
GEOHIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1
echo "$WL $L $(grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['roofline']['avg_kernel_us'],1))")"
done
done
done
