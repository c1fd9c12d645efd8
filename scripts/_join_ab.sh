# GPU box: C3 bench line, current library vs scripts/ab/libgeohip_prev.so, alternating (same box)
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
for L in spatialflink_amd/libgeohip.so scripts/ab/libgeohip_prev.so; do
GEOHIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --workload join --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1
echo "$L $(grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['roofline']['avg_kernel_us'],1))")"
done
done
