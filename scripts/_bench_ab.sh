# GPU box: C2 bench line, current vs previous bench.py, alternating (N = 1)
set -e
mkdir -p gpurun_out
for r in 1 2; do
for B in bench.py bench_prev.py; do
timeout -k 10 200 python -u $B --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-pipelined > gpurun_out/ab.log 2>&1
echo "$B $(grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,1), round(d['roofline']['avg_kernel_us'],1))")"
done
done
