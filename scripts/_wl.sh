# GPU box: bench line + rocprofv3 kernel stats of one workload.  WL=<workload> [STEPS=..]
set -e
WL=${WL:-join}
STEPS=${STEPS:-20}
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload $WL --steps $STEPS --warmup 3 --no-cpu-baseline > gpurun_out/bench_$WL.log 2>&1
grep '^{' gpurun_out/bench_$WL.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $WL -- python3 bench.py --workload $WL --steps $STEPS --warmup 3 --no-cpu-baseline > gpurun_out/prof/$WL.log 2>&1
python3 scripts/kstats.py gpurun_out/prof/${WL}_kernel_stats.csv 2>/dev/null | head -25 || true
