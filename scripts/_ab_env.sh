# GPU box: alternating A/B of an environment switch on the C2 bench line (same box)
#   VAR=SOME_SWITCH A=0 B=1 WL=knn bash scripts/_ab_env.sh  (the program must read VAR)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in ${A:-0} ${B:-1}; do
    env ${VAR}=$v timeout -k 10 200 python -u bench.py --workload ${WL:-knn} --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line > gpurun_out/ab_$v.log 2>&1
    echo "$VAR=$v $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*' gpurun_out/ab_$v.log | tr '\n' ' ')"
  done
done
