# GPU box: cost of the per-kernel dispatch stamps on the step rate -- bench lines with every step
# timed, every 5th, and only the first.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g19
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
for r in 1 2; do
for wl in knn range ppknn; do
  for te in 1 5 1000; do
    timeout -k 10 200 python -u bench.py --workload $wl --steps 50 --warmup 5 --time-every $te $B > gpurun_out/g19/b_${wl}_$te.log 2>&1 || { tail -5 gpurun_out/g19/b_${wl}_$te.log; exit 1; }
    echo "$wl te=$te $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"timed_steps": [0-9]*' gpurun_out/g19/b_${wl}_$te.log | tr '\n' ' ')"
  done
done
done
