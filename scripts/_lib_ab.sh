# GPU box: the bench line of one workload under several library builds / env settings, twice each
#   CASES="product nogen nogen:GEOHIP_INGEST_ABLATE=1" WL=ingest bash scripts/_lib_ab.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for c in $CASES; do
    lib=${c%%:*}; envs=""; [ "$c" != "$lib" ] && envs=${c#*:}
    so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
    env GEOHIP_LIB=$so $envs timeout -k 10 200 python -u bench.py --workload ${WL:-knn} --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line ${BENCH_ARGS:-} > gpurun_out/lab_$r.log 2>&1 || { tail -20 gpurun_out/lab_$r.log; exit 1; }
    echo "$c $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*' gpurun_out/lab_$r.log | tr '\n' ' ')"
  done
done
