# GPU box: rocprofv3 kernel stats of one workload's bench under several library builds / env settings
#   CASES="product psa1 psa2:GEOHIP_X=1" WL=ppoly bash scripts/_lib_prof.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lprof
export TMPDIR=/tmp
for c in $CASES; do
  lib=${c%%:*}; envs=""; [ "$c" != "$lib" ] && envs=${c#*:}
  so=$PWD/spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=$PWD/spatialflink_amd/libgeohip_$lib.so
  tag=$(echo "$c" | tr -c 'a-zA-Z0-9_\n' '_')
  for kv in $envs; do export "$kv"; done
  GEOHIP_LIB=$so GEOHIP_HOST_PROFILE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof -o $tag -- python3 bench.py --workload ${WL:-knn} --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line ${BENCH_ARGS:-} > gpurun_out/lprof/$tag.log 2>&1 || { tail -20 gpurun_out/lprof/$tag.log; exit 1; }
  for kv in $envs; do unset "${kv%%=*}"; done
  echo "== $c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lprof/$tag.log) $(grep -m1 'ppoly stream:' gpurun_out/lprof/$tag.log)"
  python3 scripts/kstats.py gpurun_out/lprof/${tag}_kernel_stats.csv | sed -n 2,${TOP:-6}p
done
