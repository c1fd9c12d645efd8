#!/bin/bash
# GPU box, end of round 6: every workload's bench line on the final tree (the PMC summaries already
# in profiles/, so `traffic` is this tree's) saved for profiles/r06_bench_*.json, the default line,
# the kNN phase trace and the dense point-polygon window's per-call lines.  Each GPU step has its
# own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lines
mkdir -p $OUT
export TMPDIR=/tmp
for w in ${WORKLOADS:-knn range c5 join ppoly ingest ppjoin ppknn knn_incr ppoly_incr}; do
  steps=50; [ "$w" = "join" ] || [ "$w" = "ppoly" ] || [ "$w" = "ppjoin" ] && steps=20
  timeout -k 10 300 python -u bench.py --workload "$w" --steps $steps --warmup 3 > $OUT/bench_$w.log 2>&1 \
      || { echo "bench $w failed"; tail -20 $OUT/bench_$w.log; exit 2; }
  grep '^{' $OUT/bench_$w.log | cut -c1-120
done
if [ "${DEFAULT:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py > $OUT/bench_default.log 2>&1 || { echo "bench default failed"; exit 3; }
  grep '^{' $OUT/bench_default.log | cut -c1-120
fi
if [ "${EXTRA:-1}" = "1" ]; then
  timeout -k 10 200 python -u scripts/trace_pass.py > $OUT/knn_trace.log 2>&1 || { echo "trace failed"; exit 4; }
  GEOHIP_HOST_PROFILE=1 timeout -k 10 400 python -u scripts/ppoly_reruns.py > $OUT/ppoly_dense.log 2>&1 || { echo "dense failed"; tail -5 $OUT/ppoly_dense.log; exit 5; }
fi
echo done
