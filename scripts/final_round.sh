#!/bin/bash
# GPU box, end of round: the GPU suite, every bench workload's line, rocprofv3 kernel stats of each
# bench command (copied to profiles/r06_*).  Every GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final/prof
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      > gpurun_out/final/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/final/pytest_gpu.log
fi
for w in ${WORKLOADS:-knn range c5 join ppoly ingest ppjoin ppknn knn_incr ppoly_incr}; do
  steps=50; [ "$w" = "join" ] || [ "$w" = "ppoly" ] || [ "$w" = "ppjoin" ] && steps=20
  timeout -k 10 300 python -u bench.py --workload "$w" --steps $steps --warmup 3 \
      > gpurun_out/final/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 gpurun_out/final/bench_$w.log; exit 2; }
  grep '^{' gpurun_out/final/bench_$w.log | cut -c1-160
  [ "${PROF:-1}" = "1" ] || continue
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o $w -- \
      python3 bench.py --workload "$w" --steps $steps --warmup 3 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line \
      > gpurun_out/final/prof/bench_$w.log 2>&1 || { echo "rocprof $w failed"; tail -20 gpurun_out/final/prof/bench_$w.log; exit 3; }
done
if [ "${DEFAULT:-0}" = "1" ]; then  # the driver's own command: no flags
  timeout -k 10 300 python -u bench.py > gpurun_out/final/bench_default.log 2>&1 || { echo "bench default failed"; exit 4; }
  grep '^{' gpurun_out/final/bench_default.log | cut -c1-160
fi
echo done
