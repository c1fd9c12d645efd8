#!/bin/bash
# One GPU box session: parity tests, every bench workload, rocprofv3 kernel stats of each bench
# command, HBM PMC passes (FETCH_SIZE / WRITE_SIZE, one per pass) of each.  Every GPU step has its
# own time limit; the script stops at the first failing GPU step.
#   WORKLOADS="knn range" PMC=0 TESTS=0 scripts/gpu_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof gpurun_out/pmc
export TMPDIR=/tmp
WORKLOADS=${WORKLOADS:-knn range join ppoly c5 ingest}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
for w in $WORKLOADS; do
  steps=50; [ "$w" = "join" ] || [ "$w" = "ppoly" ] && steps=10
  timeout -k 10 300 python -u bench.py --workload "$w" --steps $steps --warmup 3 ${BENCH_ARGS:-} \
      > gpurun_out/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 gpurun_out/bench_$w.log; exit 2; }
  grep '^{' gpurun_out/bench_$w.log
  if [ "${PROF:-1}" = "1" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $w -- \
        python3 bench.py --workload "$w" --steps $steps --warmup 3 --no-cpu-baseline --no-e2e --no-pipelined ${BENCH_ARGS:-} \
        > gpurun_out/prof/bench_$w.log 2>&1 || { echo "rocprof $w failed"; tail -20 gpurun_out/prof/bench_$w.log; exit 3; }
  fi
  if [ "${PMC:-1}" = "1" ]; then
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc -o ${w}_$c -- \
          python3 bench.py --workload "$w" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-pipelined ${BENCH_ARGS:-} \
          > gpurun_out/pmc/${w}_$c.log 2>&1 || { echo "pmc $w $c failed"; tail -20 gpurun_out/pmc/${w}_$c.log; exit 4; }
    done
  fi
done
echo done
