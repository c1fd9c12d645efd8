#!/bin/bash
# GPU box: HBM PMC passes (FETCH_SIZE / WRITE_SIZE, one rocprofv3 run each) of every bench workload,
# then the FP64 flop pass of the point-polygon ones; summarised by scripts/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for w in ${WORKLOADS:-knn range c5 join ppoly ingest ppjoin ppknn knn_incr ppoly_incr}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc -o ${w}_$c -- \
        python3 bench.py --workload "$w" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line \
        > gpurun_out/pmc/${w}_$c.log 2>&1 || { echo "pmc $w $c failed"; tail -20 gpurun_out/pmc/${w}_$c.log; exit 4; }
    echo "pmc $w $c ok"
  done
done
for w in ${FP64_WORKLOADS-ppoly ppjoin ppknn ppoly_incr}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 --output-format csv -d gpurun_out/pmc -o ${w}_SQ_INSTS_VALU_FLOPS_FP64 -- \
      python3 bench.py --workload "$w" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line \
      > gpurun_out/pmc/${w}_fp64.log 2>&1 || { echo "pmc fp64 $w failed"; tail -20 gpurun_out/pmc/${w}_fp64.log; exit 5; }
  echo "pmc $w fp64 ok"
done
echo done
