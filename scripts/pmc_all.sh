#!/bin/bash
# rocprofv3 PMC passes over bench.py workloads, one counter per pass (FETCH_SIZE, WRITE_SIZE and,
# for the FP64-bound point-polygon steps, SQ_INSTS_VALU_FLOPS_FP64), no tracing domains combined
# with --pmc.  Output: gpurun_out/pmc/<workload>_<counter>_counter_collection.csv, summarised by
# scripts/pmc_summary.py into profiles/pmc_<tag>.json.   WLS="knn join ..." to choose.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for w in ${WLS:-knn c5 range join ppoly ppjoin ppknn ingest}; do
  passes="FETCH_SIZE WRITE_SIZE"
  case $w in ppoly|ppjoin|ppknn) passes="$passes SQ_INSTS_VALU_FLOPS_FP64";; esac
  for c in $passes; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc -o ${w}_$c -- \
        python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-pipelined > gpurun_out/pmc/${w}_$c.log 2>&1 \
        || { echo "pass $w $c failed"; exit 1; }
    echo "$w $c ok"
  done
done
python3 scripts/pmc_summary.py gpurun_out/pmc r02
