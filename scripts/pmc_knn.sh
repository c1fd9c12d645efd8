#!/bin/bash
# rocprofv3 PMC passes over the headline bench (one counter group per pass; no tracing
# domains combined with --pmc).  Output: gpurun_out/pmc/<pass>_counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $counters --output-format csv -d gpurun_out/pmc -o p$i -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FLOPS_FP64 SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU
FETCH_SIZE
WRITE_SIZE
TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_RDREQ_128B
LIST
echo done
