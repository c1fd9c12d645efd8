# GPU box: SQ / TCC counter passes (one rocprofv3 --pmc run each) of one bench workload; per-kernel
# averages of the named kernels.  WL=ppoly KERNELS="ppoly_stream ppoly_cand_eval" bash scripts/_pmc_sq.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcsq
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
P2="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2" ${EXTRA_PASSES:-}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmcsq -o ${WL}_p$i -- python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line > gpurun_out/pmcsq/${WL}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcsq/${WL}_p$i.log; exit 1; }
done
python3 - "$WL" $KERNELS <<'PY'
import csv, sys, glob
from collections import defaultdict
wl, ks = sys.argv[1], sys.argv[2:]
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"gpurun_out/pmcsq/{wl}_p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        for k in ks:
            if k in name:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in ks:
    print("==", k)
    for c, v in sorted(acc[k].items()):
        print(f"  {c:24s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
