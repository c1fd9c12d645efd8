# GPU box: phase trace of the C2 kNN pass (16 timestamps per block)
set -e
mkdir -p gpurun_out
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 ${ABL:-0} > gpurun_out/tr_c2.log 2>&1
