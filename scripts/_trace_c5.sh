# GPU box: phase trace of the C5 fused kNN + range pass
set -e
mkdir -p gpurun_out
timeout -k 10 120 python scripts/trace_pass.py 25000000 100 0.05 1000 -1 > gpurun_out/tr_c5.log 2>&1
