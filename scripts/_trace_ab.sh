# GPU box: C2 phase traces, product pass vs ablation ${ABL}
set -e
mkdir -p gpurun_out
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 0 > gpurun_out/tr_c2.log 2>&1
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 ${ABL} >> gpurun_out/tr_c2.log 2>&1
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 0 >> gpurun_out/tr_c2.log 2>&1
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 ${ABL} >> gpurun_out/tr_c2.log 2>&1
