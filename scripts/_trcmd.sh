set -e
timeout -k 10 120 python scripts/trace_pass.py 25000000 100 0.05 1000 -1 >> gpurun_out/tr.log 2>&1
timeout -k 10 120 python scripts/trace_pass.py 25000000 100 0.05 1000 0 >> gpurun_out/tr.log 2>&1
