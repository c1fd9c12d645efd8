set -e
timeout -k 10 120 python scripts/trace_pass.py 10000000 50 0.5 100 >> gpurun_out/tr.log 2>&1
timeout -k 10 120 python scripts/trace_pass.py 25000000 100 0.05 1000 >> gpurun_out/tr.log 2>&1
timeout -k 10 200 python scripts/ab_knn.py > gpurun_out/ab.log 2>&1
timeout -k 10 200 python scripts/ab_knn.py 25000000 100 0.05 1000 >> gpurun_out/ab.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "knn or c2 or c5" > gpurun_out/pytest_knn.log 2>&1
tail -2 gpurun_out/pytest_knn.log
