#!/bin/bash
# tests + ablation + bench + rocprof kernel trace (each GPU step time-limited; stop on failure)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python scripts/ablate_knn.py > gpurun_out/ablate.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 50 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o knn -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit 4
echo done
