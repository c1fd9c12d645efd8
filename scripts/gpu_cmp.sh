#!/bin/bash
# tests + ablation + bench (fused and separate final selection) + rocprof of both
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python scripts/ablate_knn.py > gpurun_out/ablate.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --knn-final fused > gpurun_out/bench_fused.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --knn-final separate > gpurun_out/bench_sep.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o sep -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --knn-final separate > gpurun_out/bench_prof_sep.log 2>&1 || exit 4
echo done
