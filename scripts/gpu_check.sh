#!/bin/bash
# One GPU box session: parity tests, bench, rocprofv3 kernel trace of the same bench command.
# Every GPU step has its own time limit; the script stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-50}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
rc=$(tail -1 gpurun_out/pytest_gpu.log | awk '{print $3}')
if [ "$rc" != "0" ] && [ "$rc" != "1" ]; then echo "pytest crashed ($rc)"; exit 1; fi
timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o knn -- \
    python3 bench.py --steps "$STEPS" --warmup 5 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit 3
echo done
