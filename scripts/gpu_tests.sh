#!/bin/bash
# GPU box: the -m gpu suite (one process, per-test time limit), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 2; }
  grep '^{' gpurun_out/bench.log
fi
echo done
