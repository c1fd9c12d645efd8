#!/bin/bash
# one iteration on the GPU box: parity tests, shape sweep, phase trace (each step time-limited)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u scripts/sweep_knn.py ${SWEEP:-4,1,32 8,1,32 16,1,16} > gpurun_out/sweep.log 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/sweep.log; exit 2; }
grep -v amdgpu.ids gpurun_out/sweep.log | grep -v '^{'
timeout -k 10 300 python -u scripts/trace_knn.py ${TRACE:-4,1,32} > gpurun_out/trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/trace.log; exit 3; }
echo done
