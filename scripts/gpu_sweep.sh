#!/bin/bash
# kNN launch-shape sweep on one GPU box (each GPU step time-limited; stop on failure)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/sweep_knn.py "$@" > gpurun_out/sweep.log 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/sweep.log; exit 1; }
cat gpurun_out/sweep.log | grep -v amdgpu.ids
