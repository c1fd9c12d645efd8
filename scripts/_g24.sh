# GPU box, end of round 4 (second pass): the whole GPU suite on the final tree, then the join's
# bench line, kernel stats and PMC passes again (the join changed after the first final pass).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/final/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
TESTS=0 WORKLOADS="join" bash scripts/final_round.sh && WORKLOADS="join" FP64_WORKLOADS="" bash scripts/final_pmc.sh
