# GPU box: point-polygon kNN / pane-merge kernels timed by their dispatch stamps -- their parity
# tests, the PMC passes of every workload, then the ppknn and knn_incr lines and kernel stats again.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g18
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppoly_ext.py tests/test_gpu_incremental.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "knn" > gpurun_out/g18/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g18/pytest.log; exit 1; }
tail -1 gpurun_out/g18/pytest.log
bash scripts/final_pmc.sh && TESTS=0 WORKLOADS="ppknn knn_incr" bash scripts/final_round.sh
