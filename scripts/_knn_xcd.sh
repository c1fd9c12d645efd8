# GPU box: kNN parity subset, then an alternating same-box A/B of the C2 line (kernel stats each)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_incremental.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "knn or c2 or c5" > gpurun_out/pytest_knn.log 2>&1 || { tail -30 gpurun_out/pytest_knn.log; exit 1; }
tail -1 gpurun_out/pytest_knn.log
CASES="product noxcd product noxcd product noxcd" WL=knn STEPS=100 TOP=2 bash scripts/_lib_prof.sh
