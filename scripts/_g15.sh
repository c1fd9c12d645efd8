# GPU box: point-polygon walk with batched entry loads -- parity subset, then the C4 line per
# build (product = batch 2; b1, b3; nt = nontemporal window loads).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g15
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppoly_ext.py tests/test_gpu_parity.py tests/test_gpu_holes.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "ppoly or polygon or hole" > gpurun_out/g15/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g15/pytest.log; exit 1; }
tail -1 gpurun_out/g15/pytest.log
CASES="${CASES:-product b1 b3 nt}" WL=ppoly STEPS=40 bash scripts/_lib_ab.sh
