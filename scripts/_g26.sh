# GPU box: ppoly_cand_eval issuing an item's slot and record loads together -- point-polygon parity,
# then the C4 line of the product and the previous commit (head).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g26
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ppoly_ext.py tests/test_gpu_parity.py tests/test_gpu_holes.py tests/test_gpu_fullscale.py tests/test_gpu_incremental.py -m gpu -x -q -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "ppoly or polygon or hole or c4" > gpurun_out/g26/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g26/pytest.log; exit 1; }
tail -1 gpurun_out/g26/pytest.log
CASES="product head" WL=ppoly STEPS=40 bash scripts/_lib_ab.sh
