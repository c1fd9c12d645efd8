# GPU box: unconditional gathers (point-polygon heads / entries, binning prefetch) and jb_tiles
# loads together -- parity (point-polygon, join), then product vs the previous commit's source.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g17
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ppoly_ext.py tests/test_gpu_parity.py tests/test_gpu_holes.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "ppoly or polygon or hole or join or c3 or c4" > gpurun_out/g17/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g17/pytest.log; exit 1; }
tail -1 gpurun_out/g17/pytest.log
CASES="product head" WL=ppoly STEPS=40 bash scripts/_lib_ab.sh
CASES="product head" WL=join STEPS=20 bash scripts/_lib_ab.sh
