# GPU box: jb_tiles with its record loads issued together -- join parity (golden, random, C3 full
# scale), then rocprofv3 kernel stats of the join step (product) and of the binning alone (jb4).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g16
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_ppoly_ext.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "join or c3" > gpurun_out/g16/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g16/pytest.log; exit 1; }
tail -1 gpurun_out/g16/pytest.log
CASES="product jb4" WL=join STEPS=10 TOP=7 bash scripts/_lib_prof.sh
