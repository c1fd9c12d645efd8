# GPU box: join write pass with 768-pair stages (3 blocks per CU) -- join parity, then the join line.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g22
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_ppoly_ext.py tests/test_gpu_multirank.py tests/test_gpu_band_pack.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "join or c3 or band" > gpurun_out/g22/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g22/pytest.log; exit 1; }
tail -1 gpurun_out/g22/pytest.log
CASES="product" WL=join STEPS=20 bash scripts/_lib_ab.sh
