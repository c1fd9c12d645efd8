# GPU box: join item planning folded into jb_scan / jb_segs -- join parity, then the join line of
# the product against the previous commit (head) and two pair-stage variants of the product
# (stage 320 per wave: 31 KB LDS, 5 blocks per CU, 1280 blocks; stage 384, 1280 blocks).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g20
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_ppoly_ext.py tests/test_gpu_multirank.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "join or c3" > gpurun_out/g20/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g20/pytest.log; exit 1; }
tail -1 gpurun_out/g20/pytest.log
CASES="product head s320b1280 s384b1280" WL=join STEPS=20 bash scripts/_lib_ab.sh
