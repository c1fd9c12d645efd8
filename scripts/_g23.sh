# GPU box: level-2 binning rounds of 4096 records (2 blocks per CU) -- join parity on that build,
# then the join line of the product and both grids.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g23
export TMPDIR=/tmp
GEOHIP_LIB=$PWD/spatialflink_amd/libgeohip_r4096b512.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "join or c3" > gpurun_out/g23/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g23/pytest.log; exit 1; }
tail -1 gpurun_out/g23/pytest.log
CASES="product r4096b512 r4096b1024" WL=join STEPS=20 bash scripts/_lib_ab.sh
