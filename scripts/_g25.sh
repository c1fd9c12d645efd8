# GPU box: smoke(); jb_scan forming the item counts while the tile counts load -- join parity, then
# kernel stats of the product and the previous commit (head).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g25
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/g25/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/g25/smoke.log; exit 1; }
tail -1 gpurun_out/g25/smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_ppoly_ext.py tests/test_gpu_multirank.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "join or c3" > gpurun_out/g25/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g25/pytest.log; exit 1; }
tail -1 gpurun_out/g25/pytest.log
CASES="product head" WL=join STEPS=20 TOP=7 bash scripts/_lib_prof.sh
