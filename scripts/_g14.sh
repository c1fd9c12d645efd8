# GPU box: locate the g13 failure -- join tests alone, then the point-polygon tests alone.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g14
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "join" \
    > gpurun_out/g14/pytest_join.log 2>&1; echo "join rc=$?"; tail -3 gpurun_out/g14/pytest_join.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppoly_ext.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "ppoly or polygon" \
    > gpurun_out/g14/pytest_ppoly.log 2>&1; echo "ppoly rc=$?"; grep -c PASSED gpurun_out/g14/pytest_ppoly.log; tail -3 gpurun_out/g14/pytest_ppoly.log
