# GPU box: C2 front-rotation experiment -- kNN parity under each library build, the per-XCC phase
# trace, then an alternating same-box A/B of the C2 line.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/rot
export TMPDIR=/tmp
for lib in ${LIBS:-product rot1 rot8}; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q \
      -p no:cacheprovider --timeout 200 --timeout-method thread -k "knn and not c5 and not ppoly" > gpurun_out/rot/pytest_$lib.log 2>&1 \
      || { echo "pytest $lib failed"; tail -20 gpurun_out/rot/pytest_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/rot/pytest_$lib.log)"
  GEOHIP_LIB=$so timeout -k 10 120 python -u scripts/trace_xcd.py > gpurun_out/rot/trace_$lib.log 2>&1 || { tail -5 gpurun_out/rot/trace_$lib.log; exit 2; }
  cat gpurun_out/rot/trace_$lib.log | grep -v amdgpu.ids
done
timeout -k 10 120 python -u scripts/trace_pass.py > gpurun_out/rot/trace_pass.log 2>&1 || { tail -5 gpurun_out/rot/trace_pass.log; exit 3; }
CASES="${LIBS:-product rot1 rot8}" WL=knn STEPS=100 bash scripts/_lib_ab.sh
