# GPU box: a -k subset of the GPU suite, then optional bench lines (BENCHES="knn_incr ppknn ...")
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TMO:-600} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "${K}" > gpurun_out/sub_tests.log 2>&1 || { tail -40 gpurun_out/sub_tests.log; exit 1; }
tail -2 gpurun_out/sub_tests.log
for wl in ${BENCHES:-}; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-cells-line --no-e2e --no-pipelined > gpurun_out/b_$wl.log 2>&1 || { tail -20 gpurun_out/b_$wl.log; exit 2; }
  echo "$wl $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*' gpurun_out/b_$wl.log | tr '\n' ' ')"
done
