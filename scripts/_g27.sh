# GPU box: the final tree -- smoke(), the whole GPU suite, the C4 and C3 bench lines.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g27
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/g27/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/g27/smoke.log; exit 1; }
tail -1 gpurun_out/g27/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/g27/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g27/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/g27/pytest_gpu.log
for w in ppoly join; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/g27/bench_$w.log 2>&1 || { tail -20 gpurun_out/g27/bench_$w.log; exit 2; }
  grep '^{' gpurun_out/g27/bench_$w.log | cut -c1-200
done
