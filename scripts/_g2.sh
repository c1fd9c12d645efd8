set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest_traj.py tests/test_gpu_ingest.py tests/test_gpu_format.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/g2/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/g2/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --workload ingest --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/g2/bench_ingest.log 2>&1 || exit 2
grep '^{' gpurun_out/g2/bench_ingest.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['avg_kernel_us'], d['roofline']['frac'])"
