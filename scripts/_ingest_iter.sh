# GPU box: ingest parity tests, then the ingest bench line with kernel stats
set -e
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_ingest.log 2>&1 || { tail -30 gpurun_out/pytest_ingest.log; exit 1; }
tail -1 gpurun_out/pytest_ingest.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o ingest -- python3 bench.py --workload ingest --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/prof/ingest.log 2>&1
grep '^{' gpurun_out/prof/ingest.log | cut -c1-200
python3 scripts/kstats.py gpurun_out/prof/ingest_kernel_stats.csv 2>/dev/null | head -4 || true
