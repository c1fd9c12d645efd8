# GPU box: join with load-free emission + one-block scans -- parity, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g7
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_multirank.py tests/test_gpu_threads.py \
    -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "join" > gpurun_out/g7/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -30 gpurun_out/g7/pytest.log; exit 1; }
tail -1 gpurun_out/g7/pytest.log
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
timeout -k 10 300 python -u bench.py --workload join --steps 30 --warmup 3 $B > gpurun_out/g7/bench_join.log 2>&1 || { tail -20 gpurun_out/g7/bench_join.log; exit 2; }
grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/g7/bench_join.log | tr '\n' ' '; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g7/prof -o join -- \
    python3 bench.py --workload join --steps 20 --warmup 3 $B > gpurun_out/g7/prof_join.log 2>&1 || { tail -5 gpurun_out/g7/prof_join.log; exit 4; }
python3 scripts/kstats.py gpurun_out/g7/prof/join_kernel_stats.csv > gpurun_out/g7/ks.txt; head -16 gpurun_out/g7/ks.txt
WL=join KERNELS="jb_tiles jb_bands join_fused<false, true>" timeout -k 10 400 bash scripts/_pmc_sq.sh > gpurun_out/g7/pmc_sq.txt 2>&1 || { tail -5 gpurun_out/g7/pmc_sq.txt; exit 5; }
cat gpurun_out/g7/pmc_sq.txt
