# GPU box: join binning rounds + up-front single-block scans -- parity, bench, kernel stats; emission
# ablations (no stores / no ALL pairs / no PART pairs) by join_fused kernel time.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g8
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_multirank.py tests/test_gpu_threads.py tests/test_gpu_band_pack.py \
    -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "join or band_pack or knn_range_cells" > gpurun_out/g8/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -30 gpurun_out/g8/pytest.log; exit 1; }
tail -1 gpurun_out/g8/pytest.log
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
timeout -k 10 300 python -u bench.py --workload join --steps 30 --warmup 3 $B > gpurun_out/g8/bench_join.log 2>&1 || { tail -20 gpurun_out/g8/bench_join.log; exit 2; }
grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/g8/bench_join.log | tr '\n' ' '; echo
for lib in product; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g8/prof_$lib -o join -- \
      python3 bench.py --workload join --steps 12 --warmup 2 $B > gpurun_out/g8/prof_$lib.log 2>&1 || { tail -5 gpurun_out/g8/prof_$lib.log; exit 3; }
  python3 scripts/kstats.py gpurun_out/g8/prof_$lib/join_kernel_stats.csv > gpurun_out/g8/ks_$lib.txt
  echo "== $lib"; if [ $lib = product ]; then head -16 gpurun_out/g8/ks_$lib.txt; else head -3 gpurun_out/g8/ks_$lib.txt; fi
done
