# GPU box: join write pass A/B (fused staged vs two-role pipe) with parity; point-polygon parity
# after the revert; bench lines for join, ppoly, knn.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g11
export TMPDIR=/tmp
for lib in product; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider \
      --timeout 240 --timeout-method thread -k "join or ppoly or c4" > gpurun_out/g11/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -30 gpurun_out/g11/pytest_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/g11/pytest_$lib.log)"
done
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
for lib in product; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g11/prof_$lib -o join -- \
      python3 bench.py --workload join --steps 12 --warmup 2 $B > gpurun_out/g11/prof_$lib.log 2>&1 || { tail -5 gpurun_out/g11/prof_$lib.log; exit 3; }
  python3 scripts/kstats.py gpurun_out/g11/prof_$lib/join_kernel_stats.csv > gpurun_out/g11/ks_$lib.txt
  echo "== $lib"; head -3 gpurun_out/g11/ks_$lib.txt
done
for wl in join ppoly knn; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 3 $B > gpurun_out/g11/bench_$wl.log 2>&1 || { tail -20 gpurun_out/g11/bench_$wl.log; exit 2; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/g11/bench_$wl.log | tr '\n' ' ')"
done
