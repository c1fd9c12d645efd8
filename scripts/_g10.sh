# GPU box: join write pass with direct contiguous stores (fused product vs two-role pipe vs no
# stores) -- C3 parity for both, kernel stats; SQ counters of ppoly_stream.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g10
export TMPDIR=/tmp
for lib in product jpipe; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider \
      --timeout 240 --timeout-method thread -k "join" > gpurun_out/g10/pytest_$lib.log 2>&1 || { echo "pytest $lib failed"; tail -30 gpurun_out/g10/pytest_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/g10/pytest_$lib.log)"
done
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
for lib in product jpipe jnostore; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g10/prof_$lib -o join -- \
      python3 bench.py --workload join --steps 12 --warmup 2 $B > gpurun_out/g10/prof_$lib.log 2>&1 || { tail -5 gpurun_out/g10/prof_$lib.log; exit 3; }
  python3 scripts/kstats.py gpurun_out/g10/prof_$lib/join_kernel_stats.csv > gpurun_out/g10/ks_$lib.txt
  echo "== $lib"; head -3 gpurun_out/g10/ks_$lib.txt
done
WL=ppoly KERNELS="ppoly_stream" timeout -k 10 400 bash scripts/_pmc_sq.sh > gpurun_out/g10/pmc_ppoly.txt 2>&1 || { tail -5 gpurun_out/g10/pmc_ppoly.txt; exit 5; }
cat gpurun_out/g10/pmc_ppoly.txt
