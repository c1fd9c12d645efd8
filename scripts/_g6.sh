# GPU box: pair-store microbenchmark; join parity after the jb_scan change; join kernel stats for
# the product and the no-store measurement build.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g6
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro/store_micro > gpurun_out/g6/store_micro.log 2>&1 || { tail -5 gpurun_out/g6/store_micro.log; exit 1; }
cat gpurun_out/g6/store_micro.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py -m gpu -x -q -p no:cacheprovider \
    --timeout 240 --timeout-method thread -k "join" > gpurun_out/g6/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g6/pytest.log; exit 2; }
tail -1 gpurun_out/g6/pytest.log
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
for lib in product jnostore; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g6/prof_$lib -o join -- \
      python3 bench.py --workload join --steps 20 --warmup 3 $B > gpurun_out/g6/prof_$lib.log 2>&1 || { tail -5 gpurun_out/g6/prof_$lib.log; exit 3; }
  echo "== $lib"; python3 scripts/kstats.py gpurun_out/g6/prof_$lib/join_kernel_stats.csv > gpurun_out/g6/ks_$lib.txt; head -6 gpurun_out/g6/ks_$lib.txt
done
