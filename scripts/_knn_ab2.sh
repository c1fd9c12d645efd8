# GPU box: C2 A/B round 2 -- parity of the variants, per-XCC traces, then alternating bench lines
# (product = slot-only final; env GEOHIP_KNN_GROUPS=1: one arrival counter; tailNN: tail pools).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab2
export TMPDIR=/tmp
for lib in product tail10 tail20; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_incremental.py -m gpu -x -q \
      -p no:cacheprovider --timeout 200 --timeout-method thread -k "knn" > gpurun_out/ab2/pytest_$lib.log 2>&1 \
      || { echo "pytest $lib failed"; tail -20 gpurun_out/ab2/pytest_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab2/pytest_$lib.log)"
done
for lib in product tail20; do
  so=spatialflink_amd/libgeohip.so; [ "$lib" != product ] && so=spatialflink_amd/libgeohip_$lib.so
  GEOHIP_LIB=$so timeout -k 10 120 python -u scripts/trace_xcd.py > gpurun_out/ab2/trace_$lib.log 2>&1 || { tail -5 gpurun_out/ab2/trace_$lib.log; exit 2; }
  grep -v amdgpu.ids gpurun_out/ab2/trace_$lib.log
done
CASES="product product:GEOHIP_KNN_GROUPS=1 tail10 tail20 tail20:GEOHIP_KNN_GROUPS=1" WL=knn STEPS=100 bash scripts/_lib_ab.sh
mkdir -p gpurun_out/ab2/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab2/prof -o ppoly -- \
    python3 bench.py --workload ppoly --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line \
    > gpurun_out/ab2/prof/bench_ppoly.log 2>&1 || { tail -5 gpurun_out/ab2/prof/bench_ppoly.log; exit 3; }
python3 scripts/kstats.py gpurun_out/ab2/prof/ppoly_kernel_stats.csv | head -8
