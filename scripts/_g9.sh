# GPU box: join two-role write pass + binning rounds; point-polygon compact heads -- parity of the
# join / point-polygon / band-pack tests, bench lines, kernel stats; ppoly A/B at 3 waves per SIMD.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/g9
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullscale.py tests/test_gpu_multirank.py tests/test_gpu_threads.py \
    tests/test_gpu_band_pack.py tests/test_gpu_holes.py tests/test_gpu_incremental.py tests/test_gpu_discriminators.py \
    -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "join or band_pack or knn_range_cells or ppoly or polygon or c4 or hole or disc" \
    > gpurun_out/g9/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/g9/pytest.log; exit 1; }
tail -1 gpurun_out/g9/pytest.log
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line"
for wl in join ppoly ppjoin; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 30 --warmup 3 $B > gpurun_out/g9/bench_$wl.log 2>&1 || { tail -20 gpurun_out/g9/bench_$wl.log; exit 2; }
  echo "$wl $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/g9/bench_$wl.log | tr '\n' ' ')"
done
for wl in join ppoly; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g9/prof -o $wl -- \
      python3 bench.py --workload $wl --steps 12 --warmup 2 $B > gpurun_out/g9/prof_$wl.log 2>&1 || { tail -5 gpurun_out/g9/prof_$wl.log; exit 3; }
  python3 scripts/kstats.py gpurun_out/g9/prof/${wl}_kernel_stats.csv > gpurun_out/g9/ks_$wl.txt; head -12 gpurun_out/g9/ks_$wl.txt
done
CASES="product wpe3" WL=ppoly STEPS=30 bash scripts/_lib_ab.sh
