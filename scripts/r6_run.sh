#!/bin/bash
# GPU box, round 6: the GPU suite (or a -k subset), then bench lines of the named workloads
# (BENCH_ARGS_<wl> extra args), then rocprofv3 kernel stats of each.  Every GPU step has its own
# limit; the script stops at the first failure.
#   OUT=gpurun_out/r6a K="range_set or jni" WL="range knn" PROF=1 bash scripts/r6_run.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/r6}
mkdir -p "$OUT/prof"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  KA=(); [ -n "${K:-}" ] && KA=(-k "$K")
  # test failures (exit 1) are reported and the run goes on; anything else (a timeout, a crash,
  # an abort) ends it
  timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest tests -m gpu ${XFLAG--x} -v -p no:cacheprovider --timeout 240 \
      --timeout-method thread "${KA[@]}" > "$OUT/pytest.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pytest rc=$rc"; grep -E '^(FAILED|ERROR)' "$OUT/pytest.log" | head -20; tail -5 "$OUT/pytest.log"
    [ $rc -eq 1 ] || exit 1
  fi
  tail -1 "$OUT/pytest.log"
fi
for spec in ${WL:-}; do
  wl=${spec%%:*}; extra=""; [ "$spec" != "$wl" ] && extra="${spec#*:}"; extra=${extra//,/ }
  tag=$(echo "$spec" | tr -c 'a-zA-Z0-9_\n' '_')
  steps=${STEPS:-50}; [ "$wl" = "join" ] || [ "$wl" = "ppoly" ] || [ "$wl" = "ppjoin" ] && steps=${STEPS_BIG:-20}
  timeout -k 10 300 python -u bench.py --workload "$wl" --steps $steps --warmup 3 $extra ${BENCH_ARGS:-} \
      > "$OUT/bench_$tag.log" 2>&1 || { echo "bench $spec failed"; tail -20 "$OUT/bench_$tag.log"; exit 2; }
  echo "$spec $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*\|"counts_verified": [a-z]*' "$OUT/bench_$tag.log" | tr '\n' ' ')"
  [ "${PROF:-0}" = "1" ] || continue
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o "$tag" -- \
      python3 bench.py --workload "$wl" --steps $steps --warmup 3 $extra --no-cpu-baseline --no-e2e --no-pipelined --no-cells-line \
      > "$OUT/prof/bench_$tag.log" 2>&1 || { echo "rocprof $spec failed"; tail -20 "$OUT/prof/bench_$tag.log"; exit 3; }
  python3 scripts/kstats.py "$OUT/prof/${tag}_kernel_stats.csv" | sed -n 2,${TOP:-6}p
done
echo done
