#!/bin/bash
# One GPU-box session for a change under test: a parity subset, then bench lines (and optionally
# rocprofv3 kernel stats) of one or more workloads under one or more library builds / env
# settings, alternating so that every case sees the same box.  Each GPU step runs under its own
# time limit; the script stops at the first failing step.
#
#   OUT=gpurun_out/t1 TESTS="join or ppoly" WL="join ppoly" CASES="product v2 product:GEOHIP_X=1" \
#       REPS=2 PROF=1 bash scripts/gpu_ab.sh
#
#   TESTS      pytest -k expression over the -m gpu suite ("" = no tests, "all" = the whole suite)
#   TEST_FILES test files (default: tests)
#   WL         bench workloads ("" = none)
#   CASES      "product" = spatialflink_amd/libgeohip.so; "<name>" = libgeohip_<name>.so (a
#              measurement build, scripts/build_variant.sh); ":K=V ..." appends env settings
#   REPS       bench repetitions per case (alternating), STEPS bench steps (default 30 / 10 with PROF)
#   PROF       1 = a rocprofv3 --kernel-trace --stats run per (workload, case), top kernels printed
#   BENCH_ARGS extra bench.py arguments
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=${TESTS:-}
if [ -n "$TESTS" ]; then
  K=(-k "$TESTS"); [ "$TESTS" = "all" ] && K=()
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest ${TEST_FILES:-tests} -m gpu -x -q -p no:cacheprovider \
      --timeout ${TEST_TIMEOUT:-240} --timeout-method thread "${K[@]}" > "$OUT/pytest.log" 2>&1 \
      || { echo "pytest failed"; tail -40 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
B="--no-cpu-baseline --no-e2e --no-pipelined --no-cells-line ${BENCH_ARGS:-}"
lib_of() { local lib=${1%%:*}; if [ "$lib" = product ]; then echo "$PWD/spatialflink_amd/libgeohip.so"; else echo "$PWD/spatialflink_amd/libgeohip_$lib.so"; fi; }
envs_of() { local c=$1 lib=${1%%:*}; [ "$c" != "$lib" ] && echo "${c#*:}"; }
for wl in ${WL:-}; do
  for r in $(seq 1 ${REPS:-1}); do
    for c in ${CASES:-product}; do
      tag=$(echo "${wl}_${c}_$r" | tr -c 'a-zA-Z0-9_\n' '_')
      env GEOHIP_LIB=$(lib_of "$c") $(envs_of "$c") timeout -k 10 300 python -u bench.py --workload $wl \
          --steps ${STEPS:-30} --warmup 3 $B > "$OUT/bench_$tag.log" 2>&1 || { echo "bench $tag failed"; tail -20 "$OUT/bench_$tag.log"; exit 2; }
      echo "$wl $c #$r $(grep -o '"ms_per_step": [0-9.]*\|"avg_kernel_us": [0-9.]*\|"frac": [0-9.]*' "$OUT/bench_$tag.log" | tr '\n' ' ')"
    done
  done
  if [ "${PROF:-0}" = "1" ]; then
    for c in ${CASES:-product}; do
      tag=$(echo "${wl}_${c}" | tr -c 'a-zA-Z0-9_\n' '_')
      env GEOHIP_LIB=$(lib_of "$c") $(envs_of "$c") timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/prof" -o "$tag" -- python3 bench.py --workload $wl --steps ${PROF_STEPS:-10} --warmup 3 $B \
          > "$OUT/prof_$tag.log" 2>&1 || { echo "rocprof $tag failed"; tail -20 "$OUT/prof_$tag.log"; exit 3; }
      echo "== $wl $c"
      python3 scripts/kstats.py "$OUT/prof/${tag}_kernel_stats.csv" | sed -n 2,${TOP:-8}p
    done
  fi
done
echo done
