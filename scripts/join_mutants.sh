#!/bin/bash
# Which join tests see an emission fault that keeps every per-point decision (and so the pair
# count) and changes only pair identities -- the round-4 g8 symptom (full-scale C3: right count,
# wrong digest, every smaller join test green).  Builds two mutants of cell_kernels.hip (CPU side):
#   allpid  the full-chunk ALL run (jemit_chunk's direct 512-B stores) emits the first query of
#           each group of four with window index pid ^ 1 instead of pid
#   allq    the same run pairs its second query of each group of four with the first query's id
#   scripts/join_mutants.sh build      (here)
#   scripts/join_mutants.sh run        (GPU box: each mutant under the small and the mid-size tests)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SRC=spatialflink_amd/csrc/cell_kernels.hip
if [ "${1:-}" = build ]; then
  mkdir -p build/mut
  sed 's/if (p < a.cap) jpair_store(a, p, pid, q4.x);/if (p < a.cap) jpair_store(a, p, pid ^ 1u, q4.x);/' $SRC > build/mut/allpid.hip
  sed 's/if (p + kWave < a.cap) jpair_store(a, p + kWave, pid, q4.y);/if (p + kWave < a.cap) jpair_store(a, p + kWave, pid, q4.x);/' $SRC > build/mut/allq.hip
  for m in allpid allq; do
    cmp -s $SRC build/mut/$m.hip && { echo "mutant $m: pattern not found"; exit 1; }
    cp build/mut/$m.hip spatialflink_amd/csrc/_mut_$m.hip
    VARIANT_SRC=spatialflink_amd/csrc/_mut_$m.hip bash scripts/build_variant.sh mut_$m cell_kernels.hip
    rm -f spatialflink_amd/csrc/_mut_$m.hip
  done
  exit 0
fi
OUT=${OUT:-gpurun_out/mut}
mkdir -p $OUT
export TMPDIR=/tmp
SMALL="tests/test_gpu_parity.py"
for m in allpid allq; do
  for t in small mid; do
    if [ $t = small ]; then files=$SMALL; k="join"; else files=tests/test_gpu_join_mid.py; k="exact"; fi
    GEOHIP_LIB=$PWD/spatialflink_amd/libgeohip_mut_$m.so timeout -k 10 400 python -u -m pytest $files -m gpu -q \
        -p no:cacheprovider --timeout 240 --timeout-method thread -k "$k" > $OUT/${m}_$t.log 2>&1
    rc=$?
    [ $rc -ge 124 ] && { echo "$m $t: time limit or crash ($rc)"; tail -5 $OUT/${m}_$t.log; exit 1; }
    echo "$m $t: $(tail -1 $OUT/${m}_$t.log)"
  done
done
