# GPU box: C4 ppoly_eval time per ablation build (measurement only; wrong results by design)
set -e
mkdir -p gpurun_out/ppabl
export TMPDIR=/tmp
for a in ${ABLS:-0 1 2 3}; do
  lib=spatialflink_amd/libgeohip.so; [ $a = 0 ] || lib=scripts/abl/libgeohip_abl$a.so
  GEOHIP_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ppabl -o a$a -- python3 scripts/ppoly_pmc.py > gpurun_out/ppabl/a$a.log 2>&1
  echo "abl $a"; python3 scripts/kstats.py gpurun_out/ppabl/a${a}_kernel_stats.csv | grep ppoly_eval
done
