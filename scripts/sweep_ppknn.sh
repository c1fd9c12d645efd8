#!/bin/bash
# ppknn scan launch-shape sweep (GEOHIP_PPKNN_BLOCKS), kernel stats per setting
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for b in 256 512 1024 4096 8192; do
  GEOHIP_PPKNN_BLOCKS=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sweep -o b$b -- \
    python3 bench.py --workload ppknn --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/sweep/b$b.log 2>&1 || exit 1
done
echo done
