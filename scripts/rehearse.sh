#!/bin/bash
# GPU box (one GPU): the N > 1 bench paths rehearsed with W ranks on cuda:0 over gloo (host-staged
# collectives; functional, not a measurement), plus the N = 1 lines of the partitioned workloads.
# Usage: WORLDS="4 8" WORKLOADS="knn c5 join" bash scripts/rehearse.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rehearse
export TMPDIR=/tmp
port=29611
for wl in ${WORKLOADS:-knn c5 join}; do
  for w in ${WORLDS:-4 8}; do
    for part in ${PARTS:-arrival}; do
      log=gpurun_out/rehearse/w${w}_${wl}_${part}.log
      GEOHIP_BENCH_ONE_DEVICE=1 GEOHIP_BENCH_BACKEND=gloo timeout -k 10 ${TMO:-420} \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port $port \
        bench.py --gpus $w --workload $wl --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --check \
        --partition $part --cells-steps 3 > $log 2>&1 || { echo "FAILED $log"; tail -30 $log; exit 1; }
      grep '^{' $log > gpurun_out/rehearse/w${w}_${wl}_${part}.json
      echo "ok $log"
      port=$((port + 1))
    done
  done
done
echo done
