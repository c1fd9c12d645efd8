# GPU box: functional rehearsal of bench.py's N > 1 path (two ranks on the one GPU, gloo,
# host-staged collectives) for the kNN and C5 workloads, then the N = 1 lines.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp GEOHIP_BENCH_ONE_DEVICE=1 GEOHIP_BENCH_BACKEND=gloo
for WL in knn c5 range; do
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 20 --warmup 3 --workload $WL --no-cpu-baseline --check > gpurun_out/bench_w2_$WL.log 2>&1 || { tail -30 gpurun_out/bench_w2_$WL.log; exit 1; }
grep '^{' gpurun_out/bench_w2_$WL.log | cut -c1-300
done
unset GEOHIP_BENCH_ONE_DEVICE GEOHIP_BENCH_BACKEND
for WL in knn c5; do
timeout -k 10 240 python -u bench.py --workload $WL --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-pipelined > gpurun_out/bench_$WL.log 2>&1
grep '^{' gpurun_out/bench_$WL.log | cut -c1-300
done
