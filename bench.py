"""Headline benchmark: windowed point-point kNN (BASELINE.json configs[1]).

One step = one window: kNN (k = 50) of the README query point over 10M uniform points per
GPU (100x100 Beijing grid, r = 0.5) -- the scan kernel, the final selection and, for N > 1,
the RCCL all-gather of each rank's top-k plus the device merge (weak scaling: every rank
holds its own 10M-point shard of the window; ranks shard by arrival order, which gives the
identical result for a single-query kNN).

Windows are device-resident before the timed region (synthetic, generated on the device with
the counter-based generator of spatialflink_amd.synth); a ring of WINDOWS distinct windows
(> 256 MiB in total) is cycled so no step reads a window the Infinity Cache still holds.

Prints ONE JSON line (rank 0) with roofline and cpu_baseline objects.

    python bench.py --gpus 1 --steps 50 --warmup 5
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "points/sec (whole node) for windowed range/kNN/join at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
N_PER_GPU = 10_000_000
GRID_N = 100
K = 50
RADIUS = 0.5
WINDOWS = 4
BYTES_PER_POINT = 16  # algorithmic: x + y fp64 read once


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--points", type=int, default=N_PER_GPU)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--knn-final", choices=("fused", "separate"), default="fused",
                   help="final selection in the scan's last block, or a separate knn_final launch")
    return p.parse_args()


def cpu_baseline(seconds: float):
    """The C oracle (oracle/geohip_oracle.c, a single-threaded port of the reference
    predicate + heap kNN) on the same workload, bounded to ~`seconds` of CPU work."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import cref
    from spatialflink_amd import synth

    bj = synth.BEIJING
    q = synth.README_QUERY
    cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / GRID_N, GRID_N)
    n = 2_000_000
    done = 0
    wins = 0
    t_total = 0.0
    while t_total < seconds and wins < 30:
        x, y = synth.uniform(n, 1000 + wins)
        t0 = time.perf_counter()
        cref.knn_pp(cg, x, y, q[0], q[1], RADIUS, K)
        t_total += time.perf_counter() - t0
        done += n
        wins += 1
    return {"value": done / t_total, "unit": "points/sec", "cores": 1, "kind": "port",
            "sample": f"{wins} windows x {n} uniform points (C2 shape: k={K}, {GRID_N}x{GRID_N}, r={RADIUS}), "
                      f"oracle/geohip_oracle.c single thread, {t_total:.1f} s"}


def pmc_traffic():
    """HBM bytes per scan launch from the committed rocprofv3 PMC pass, if present."""
    f = ROOT / "profiles" / "pmc_knn_scan_r01.json"
    if f.exists():
        try:
            return json.loads(f.read_text()).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    from spatialflink_amd import Context, _abi, synth

    dev = torch.device("cuda", local)
    ctx = Context(local)
    _abi.debug_set_knn_fused(args.knn_final == "fused")
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)  # kernels and RCCL ordered on one stream
    bj = synth.BEIJING
    q = synth.README_QUERY
    grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / GRID_N, GRID_N)
    n = args.points

    xs, ys = [], []
    for w in range(WINDOWS):
        x = torch.empty(n, dtype=torch.float64, device=dev)
        y = torch.empty(n, dtype=torch.float64, device=dev)
        # window w of rank r = slice [r*n, (r+1)*n) of the N*n-point window w
        ctx.synth_uniform_async(x, y, rank * n, 2 + 7919 * w, bj)
        xs.append(x)
        ys.append(y)
    out_i = torch.empty(K, dtype=torch.int32, device=dev)
    out_d = torch.empty(K, dtype=torch.float64, device=dev)
    cnt = torch.zeros(2, dtype=torch.int32, device=dev)
    g_d = torch.empty((world, K), dtype=torch.float64, device=dev)
    g_i = torch.empty((world, K), dtype=torch.int32, device=dev)
    m_i = torch.empty(K, dtype=torch.int32, device=dev)
    m_d = torch.empty(K, dtype=torch.float64, device=dev)
    base = torch.tensor(rank * n, dtype=torch.int64, device=dev)

    def step(s):
        w = s % WINDOWS
        ctx.knn_pp_async(grid, xs[w], ys[w], q[0], q[1], RADIUS, K, out_i, out_d, cnt[0:1])
        if world > 1:
            gi = torch.where(out_i >= 0, (out_i.to(torch.int64) + base).to(torch.int32), out_i)
            dist.all_gather_into_tensor(g_d.view(-1), out_d)
            dist.all_gather_into_tensor(g_i.view(-1), gi)
            ctx.knn_merge_async(g_d, g_i, world, K, K, m_i, m_d, cnt[1:2])

    torch.cuda.synchronize(dev)
    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize(dev)
    ctx.timing(reset=True)
    ctx.set_timing(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(args.warmup + s)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    scan_ms, launches = ctx.timing(reset=True)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_points = n * world * args.steps
    value = total_points / elapsed
    avg_scan_s = scan_ms / 1e3 / max(launches, 1)
    achieved = BYTES_PER_POINT * n / avg_scan_s / 1e9
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "points/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "C2: point-point kNN k=50, 100x100 Beijing UniformGrid, r=0.5, README query, "
                               f"{n} uniform points per window per GPU (BASELINE.json configs[1])",
                   "points_per_window_per_gpu": n, "grid": GRID_N, "k": K, "radius": RADIUS,
                   "windows_resident": WINDOWS, "final_selection": args.knn_final,
                   "parallelism": f"shard{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(),
                     "kernel": "geohip::knn_scan<1>", "avg_kernel_us": avg_scan_s * 1e6,
                     "algorithmic_bytes_per_launch": BYTES_PER_POINT * n},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
