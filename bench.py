"""Benchmark: GeoFlink windowed spatial queries on MI355X (BASELINE.json).

Default workload (the headline, BASELINE.json configs[1] = C2): one step = one window of
point-point kNN (k = 50) of the README query over 10M uniform points per GPU (100x100 Beijing
grid, r = 0.5): one knn_pass launch (scan + the last block's final selection) and, for N > 1, the RCCL
all-gather of each rank's top-k plus the device merge (weak scaling: every rank holds its own
10M-point shard of the window; ranks shard by arrival order, which gives the identical result
for a single-query kNN).

The other configs are measured with ``--workload`` (same JSON contract, one line each):
  range  C1 query shape (100x100, README query, r = 0.5) over 10M uniform points per GPU
  join   C3: 10k queries x 10M Gaussian-clustered data points per GPU, 500x500, r = 0.05
  ppoly  C4: 1k polygons (50 vertices) over 50M uniform points per GPU, 500x500, r = 0.005
  c5     C5 per shard: 25M uniform points per GPU, 1000x1000, kNN k = 100 + range r = 0.05
  ingest SURVEY.md 8(f) row 1: 10M CSV records -> SoA x/y + ts + cell (device-resident text)
  ppjoin SURVEY.md 8(f) row 2: the C4 shape as a point-polygon join (1k polygons x 50M points)
  ppknn  SURVEY.md 8(f) row 2: point-polygon kNN k = 50 of one polygon over 50M points
  knn_incr SURVEY.md 8(f) row 3: C2 over 10 s / 5 s sliding windows, pane reuse (5M-point panes)
  ppoly_incr SURVEY.md 8(f) row 3: C4 over 10 s / 5 s sliding windows, pane reuse (25M-point panes)

Windows are device-resident before the timed region (synthetic: uniform windows are made on
the device by the counter-based generator of spatialflink_amd.synth; Gaussian windows on the
host by synth.gaussian_clusters then copied).  A ring of distinct windows (> 256 MiB in total)
is cycled so no step reads a window the Infinity Cache still holds.

Prints ONE JSON line (rank 0) with roofline and cpu_baseline objects.

    python bench.py --gpus 1 --steps 50 --warmup 5 [--workload knn|range|join|ppoly|c5|ingest|ppjoin|ppknn|knn_incr|ppoly_incr]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "points/sec (whole node) for windowed range/kNN/join at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# FP64 vector peak: half the FP32 vector rate of MI355X_MICROARCH.md (157.3 TFLOP/s; a wave64
# FP64 FMA issues over 4 cycles on the SIMD-32 units), 78.6 TFLOP/s
FP64_PEAK_TFLOPS = 78.6
BYTES_PER_POINT = 16  # algorithmic: x + y fp64 read once


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--workload", choices=("knn", "range", "join", "ppoly", "c5", "ingest", "ppjoin", "ppknn", "knn_incr", "ppoly_incr"), default="knn")
    p.add_argument("--points", type=int, default=None, help="points per window per GPU (default: the config's)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--range-ascending", action="store_true",
                   help="range: ascending hit order (GEOHIP_ORDER_ASCENDING, range_fused) instead of the unordered set")
    p.add_argument("--no-e2e", action="store_true", help="skip the host-resident end-to-end line")
    p.add_argument("--no-pipelined", action="store_true", help="skip the multi-stream pipelined line")
    p.add_argument("--pipeline-streams", type=int, default=3, help="contexts / HIP streams of the pipelined line")
    p.add_argument("--check", action="store_true", help="N > 1 kNN / C5: check the merged top-k against rank 0's full window")
    p.add_argument("--partition", choices=("arrival", "cells"), default="arrival",
                   help="knn / c5 / join: the timed step's layout -- arrival-order shards (default) or the north-star "
                        "grid-cell key bands (filter, keyBy(gridID) as one all-to-all, halo queries for the join)")
    p.add_argument("--no-cells-line", action="store_true", help="skip the key-band layout side line (knn / c5 / join)")
    p.add_argument("--cells-steps", type=int, default=10, help="timed steps of the key-band side line")
    p.add_argument("--time-every", type=int, default=5,
                   help="time every N-th step's kernels with their dispatch stamps (default 5, at least 4 timed "
                        "steps): a stamped dispatch costs the step ~4 us of launch (C2: 44.4 us per step with "
                        "every step stamped, 40.4 with every 5th, 40.1 with one), so stamping them all would "
                        "lower the measured rate")
    return p.parse_args()


def _oracle():
    sys.path.insert(0, str(ROOT / "oracle"))
    import cref  # the checker / CPU baseline only (test infrastructure)
    return cref


def _timed_loop(fn, seconds, max_iter):
    """Run fn(i) until ~seconds of measured time or max_iter calls; returns (calls, seconds)."""
    t_total, i = 0.0, 0
    while t_total < seconds and i < max_iter:
        t_total += fn(i)
        i += 1
    return i, t_total


def pmc_traffic(kernel_tag: str, key: str = "hbm_bytes_per_launch"):
    """Per-launch value from the committed rocprofv3 PMC passes (profiles/pmc_<tag>.json): HBM
    bytes (FETCH_SIZE x 2 + WRITE_SIZE) or FP64 FLOPs (SQ_INSTS_VALU_FLOPS_FP64)."""
    f = ROOT / "profiles" / f"pmc_{kernel_tag}.json"
    if f.exists():
        try:
            return json.loads(f.read_text()).get(key)
        except Exception:
            return None
    return None


# ----------------------------------------------------------------------------------------------
class Workload:
    """One config: device-resident windows, one step = one window through the C ABI."""
    tag = ""
    kernel = ""
    windows = 4

    def __init__(self, args, ctx, dev, rank, world, dist):
        self.args, self.ctx, self.dev, self.rank, self.world, self.dist = args, ctx, dev, rank, world, dist

    def units_per_step(self) -> int:  # points of one window on this rank
        raise NotImplementedError

    def step(self, s: int) -> None:
        raise NotImplementedError

    def algorithmic_bytes(self) -> float:  # per timed launch (ctx timing events)
        raise NotImplementedError

    def config(self) -> dict:
        raise NotImplementedError

    def cpu_baseline(self, seconds: float) -> dict:
        raise NotImplementedError

    def roofline_extra(self) -> dict:
        return {}

    def e2e(self) -> dict | None:  # host-resident window -> results on host (rank 0, N = 1)
        return None

    def cells_partition(self, steps: int) -> dict | None:  # the key-band layout side line
        return None

    def verify(self) -> bool | None:  # after the timed region: the async steps' device counts
        return None

    def _timed_side(self, fn, steps):
        """Max-over-ranks wall time of `steps` calls of fn(s) (barrier + synchronize around)."""
        import torch
        fn(0)
        torch.cuda.synchronize(self.dev)
        if self.dist:
            self.dist.barrier()
        t0 = time.perf_counter()
        out = None
        for s in range(steps):
            out = fn(s)
        torch.cuda.synchronize(self.dev)
        if self.dist:
            self.dist.barrier()
        t = time.perf_counter() - t0
        if self.dist:
            tt = torch.tensor([t], dtype=torch.float64, device=self.dev if self.dist.get_backend() == "nccl" else "cpu")
            self.dist.all_reduce(tt, op=self.dist.ReduceOp.MAX)
            t = float(tt.item())
        return t, out

    def _gather_ints(self, v):
        import torch
        if not self.dist:
            return [int(v)]
        from spatialflink_amd import distributed as D
        t = torch.tensor([int(v)], dtype=torch.int64, device=self.dev)
        allv = torch.empty(self.world, dtype=torch.int64, device=self.dev)
        D.all_gather_into(allv, t)
        return [int(a) for a in allv.cpu().tolist()]


def _uniform_windows(ctx, dev, n, rank, seeds, bbox):
    import torch
    xs, ys = [], []
    for sd in seeds:
        x = torch.empty(n, dtype=torch.float64, device=dev)
        y = torch.empty(n, dtype=torch.float64, device=dev)
        # window of rank r = slice [r*n, (r+1)*n) of the N*n-point window
        ctx.synth_uniform_async(x, y, rank * n, sd, bbox)
        xs.append(x)
        ys.append(y)
    return xs, ys


class KnnWorkload(Workload):
    """C2 (BASELINE.json configs[1]): kNN k=50, 100x100, r=0.5, 10M uniform points per GPU."""
    tag = "knn_scan"
    kernel = "geohip::knn_pass<16> (one launch per window: scan, block lists, last block's final selection)"
    grid_n, k, radius, n_default, seed0 = 100, 50, 0.5, 10_000_000, 2
    label = "C2: point-point kNN k=50, 100x100 Beijing UniformGrid, r=0.5, README query"
    has_range = False

    def __init__(self, *a):
        super().__init__(*a)
        import torch
        from spatialflink_amd import _abi, synth
        self.n = self.args.points or self.n_default
        bj = synth.BEIJING
        self.q = synth.README_QUERY
        self.grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        self.xs, self.ys = _uniform_windows(self.ctx, self.dev, self.n, self.rank,
                                            [self.seed0 + 7919 * w for w in range(self.windows)], bj)
        K, W, dev = self.k, self.world, self.dev
        # Per step, rank r's result goes out in ONE packed all-gather row: [k dist (f64 as 2k
        # int32) | k idx (int32) | range count (int64 as 2 int32, C5)]; the kNN pass writes straight
        # into views of the row.  Two rows alternate so the all-gather + merge of window i (on the
        # communication stream) overlaps the scan of window i + 1 (on the compute stream).
        self.row = 3 * K + 2 + (K & 1)
        self.pack = [torch.zeros(self.row, dtype=torch.int32, device=dev) for _ in range(2)]
        self.out_d = [p[:2 * K].view(torch.float64) for p in self.pack]
        self.out_i = [p[2 * K:3 * K] for p in self.pack]
        self.out_rc = [p[3 * K + (K & 1):].view(torch.int64) for p in self.pack]
        self.cnt = torch.zeros(2, dtype=torch.int32, device=dev)
        self.m_i = torch.empty(K, dtype=torch.int32, device=dev)
        self.m_d = torch.empty(K, dtype=torch.float64, device=dev)
        self.mcnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self.counts = torch.zeros(W, dtype=torch.int64, device=dev)
        self.host_staged = W > 1 and self.dist.get_backend() == "gloo"
        if W > 1:
            from spatialflink_amd import Context
            self.g = [torch.empty(W * self.row, dtype=torch.int32, device=dev) for _ in range(2)]
            self.offs = (torch.arange(W, dtype=torch.int32, device=dev) * self.n).view(W, 1)  # shard bases
            self.cs = torch.cuda.Stream(dev)
            self.mctx = Context(dev.index)  # merges on the communication stream
            self.ev_scan = [torch.cuda.Event() for _ in range(2)]
            self.ev_done = [None, None]

    def units_per_step(self):
        return self.n

    def scan(self, w, j):
        self.ctx.knn_pp_async(self.grid, self.xs[w], self.ys[w], self.q[0], self.q[1], self.radius, self.k,
                              self.out_i[j], self.out_d[j], self.cnt[0:1])

    def gather_merge(self, j):
        """All-gather of the ranks' packed rows, then every rank merges the W top-k lists
        (geohip_knn_merge_async; the reference's parallelism-1 windowAll funnel,
        PointPointKNNQuery.java:188-190) -- all on the communication stream."""
        import torch
        K, W = self.k, self.world
        if self.host_staged:  # gloo (functional rehearsal of the N > 1 path on one GPU): via host
            gh = torch.empty(W * self.row, dtype=torch.int32)
            self.dist.all_gather_into_tensor(gh, self.pack[j].cpu())
            self.g[j].copy_(gh)
        else:
            self.dist.all_gather_into_tensor(self.g[j], self.pack[j])
        g = self.g[j].view(W, self.row)
        gd = g[:, :2 * K].contiguous().view(torch.float64)
        gi = g[:, 2 * K:3 * K]
        gi = torch.where(gi >= 0, gi + self.offs, gi).contiguous()  # window ids; -1 sentinels stay
        self.mctx.knn_merge_async(gd, gi, W, K, K, self.m_i, self.m_d, self.mcnt)
        if self.has_range:
            self.counts.copy_(g[:, 3 * K + (K & 1):].contiguous().view(torch.int64).view(-1))

    def check_merged(self, last_step):
        """N > 1 (--check): the last step's merged top-k against the kNN of the whole
        W * n-point window evaluated on rank 0 alone (the counter-based generator makes the
        concatenated shards).  True / False on rank 0, None elsewhere."""
        import torch
        from spatialflink_amd import synth
        torch.cuda.synchronize(self.dev)
        if self.rank != 0:
            return None
        w = last_step % self.windows
        N = self.n * self.world
        x = torch.empty(N, dtype=torch.float64, device=self.dev)
        y = torch.empty(N, dtype=torch.float64, device=self.dev)
        self.ctx.synth_uniform_async(x, y, 0, self.seed0 + 7919 * w, synth.BEIJING)
        wi, wd = self.ctx.knn_pp(self.grid, x, y, self.q[0], self.q[1], self.radius, self.k)
        if self.args.partition == "cells":  # the key-band step's own merged result
            res, (_, _, total), _ = self.cells_last.result()
            m_i, m_d, m = res.idx, res.dist, int(res.count)
            if self.has_range:
                want = self.ctx.range_pp(self.grid, x, y, self.q[0], self.q[1], self.radius)
                if int(total) != len(want):
                    return False
        else:
            m_i, m_d, m = self.m_i, self.m_d, int(self.mcnt.item())
        return (m == len(wi) and m_i[:m].cpu().numpy().astype(np.uint32).tolist() ==
                wi.cpu().numpy().astype(np.uint32).tolist() and
                torch.equal(m_d[:m].cpu().view(torch.int64), wd.cpu().view(torch.int64)))

    def cells_window(self, w):
        """One window in the north-star layout: the points of this rank's shard in the query's
        G u C cells packed by key band (geohip_band_pack_query_async), one all-to-all to their
        owner, the owner's kNN (+ range) of its band, one all-gather of the top-k + merge
        (distributed.knn_range_cells)."""
        from spatialflink_amd import distributed as D

        if getattr(self, "cbufs", None) is None:  # preallocated rows: the step enqueues only
            self.cbufs = D.CellsBuffers(self.k, self.n, self.world, self.dev, with_range=self.has_range)
        return D.knn_range_cells(self.xs[w], self.ys[w], self.rank * self.n, self.q[0], self.q[1], self.radius,
                                 self.k, grid=self.grid, ctx=self.ctx, bufs=self.cbufs)

    def cells_partition(self, steps):
        """Side line: the key-band layout timed per window (max over ranks), per-rank skew of the
        points each band owner receives, and a check against the arrival-sharded result."""
        import torch
        from spatialflink_amd import distributed as D
        t, out = self._timed_side(lambda s: self.cells_window(s % self.windows), steps)
        res, (hits, _, total), nrecv = out.result()
        w = (steps - 1) % self.windows
        ref = D.knn_sharded(self.xs[w], self.ys[w], self.rank * self.n, self.q[0], self.q[1], self.radius, self.k,
                            grid=self.grid, ctx=self.ctx)
        same = (res.count == ref.count and torch.equal(res.idx.cpu(), ref.idx.cpu()) and
                torch.equal(res.dist.cpu().view(torch.int64), ref.dist.cpu().view(torch.int64)))
        if self.has_range:
            _, _, rtotal = D.range_sharded(self.xs[w], self.ys[w], self.rank * self.n, self.q[0], self.q[1],
                                           self.radius, grid=self.grid, ctx=self.ctx)
            same = same and rtotal == total
        ok = self._gather_ints(1 if same else 0)
        recv = self._gather_ints(nrecv)
        mean = sum(recv) / len(recv)
        return {"value": self.n * self.world * steps / t, "unit": "points/sec", "ms_per_step": t / steps * 1e3,
                "steps": steps, "layout": "grid-cell key bands (column cx -> rank cx*W/n): G u C filter + pack by owner "
                "(geohip_band_pack_query_async), all_to_all, owner's kNN" + (" + range" if self.has_range else "") +
                ", all_gather of top-k + geohip_knn_merge_async", "points_received_per_rank": recv,
                "skew_max_over_mean": (max(recv) / mean) if mean else None,
                "matches_arrival_sharding": all(ok)}

    def verify(self):
        """After the timed region: the last timed step's own top-k (indices and distance bits) --
        and for C5 its range hit count -- against the synchronous calls on the same window."""
        import torch
        if self.args.partition == "cells" or getattr(self, "last_s", None) is None:
            return None
        self.ctx.sync()
        s = self.last_s
        j, w = s & 1, s % self.windows
        m = int(self.cnt[0].item())
        wi, wd = self.ctx.knn_pp(self.grid, self.xs[w], self.ys[w], self.q[0], self.q[1], self.radius, self.k)
        ok = (m == len(wi) and torch.equal(self.out_i[j][:m].cpu().to(torch.int64), wi.cpu().to(torch.int64)) and
              torch.equal(self.out_d[j][:m].cpu().view(torch.int64), wd.cpu().view(torch.int64)))
        if ok and self.has_range:
            want = self.ctx.range_pp(self.grid, self.xs[w], self.ys[w], self.q[0], self.q[1], self.radius)
            ok = int(self.out_rc[j].item()) == len(want)
        return ok

    def step(self, s):
        import torch
        if self.args.partition == "cells":
            self.cells_last = self.cells_window(s % self.windows)  # (merged top-k, range hits, received)
            return
        self.last_s = s
        j = s & 1
        if self.world > 1 and self.ev_done[j] is not None:
            torch.cuda.current_stream(self.dev).wait_event(self.ev_done[j])  # row j free again
        self.scan(s % self.windows, j)
        if self.world > 1:
            self.ev_scan[j].record(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(self.cs):
                self.cs.wait_event(self.ev_scan[j])
                self.gather_merge(j)
                ev = torch.cuda.Event()
                ev.record(self.cs)
                self.ev_done[j] = ev

    def algorithmic_bytes(self):
        return BYTES_PER_POINT * self.n

    def config(self):
        return {"workload": f"{self.label}, {self.n} uniform points per window per GPU (BASELINE.json configs[1])",
                "points_per_window_per_gpu": self.n, "grid": self.grid_n, "k": self.k, "radius": self.radius,
                "windows_resident": self.windows,
                "parallelism": f"shard{self.world}"}

    def e2e(self):
        """The C2 window as a host (pageable numpy) array through geohip_knn_pp in
        GEOHIP_MEM_HOST mode: pinned two-slot staging in 1M-point chunks, each chunk's knn_pass
        launched as its DMA lands (overlapping the later copies), chunk lists merged, k results
        copied back.  Wall clock per window, results on the host."""
        import torch
        from spatialflink_amd import Context
        hx = self.xs[0].cpu().numpy()
        hy = self.ys[0].cpu().numpy()
        ctx = Context(self.dev.index)
        want = self.ctx.knn_pp(self.grid, self.xs[0], self.ys[0], self.q[0], self.q[1], self.radius, self.k)
        torch.cuda.synchronize(self.dev)
        gi, gd = ctx.knn_pp(self.grid, hx, hy, self.q[0], self.q[1], self.radius, self.k)  # warm-up, check
        same = gi.tolist() == want[0].cpu().numpy().astype(np.uint32).tolist()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.knn_pp(self.grid, hx, hy, self.q[0], self.q[1], self.radius, self.k)
        t = (time.perf_counter() - t0) / reps
        ctx.close()
        return {"value": self.n / t, "unit": "points/sec", "ms_per_window": t * 1e3,
                "h2d_GBps": BYTES_PER_POINT * self.n / t / 1e9, "matches_device_path": same, "windows_timed": reps,
                "path": "pageable host x/y -> ctx-owned pinned 2-slot staging (1M-point chunks, persistent copy workers) -> "
                        "per-chunk knn_pass as each chunk lands (copy stream / compute stream overlap) -> "
                        "rebase + merge -> k results to host"}

    def pipelined(self, windows=400, nstreams=2):
        """Consecutive windows on nstreams contexts / HIP streams (as Flink task slots sharing
        the GPU would run them): window i+1's scan starts on the CUs window i's blocks free, so
        the per-window tail (block lists, the last block's final selection) overlaps the next
        stream.  Reported beside the strict one-window-per-step line, not as `value`."""
        import torch
        from spatialflink_amd import Context
        ctxs = [self.ctx] + [Context(self.dev.index) for _ in range(nstreams - 1)]
        streams = [torch.cuda.Stream(self.dev) for _ in ctxs]
        # every window writes its own result slot, so every window is checked afterwards
        oi = torch.empty((windows, self.k), dtype=torch.int32, device=self.dev)
        od = torch.empty((windows, self.k), dtype=torch.float64, device=self.dev)
        oc = torch.zeros(windows, dtype=torch.int32, device=self.dev)
        old = self.ctx._bound
        try:
            for c in ctxs:
                c.follow_torch_stream(True)

            def run(nw):
                for i in range(nw):
                    j = i % nstreams
                    with torch.cuda.stream(streams[j]):
                        ctxs[j].knn_pp_async(self.grid, self.xs[i % self.windows], self.ys[i % self.windows],
                                             self.q[0], self.q[1], self.radius, self.k, oi[i], od[i], oc[i:i + 1])
            torch.cuda.synchronize(self.dev)
            run(16)
            torch.cuda.synchronize(self.dev)
            oi.fill_(-7)
            od.fill_(-7.0)
            t0 = time.perf_counter()
            run(windows)
            torch.cuda.synchronize(self.dev)
            t = (time.perf_counter() - t0) / windows
            # every window against the sequential path of the same window: indices and distance bits
            ref = []
            for w in range(self.windows):
                wi, wd = self.ctx.knn_pp(self.grid, self.xs[w], self.ys[w], self.q[0], self.q[1], self.radius, self.k)
                ref.append((wi.cpu().numpy().astype(np.uint32), wd.cpu().numpy().view(np.uint64)))
            gi = oi.cpu().numpy().astype(np.uint32)
            gd = od.cpu().numpy().view(np.uint64)
            same = all(np.array_equal(gi[i], ref[i % self.windows][0]) and np.array_equal(gd[i], ref[i % self.windows][1])
                       for i in range(windows))
        finally:
            for c in ctxs[1:]:
                c.close()
            self.ctx.set_stream(old)
        return {"value": self.n / t, "unit": "points/sec", "us_per_window": t * 1e6,
                "hbm_GBps": BYTES_PER_POINT * self.n / t / 1e9,
                "hbm_frac": BYTES_PER_POINT * self.n / t / 1e9 / HBM_PEAK_GBS, "streams": nstreams, "windows": windows,
                "matches_sequential": same, "checked": "every window: indices and distance bits"}

    def cpu_baseline(self, seconds):
        cref = _oracle()
        from spatialflink_amd import synth
        bj, q = synth.BEIJING, synth.README_QUERY
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        n = self.n
        x, y = synth.uniform(n, self.seed0)  # the benchmarked window itself

        def one(i):
            t0 = time.perf_counter()
            cref.knn_pp(cg, x, y, q[0], q[1], self.radius, self.k)
            return time.perf_counter() - t0
        wins, t = _timed_loop(one, seconds, 1000)
        return {"value": wins * n / t, "unit": "points/sec", "cores": cref.threads(), "kind": "port",
                "sample": f"{wins} windows x {n} uniform points (k={self.k}, {self.grid_n}x{self.grid_n}, "
                          f"r={self.radius}), oracle/geohip_oracle.c, OpenMP {cref.threads()} threads "
                          f"(points of a window in parallel, per-thread heaps merged), {t:.1f} s"}


class RangeWorkload(Workload):
    """C1 query shape (BASELINE.json configs[0]: 100x100, README query, r=0.5) at 10M points per
    GPU (C1's 1M-point window is the reference's CPU case; on the GPU it is launch-bound)."""
    tag = "range"
    kernel = ("geohip::range_set (one launch per window: classify, exact distances in C cells, hits staged per wave "
              "and stored in reserved runs while the window streams; unordered-set output, GEOHIP_ORDER_ANY)")
    grid_n, radius, n_default = 100, 0.5, 10_000_000

    def __init__(self, *a):
        super().__init__(*a)
        import torch
        from spatialflink_amd import _abi, synth
        self.n = self.args.points or self.n_default
        bj = synth.BEIJING
        self.q = synth.README_QUERY
        self.grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        self.xs, self.ys = _uniform_windows(self.ctx, self.dev, self.n, self.rank,
                                            [1 + 7919 * w for w in range(self.windows)], bj)
        # the reference's window result is a set (PointPointRangeQuery.java:117-136)
        self.ctx.set_range_order(not self.args.range_ascending)
        if self.args.range_ascending:
            self.kernel = ("geohip::range_fused (one launch per window: classify, exact distances in C cells, per-block "
                           "hit masks, ticket-ordered look-back over block counts, ascending emission)")
        self.out = torch.empty(self.n, dtype=torch.int32, device=self.dev)
        self.cnt = torch.zeros(self.windows, dtype=torch.int64, device=self.dev)
        self.counts = torch.zeros(self.world, dtype=torch.int64, device=self.dev)
        self.hits = None
        self.cs = torch.cuda.Stream(self.dev) if self.world > 1 else None
        self.done = [None] * self.windows
        self.stepped = set()

    def units_per_step(self):
        return self.n

    def step(self, s):
        import torch
        w = s % self.windows
        cur = torch.cuda.current_stream(self.dev)
        if self.world > 1 and self.done[w] is not None:
            cur.wait_event(self.done[w])  # window w's count slot gathered
        self.last_w = w
        self.stepped.add(w)
        self.ctx.range_pp_async(self.grid, self.xs[w], self.ys[w], self.q[0], self.q[1], self.radius, False,
                                self.out, self.n, self.cnt[w:w + 1])
        if self.world > 1:  # result gather: every rank learns each shard's hit count (offsets), on the
            ev = torch.cuda.Event()  # communication stream, overlapping the next window's pass
            ev.record(cur)
            with torch.cuda.stream(self.cs):
                self.cs.wait_event(ev)
                if self.dist.get_backend() == "gloo":
                    ch = torch.empty(self.world, dtype=torch.int64)
                    self.dist.all_gather_into_tensor(ch, self.cnt[w:w + 1].cpu())
                    self.counts.copy_(ch)
                else:
                    self.dist.all_gather_into_tensor(self.counts, self.cnt[w:w + 1])
                self.done[w] = torch.cuda.Event()
                self.done[w].record(self.cs)

    def verify(self):
        """After the timed region: every resident window's device hit count, and the last step's
        hit set, against the synchronous call on the same window."""
        import torch
        self.ctx.sync()
        got = self.cnt.cpu().tolist()
        want = {w: self.ctx.range_pp(self.grid, self.xs[w], self.ys[w], self.q[0], self.q[1], self.radius)
                for w in self.stepped}
        if any(got[w] != len(h) for w, h in want.items()):
            return False
        w = self.last_w
        m = got[w]
        return torch.equal(torch.sort(self.out[:m].to(torch.int64)).values.cpu(),
                           torch.sort(want[w].to(torch.int64)).values.cpu())

    def algorithmic_bytes(self):
        if self.hits is None:
            self.hits = float(self.cnt.double().mean().item())
        return BYTES_PER_POINT * self.n + 4 * self.hits

    def config(self):
        return {"workload": f"C1 query shape (point-point range, 100x100 Beijing UniformGrid, README query, r=0.5, "
                            f"exact) over {self.n} uniform points per window per GPU",
                "output": "ascending hit indices" if self.args.range_ascending else "unordered hit set (GEOHIP_ORDER_ANY)",
                "points_per_window_per_gpu": self.n, "grid": self.grid_n, "radius": self.radius,
                "hits_per_window_per_gpu": self.hits, "windows_resident": self.windows,
                "parallelism": f"shard{self.world}"}

    def cpu_baseline(self, seconds):
        cref = _oracle()
        from spatialflink_amd import synth
        bj, q = synth.BEIJING, synth.README_QUERY
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        n = 1_000_000  # C1's own window size
        x, y = synth.uniform(n, 1)

        def one(i):
            t0 = time.perf_counter()
            cref.range_pp(cg, x, y, q[0], q[1], self.radius)
            return time.perf_counter() - t0
        wins, t = _timed_loop(one, seconds, 5000)
        return {"value": wins * n / t, "unit": "points/sec", "cores": cref.threads(), "kind": "port",
                "sample": f"{wins} windows x {n} uniform points (C1: 100x100, r={self.radius}), "
                          f"oracle/geohip_oracle.c, OpenMP {cref.threads()} threads, {t:.1f} s"}


class JoinWorkload(Workload):
    """C3 (BASELINE.json configs[2]): 10k queries x 10M Gaussian-clustered data points per
    window, 500x500, r = 0.05 (32 shared centres, sigma 0.1)."""
    tag = "join_probe"
    kernel = ("geohip join step: query block lists (jq_rect / jq_build / jq_starts), tile binning into 16-B "
              "records with the work-item plan (jb_bands / jb_scan / jb_segs / jb_tiles), join_fused (work "
              "items, decoupled look-back, LDS-staged 512-B pair stores); every kernel timed by its dispatch stamps")
    grid_n, radius, n_default, nq, sigma = 500, 0.05, 10_000_000, 10_000, 0.1
    windows = 2

    def __init__(self, *a):
        super().__init__(*a)
        import torch
        from spatialflink_amd import _abi, synth
        self.n = self.args.points or self.n_default
        bj = synth.BEIJING
        self.grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        self.dx, self.dy = [], []
        for w in range(self.windows):
            hx, hy = synth.gaussian_clusters(self.n, 3 + 100 * w + 7 * self.rank, sigma=self.sigma)
            self.dx.append(torch.from_numpy(hx).to(self.dev))
            self.dy.append(torch.from_numpy(hy).to(self.dev))
        hqx, hqy = synth.gaussian_clusters(self.nq, 4, sigma=self.sigma)  # the query stream, on every rank
        self.qx = torch.from_numpy(hqx).to(self.dev)
        self.qy = torch.from_numpy(hqy).to(self.dev)
        self.pairs = [self.ctx.join_pp_count(self.grid, self.grid, self.dx[w], self.dy[w], self.qx, self.qy,
                                             self.radius) for w in range(self.windows)]
        self.out = torch.empty((max(self.pairs) + 1, 2), dtype=torch.int32, device=self.dev)
        self.counts = torch.zeros(self.world, dtype=torch.int64, device=self.dev)
        self.cnt = torch.zeros(self.windows, dtype=torch.int64, device=self.dev)  # async steps' pair totals

    def units_per_step(self):
        return self.n

    def cells_window(self, w):
        """One window in the north-star layout (PointPointJoinQuery.java:137-150): data points
        packed by owner key band (geohip_band_pack_async), one all-to-all, each owner joins its
        band against the query window (geohip_join_pp_async into preallocated rows), the ranks'
        pair counts in one device all-gather -- enqueue-only but for the shuffle's split sizes
        (distributed.join_cells_enqueue)."""
        import torch
        from spatialflink_amd import distributed as D
        if getattr(self, "cout", None) is None:  # any rank's pairs <= the whole window's
            cap = sum(self._gather_ints(max(self.pairs)))
            self.cout = torch.empty((cap + 1, 2), dtype=torch.int32, device=self.dev)
            self.ccount = torch.zeros(1, dtype=torch.int64, device=self.dev)
            self.ccounts = torch.zeros(self.world, dtype=torch.int64, device=self.dev)
        return D.join_cells_enqueue(self.dx[w], self.dy[w], self.rank * self.n, self.qx, self.qy, self.radius,
                                    grid_data=self.grid, grid_query=self.grid, ctx=self.ctx, out=self.cout,
                                    count=self.ccount, counts=self.ccounts)

    def cells_partition(self, steps):
        if self.world == 1:
            return None  # one band: the arrival line itself
        t, out = self._timed_side(lambda s: self.cells_window(s % self.windows), steps)
        m, _, total = out.totals()  # counts only (the pairs stay on the device)
        w = (steps - 1) % self.windows
        want = sum(self._gather_ints(self.pairs[w]))
        pr = self._gather_ints(m)
        mean = sum(pr) / len(pr)
        return {"value": self.n * self.world * steps / t, "unit": "points/sec", "ms_per_step": t / steps * 1e3,
                "steps": steps, "layout": "grid-cell key bands: data points packed by owner band "
                "(geohip_band_pack_async), all_to_all, owner's join of its band against the query window "
                "(geohip_join_pp_async), device all-gather of the pair counts",
                "pairs_per_rank": pr, "skew_max_over_mean": (max(pr) / mean) if mean else None,
                "matches_arrival_sharding": total == want}

    def step(self, s):
        import torch
        w = s % self.windows
        if self.args.partition == "cells":
            self.cells_last = self.cells_window(w)  # (this rank's pairs, offset, window total)
            return
        # enqueue-only (geohip_join_pp_async): the pair total stays on the device, no host round trip
        self.ctx.join_pp_async(self.grid, self.grid, self.dx[w], self.dy[w], self.qx, self.qy, self.radius, False,
                               self.out, self.cnt[w:w + 1])
        if self.world > 1:  # result gather: each rank's pair count of this step (output offsets)
            self.dist.all_gather_into_tensor(self.counts, self.cnt[w:w + 1])

    def verify(self):
        if self.args.partition == "cells":
            return None
        self.ctx.sync()  # faults of the async steps (query keys) raise here
        return self.cnt.cpu().tolist() == self.pairs

    def check_merged(self, last_step):
        """N > 1, key-band step (--check): the window's pair total over the band owners against the
        arrival-sharded join's (every rank joins its own shard in __init__).  Rank 0 only."""
        if self.args.partition != "cells":
            return None
        want = sum(self._gather_ints(self.pairs[last_step % self.windows]))
        return (int(self.cells_last.totals()[2]) == want) if self.rank == 0 else None

    def algorithmic_bytes(self):
        if self.args.partition == "cells" and getattr(self, "cells_last", None) is not None:
            # key bands: this rank's own step (ranks' bands differ: skew) -- its shard read by the
            # pack, its received band and the queries read by its join, its own pairs written
            m, _, _ = self.cells_last.totals()
            nrecv = int(self.cells_last.rg.numel())
            return BYTES_PER_POINT * (self.n + nrecv + self.nq) + 8 * float(m)
        return BYTES_PER_POINT * self.n + BYTES_PER_POINT * self.nq + 8 * float(np.mean(self.pairs))

    def config(self):
        return {"workload": f"C3: point-point join, {self.nq} queries x {self.n} data points per window per GPU, "
                            f"Gaussian-clustered (32 shared centres, sigma={self.sigma}), {self.grid_n}x{self.grid_n}, "
                            f"r={self.radius}; units = data points",
                "points_per_window_per_gpu": self.n, "queries": self.nq, "grid": self.grid_n, "radius": self.radius,
                "pairs_per_window_per_gpu": float(np.mean(self.pairs)), "windows_resident": self.windows,
                "parallelism": f"shard{self.world} (data by arrival, queries replicated)"}

    def cpu_baseline(self, seconds):
        cref = _oracle()
        from spatialflink_amd import synth
        bj = synth.BEIJING
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        n = 2_000_000  # data slice of the C3 window; all 10k queries
        qx, qy = synth.gaussian_clusters(self.nq, 4, sigma=self.sigma)
        x, y = synth.gaussian_clusters(n, 3, sigma=self.sigma)

        def one(i):
            t0 = time.perf_counter()
            cref.join_pp_hash(cg, cg, x, y, qx, qy, self.radius)  # one pass, as the reference
            return time.perf_counter() - t0
        wins, t = _timed_loop(one, seconds, 200)
        return {"value": wins * n / t, "unit": "points/sec", "cores": cref.threads(), "kind": "port",
                "sample": f"{wins} x ({n} Gaussian data points x {self.nq} queries) (C3 shape, pairs counted and "
                          f"hashed, not stored), oracle/geohip_oracle.c, OpenMP {cref.threads()} threads, {t:.1f} s"}


class PpolyWorkload(Workload):
    """C4 (BASELINE.json configs[3]): 1k star polygons (50 vertices) over 50M uniform points per
    window, 500x500, r = 0.005 (conf/geoflink-conf.yml:52)."""
    tag = "ppoly_probe"
    kernel = ("geohip point-polygon step: ppoly_stream (one pass over the window: cell-table heads, decided pairs, "
              "mixed-subcell candidates, one reservation per chunk) + ppoly_cand_refine (4x4 parts of mixed "
              "subcells) + candidates grouped by polygon + ppoly_cand_eval (exact JTS tests); the whole device "
              "step is timed")
    grid_n, radius, n_default, npoly = 500, 0.005, 50_000_000, 1000
    windows = 2

    def __init__(self, *a):
        super().__init__(*a)
        import torch
        from spatialflink_amd import _abi, synth
        self.n = self.args.points or self.n_default
        bj = synth.BEIJING
        self.grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        self.xs, self.ys = _uniform_windows(self.ctx, self.dev, self.n, self.rank,
                                            [5 + 7919 * w for w in range(self.windows)], bj)
        self.off, self.vx, self.vy = synth.star_polygons(self.npoly, 6)
        torch.cuda.synchronize(self.dev)
        self.hits = [len(self.ctx.range_ppoly(self.grid, self.xs[w], self.ys[w], self.off, self.vx, self.vy,
                                              self.radius)) for w in range(self.windows)]
        self.out = torch.empty((max(self.hits) + 1, 2), dtype=torch.int32, device=self.dev)
        self.cnt = torch.zeros(self.windows, dtype=torch.int64, device=self.dev)  # async steps' pair totals

    def units_per_step(self):
        return self.n

    def step(self, s):
        w = s % self.windows
        # enqueue-only (geohip_range_ppoly_async): no end-of-step count readback
        self.ctx.range_ppoly_async(self.grid, self.xs[w], self.ys[w], self.off, self.vx, self.vy, self.radius, False,
                                   self.out, self.cnt[w:w + 1])

    def verify(self):
        self.ctx.sync()  # a candidate-buffer overflow of an async step raises here
        return self.cnt.cpu().tolist() == self.hits

    def algorithmic_bytes(self):
        return BYTES_PER_POINT * self.n + 16 * len(self.vx) + 8 * float(np.mean(self.hits))

    def algorithmic_flops(self):
        """candidate pairs x ~1.85 kflop (50 crossings + 50 segment distances per
        JTS DistanceOp).  Candidate pairs = the window's points in each polygon's G u C cells (the
        reference's per-candidate distance work): the bbox-cell rectangle (HelperClass.java:123-143)
        dilated by Lc = ceil(r / l) (UniformGrid.java:398-444), clipped, counted from the window's
        cell histogram (first window)."""
        if getattr(self, "_alg_flops", None) is None:
            from spatialflink_amd import synth
            bj = synth.BEIJING
            n_, l = self.grid_n, (bj[1] - bj[0]) / self.grid_n
            x = self.xs[0].cpu().numpy()
            y = self.ys[0].cpu().numpy()
            cx = np.floor((x - bj[0]) / l)
            cy = np.floor((y - bj[2]) / l)
            ok = (cx >= 0) & (cx < n_) & (cy >= 0) & (cy < n_)
            h = np.zeros((n_ + 1, n_ + 1), np.int64)
            np.add.at(h, (cx[ok].astype(np.int64) + 1, cy[ok].astype(np.int64) + 1), 1)
            S = h.cumsum(0).cumsum(1)  # S[a, b] = points in cells [0, a) x [0, b)
            lc = int(math.ceil(self.radius / l))
            cand = 0
            for p in range(self.npoly):
                a, b = int(self.off[p]), int(self.off[p + 1])
                px, py = self.vx[a:b], self.vy[a:b]
                x0 = max(int(math.floor((px.min() - bj[0]) / l)) - lc, 0)
                x1 = min(int(math.floor((px.max() - bj[0]) / l)) + lc, n_ - 1)
                y0 = max(int(math.floor((py.min() - bj[2]) / l)) - lc, 0)
                y1 = min(int(math.floor((py.max() - bj[2]) / l)) + lc, n_ - 1)
                if x0 <= x1 and y0 <= y1:
                    cand += int(S[x1 + 1, y1 + 1] - S[x0, y1 + 1] - S[x1 + 1, y0] + S[x0, y0])
            self._alg_cand = cand
            self._alg_flops = cand * 1850.0
        return self._alg_flops

    def config(self):
        return {"workload": f"C4: point-polygon range, {self.npoly} polygons x 50 vertices over {self.n} uniform "
                            f"points per window per GPU, {self.grid_n}x{self.grid_n}, r={self.radius}",
                "points_per_window_per_gpu": self.n, "polygons": self.npoly, "grid": self.grid_n,
                "radius": self.radius, "hits_per_window_per_gpu": float(np.mean(self.hits)),
                "windows_resident": self.windows, "parallelism": f"shard{self.world}"}

    def cpu_baseline(self, seconds):
        cref = _oracle()
        from spatialflink_amd import synth
        bj = synth.BEIJING
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        n = 5_000_000  # a 5M-point slice of the C4 window, all 1k polygons
        x, y = synth.uniform(n, 5)

        def one(i):
            t0 = time.perf_counter()
            cref.range_ppoly_hash(cg, x, y, self.off, self.vx, self.vy, self.radius)
            return time.perf_counter() - t0
        reps, t = _timed_loop(one, seconds, 200)
        return {"value": reps * n / t, "unit": "points/sec", "cores": cref.threads(), "kind": "port",
                "sample": f"{reps} x ({n} uniform points x {self.npoly} polygons) (C4 shape), oracle/geohip_oracle.c "
                          f"(polygons in parallel over OpenMP {cref.threads()} threads, each visiting its G u C "
                          f"cells), {t:.1f} s"}


class PpJoinWorkload(PpolyWorkload):
    """the C4 shape as a point-polygon join (PointPolygonJoinQuery,
    polygon stream replicated to its G/C cells, every candidate distance-checked)."""
    tag = "ppjoin"
    kernel = ("geohip point-polygon join step: ppoly_stream + refinement + candidate grouping + ppoly_cand_eval in join mode; "
              "the whole device step is timed")

    def __init__(self, *a):
        Workload.__init__(self, *a)
        import torch
        from spatialflink_amd import _abi, synth
        self.n = self.args.points or self.n_default
        bj = synth.BEIJING
        self.grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        self.xs, self.ys = _uniform_windows(self.ctx, self.dev, self.n, self.rank,
                                            [5 + 7919 * w for w in range(self.windows)], bj)
        self.off, self.vx, self.vy = synth.star_polygons(self.npoly, 6)
        torch.cuda.synchronize(self.dev)
        self.hits = [len(self.ctx.join_ppoly(self.grid, self.grid, self.xs[w], self.ys[w], self.off, self.vx, self.vy,
                                             self.radius)) for w in range(self.windows)]
        self.out = torch.empty((max(self.hits) + 1, 2), dtype=torch.int32, device=self.dev)
        self.cnt = torch.zeros(self.windows, dtype=torch.int64, device=self.dev)

    def step(self, s):
        w = s % self.windows
        self.ctx.join_ppoly_async(self.grid, self.grid, self.xs[w], self.ys[w], self.off, self.vx, self.vy,
                                  self.radius, False, self.out, self.cnt[w:w + 1])

    def config(self):
        c = super().config()
        c["workload"] = (f"point-polygon join: {self.npoly} polygons (50 vertices) x {self.n} uniform points per window "
                         f"per GPU, {self.grid_n}x{self.grid_n}, r={self.radius} (C4 shape, PointPolygonJoinQuery)")
        c["pairs_per_window_per_gpu"] = c.pop("hits_per_window_per_gpu")
        return c

    def cpu_baseline(self, seconds):
        cref = _oracle()
        from spatialflink_amd import synth
        bj = synth.BEIJING
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        n = 5_000_000
        x, y = synth.uniform(n, 5)

        def one(i):
            t0 = time.perf_counter()
            cref.join_ppoly_hash(cg, cg, x, y, self.off, self.vx, self.vy, self.radius)
            return time.perf_counter() - t0
        reps, t = _timed_loop(one, seconds, 200)
        return {"value": reps * n / t, "unit": "points/sec", "cores": cref.threads(), "kind": "port",
                "sample": f"{reps} x ({n} uniform points x {self.npoly} polygons), oracle/geohip_oracle.c join_ppoly, "
                          f"OpenMP {cref.threads()} threads, {t:.1f} s"}


class PpKnnWorkload(Workload):
    """point-polygon kNN (PointPolygonKNNQuery) of one star polygon,
    k = 50, over the C4 window (50M uniform points per GPU, 500x500, r = 0.005)."""
    tag = "ppknn"
    kernel = "geohip ppknn_scan_boxes + ppknn_dist + one-workgroup radix select (rsel_small); plan cached, no host sync"
    grid_n, radius, n_default, k = 500, 0.005, 50_000_000, 50
    windows = 2

    def __init__(self, *a):
        super().__init__(*a)
        from spatialflink_amd import _abi, synth
        self.n = self.args.points or self.n_default
        bj = synth.BEIJING
        self.grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        self.xs, self.ys = _uniform_windows(self.ctx, self.dev, self.n, self.rank,
                                            [5 + 7919 * w for w in range(self.windows)], bj)
        off, vx, vy = synth.star_polygons(1, 6)
        self.vx, self.vy = vx, vy
        import torch
        self.oi = torch.empty(self.k, dtype=torch.int32, device=self.dev)
        self.od = torch.empty(self.k, dtype=torch.float64, device=self.dev)
        self.oc = torch.zeros(1, dtype=torch.int32, device=self.dev)

    def units_per_step(self):
        return self.n

    def step(self, s):
        w = s % self.windows  # the device form: plan cached by the ctx, no host round trip
        self.ctx.knn_ppoly_async(self.grid, self.xs[w], self.ys[w], self.vx, self.vy, self.radius, self.k, False,
                                 self.oi, self.od, self.oc)

    def algorithmic_bytes(self):
        return BYTES_PER_POINT * self.n

    def config(self):
        return {"workload": f"point-polygon kNN k={self.k}: one 50-vertex star polygon over {self.n} uniform points per "
                            f"window per GPU, {self.grid_n}x{self.grid_n}, r={self.radius} (C4 window, "
                            f"PointPolygonKNNQuery)",
                "points_per_window_per_gpu": self.n, "grid": self.grid_n, "k": self.k, "radius": self.radius,
                "windows_resident": self.windows, "parallelism": f"shard{self.world}"}

    def cpu_baseline(self, seconds):
        cref = _oracle()
        from spatialflink_amd import synth
        bj = synth.BEIJING
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        n = 10_000_000
        x, y = synth.uniform(n, 5)

        def one(i):
            t0 = time.perf_counter()
            cref.knn_ppoly(cg, x, y, self.vx, self.vy, self.radius, self.k)
            return time.perf_counter() - t0
        reps, t = _timed_loop(one, seconds, 500)
        return {"value": reps * n / t, "unit": "points/sec", "cores": cref.threads(), "kind": "port",
                "sample": f"{reps} windows x {n} uniform points (same polygon, k, grid, r), oracle/geohip_oracle.c "
                          f"knn_ppoly, OpenMP {cref.threads()} threads, {t:.1f} s"}


class PpolyIncrWorkload(PpolyWorkload):
    """SURVEY.md 8(f) row 3 where pane reuse pays: the C4 point-polygon range over 10 s / 5 s
    sliding windows -- one step = one new 25M-point pane (half the 50M-point window) evaluated
    once against the 1k polygons, the window's pairs assembled from its two panes
    (spatialflink_amd.incremental.IncrementalPPolyRange).  value = stream points/sec."""
    tag = "ppoly_incr"
    kernel = "geohip point-polygon step on one pane (ppoly_stream + refinement + candidate grouping + ppoly_cand_eval, timed)"
    n_default = 25_000_000
    windows = 4

    def __init__(self, *a):
        super().__init__(*a)
        from spatialflink_amd.incremental import IncrementalPPolyRange
        import torch
        self.inc = IncrementalPPolyRange(self.ctx, self.grid, self.off, self.vx, self.vy, self.radius, False, 2)
        self.outs = [torch.empty((max(self.hits) + 1, 2), dtype=torch.int32, device=self.dev) for _ in range(2)]
        self.pcnt = torch.zeros((self.windows, 1), dtype=torch.int64, device=self.dev)  # per window slot

    def verify(self):
        self.ctx.sync()  # a candidate-buffer overflow of an async pane raises here
        return self.pcnt.view(-1).cpu().tolist() == self.hits

    def step(self, s):
        w = s % self.windows
        # enqueue-only pane (geohip_range_ppoly_pane_async): no end-of-step count readback
        self.inc.push(self.xs[w], self.ys[w], out=self.outs[s % 2], count=self.pcnt[w])

    def config(self):
        c = super().config()
        c["workload"] = (f"C4 over 10s/5s sliding windows with pane reuse: {self.npoly} polygons x 50 vertices, "
                         f"{self.n} new uniform points per pane (window = 2 panes) per GPU, "
                         f"{self.grid_n}x{self.grid_n}, r={self.radius}")
        c["points_per_pane_per_gpu"] = c.pop("points_per_window_per_gpu")
        c["panes_per_window"] = 2
        return c


class KnnIncrWorkload(KnnWorkload):
    """the C2 kNN over 10 s / 5 s sliding windows with pane reuse -- one
    step = one new 5M-point pane (half a 10M-point window) evaluated once, then the window's
    top-k merged from its two panes' top-k lists (spatialflink_amd.incremental.IncrementalKNN).
    value = stream points/sec (each point is evaluated once, not once per window)."""
    tag = "knn_incr"
    kernel = "geohip::knn_pass<16> on one pane + one knn_merge_panes launch (2 panes, rebase folded in)"
    n_default = 5_000_000
    label = "C2 over 10s/5s sliding windows with pane reuse: kNN k=50, 100x100 Beijing UniformGrid, r=0.5"

    def cells_partition(self, steps):  # pane reuse is a single-GPU stream form
        return None

    def __init__(self, *a):
        super().__init__(*a)
        from spatialflink_amd.incremental import IncrementalKNN
        self.inc = IncrementalKNN(self.ctx, self.grid, self.q[0], self.q[1], self.radius, self.k, 2)

    def step(self, s):
        w = s % self.windows
        self.inc.push(self.xs[w], self.ys[w], sync=False)

    def verify(self):  # the pane merges are checked by tests/test_gpu_incremental.py
        return None

    def config(self):
        c = super().config()
        c["workload"] = f"{self.label}, {self.n} new points per pane (window = 2 panes) per GPU"
        c["points_per_pane_per_gpu"] = c.pop("points_per_window_per_gpu")
        c["panes_per_window"] = 2
        return c


class C5Workload(KnnWorkload):
    """C5 per shard (BASELINE.json configs[4]): 1000x1000 grid, 25M uniform points per GPU
    (200M per window on 8 GPUs), kNN k=100 + range r=0.05 of the README query -- both queries in
    one pass over the shard (geohip_knn_range_pp), then for N > 1 the RCCL all-gather of the
    ranks' top-k + the device merge and the all-gather of the range hit counts."""
    tag = "knn_scan_c5"
    kernel = "geohip::knn_pass<16, range> (kNN k=100 + range r=0.05 in one pass: one launch per step)"
    grid_n, k, radius, n_default, seed0 = 1000, 100, 0.05, 25_000_000, 7
    windows = 2
    has_range = True
    label = "C5 shard: kNN k=100 + range r=0.05, 1000x1000 Beijing UniformGrid, README query"

    def __init__(self, *a):
        super().__init__(*a)
        import torch
        # the range part's output is a set (PointPointRangeQuery.java:117-136): the fused pass then
        # sweeps the window in interleaved fronts and reserves its hits without a look-back
        self.ctx.set_range_order(not self.args.range_ascending)
        if not self.args.range_ascending:
            self.kernel = ("geohip::knn_pass<16, range, unordered> (kNN k=100 + range r=0.05 in one pass, interleaved "
                           "fronts, range hits reserved per block: one launch per step)")
        self.rout = torch.empty(self.n, dtype=torch.int32, device=self.dev)
        self.hits = None

    def scan(self, w, j):
        # the range hit count rides in the packed row: one all-gather carries the top-k and the
        # counts (the ranks' output offsets of the concatenated range result)
        self.ctx.knn_range_pp_async(self.grid, self.xs[w], self.ys[w], self.q[0], self.q[1], self.radius, self.k, False,
                                    self.out_i[j], self.out_d[j], self.cnt[0:1], self.rout, self.n, self.out_rc[j])

    def algorithmic_bytes(self):  # per step: the shard read once (16 B/pt) + the range hits written
        if self.hits is None:
            if self.args.partition == "cells" and getattr(self, "cells_last", None) is not None:
                self.hits = float(self.cells_last.result()[1][2]) / self.world  # the window's hits, per GPU
            else:
                self.hits = float(self.out_rc[0].item())
        return BYTES_PER_POINT * self.n + 4 * self.hits

    def config(self):
        c = super().config()
        c["workload"] = f"{self.label}, {self.n} uniform points per window per GPU (BASELINE.json configs[4])"
        c["range_hits_per_window_per_gpu"] = self.hits
        c["range_output"] = "ascending hit indices" if self.args.range_ascending else "unordered hit set (GEOHIP_ORDER_ANY)"
        return c

    def cpu_baseline(self, seconds):
        cref = _oracle()
        from spatialflink_amd import synth
        bj, q = synth.BEIJING, synth.README_QUERY
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        n = self.n
        x, y = synth.uniform(n, self.seed0)  # rank 0's shard of the C5 window

        def one(i):
            t0 = time.perf_counter()
            cref.knn_pp(cg, x, y, q[0], q[1], self.radius, self.k)
            cref.range_pp_hash(cg, x, y, q[0], q[1], self.radius)
            return time.perf_counter() - t0
        wins, t = _timed_loop(one, seconds, 1000)
        return {"value": wins * n / t, "unit": "points/sec", "cores": cref.threads(), "kind": "port",
                "sample": f"{wins} x one {n}-point C5 shard (kNN k={self.k} + range r={self.radius}, "
                          f"{self.grid_n}x{self.grid_n}), oracle/geohip_oracle.c, OpenMP {cref.threads()} threads, "
                          f"{t:.1f} s"}


class IngestWorkload(Workload):
    """the window's CSV records (CSVTSVToTSpatial, Deserialization.java:
    288-322, schema [oid, ts, x, y]) parsed into SoA x/y + Long ts + the Point constructor's cell
    (Point.java:91-100 -> HelperClass.java:104-116) on the device; the C2 window size (10M records)
    and grid (100x100).  Text is device-resident before the timed region."""
    tag = "ingest"
    kernel = "geohip ingest: ingest_fused (one launch per batch: chunk ticket, record split, look-back record base, parse)"
    grid_n, n_default = 100, 10_000_000
    windows = 1  # one batch of ~570 MB is > the 256 MiB Infinity Cache

    def __init__(self, *a):
        super().__init__(*a)
        import torch
        from spatialflink_amd import _abi, synth
        self.n = self.args.points or self.n_default
        bj = synth.BEIJING
        self.grid = _abi.make_grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        text, self.X, self.Y = synth.csv_text(self.n, 2 + 7 * self.rank)
        self.nbytes = int(text.size)
        self.text = torch.from_numpy(text).to(self.dev)
        del text
        self.spec = _abi.make_ingest_spec(_abi.FMT_CSV, ",", 2, 3, 1)
        mk = lambda dt: torch.empty(self.n, dtype=dt, device=self.dev)  # noqa: E731
        self.out = {"x": mk(torch.float64), "y": mk(torch.float64), "ts": mk(torch.int64), "cell": mk(torch.int32)}
        got = self.ctx.ingest_points(self.spec, self.text, self.grid, with_ts=True, with_cell=True, cap=self.n,
                                     out=self.out)
        assert len(got["x"]) == self.n, "ingest record count"

    def units_per_step(self):
        return self.n

    def step(self, s):
        self.ctx.ingest_points(self.spec, self.text, self.grid, with_ts=True, with_cell=True, cap=self.n, out=self.out)

    def algorithmic_bytes(self):  # text read once + x, y, ts, cell written
        return self.nbytes + (8 + 8 + 8 + 4) * self.n

    def config(self):
        return {"workload": f"ingest: {self.n} CSV records 'oid,ts,x,y' (CSVTSVToTSpatial, 13 fraction digits) -> "
                            f"SoA x/y + ts + cell, 100x100 Beijing UniformGrid (C2 window size)",
                "records_per_batch_per_gpu": self.n, "text_bytes": self.nbytes, "grid": self.grid_n,
                "parallelism": f"shard{self.world}"}

    def cpu_baseline(self, seconds):
        cref = _oracle()
        from spatialflink_amd import synth
        bj = synth.BEIJING
        cg = cref.grid(bj[0], bj[2], (bj[1] - bj[0]) / self.grid_n, self.grid_n)
        spec = cref.ingest_spec(0, ",", 2, 3, 1)  # GEOHIP_FMT_CSV
        n = 1_000_000
        text = bytes(synth.csv_text(n, 9)[0])

        def one(i):
            t0 = time.perf_counter()
            cref.ingest(spec, text, cg)
            return time.perf_counter() - t0
        reps, t = _timed_loop(one, seconds, 30)
        return {"value": reps * n / t, "unit": "points/sec", "cores": 1, "kind": "port",
                "sample": f"{reps} x {n} CSV records (same grammar and shape), oracle/ingest_oracle.c single thread "
                          f"(strtod-class parse + cell), {t:.1f} s"}


WORKLOADS = {"knn": KnnWorkload, "range": RangeWorkload, "join": JoinWorkload, "ppoly": PpolyWorkload,
             "c5": C5Workload, "ingest": IngestWorkload, "ppjoin": PpJoinWorkload, "ppknn": PpKnnWorkload,
             "knn_incr": KnnIncrWorkload, "ppoly_incr": PpolyIncrWorkload}


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # GEOHIP_BENCH_ONE_DEVICE=1 + GEOHIP_BENCH_BACKEND=gloo: every rank on cuda:0 with host-staged
    # collectives -- a functional rehearsal of the N > 1 path on a one-GPU box (not a measurement)
    if os.environ.get("GEOHIP_BENCH_ONE_DEVICE") == "1":
        local = 0
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        backend = os.environ.get("GEOHIP_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)

    from spatialflink_amd import Context, _abi

    dev = torch.device("cuda", local)
    ctx = Context(local)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)  # kernels and RCCL ordered on one stream (0 = the null stream)
    wl = WORKLOADS[args.workload](args, ctx, dev, rank, world, dist)

    torch.cuda.synchronize(dev)
    for s in range(args.warmup):
        wl.step(s)
    torch.cuda.synchronize(dev)
    ctx.timing(reset=True)
    every = max(1, min(args.time_every, args.steps // 4))  # at least 4 timed steps
    ctx.set_timing(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        if every > 1:
            ctx.set_timing(s % every == 0)
        wl.step(args.warmup + s)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    step_ms, launches, kern_ms, kernels = ctx.timing_kernels(reset=True)
    verified = wl.verify()  # the enqueue-only steps' device counts against the counts of __init__
    if verified is False:
        raise SystemExit(f"bench: {args.workload} steps returned counts that differ from the synchronous calls'")
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_points = wl.units_per_step() * world * args.steps
    value = total_points / elapsed
    # the timed kernels' own durations per step (dispatch begin / end stamps, as rocprofv3 reports
    # them; for a multi-launch step the sum over its kernels), and the step bracket beside it
    avg_s = kern_ms / 1e3 / launches if launches and kernels else 0.0
    avg_step_s = step_ms / 1e3 / launches if launches else 0.0
    abytes = wl.algorithmic_bytes()
    achieved = abytes / avg_s / 1e9 if avg_s > 0 else 0.0
    roofline = None
    if avg_s > 0:  # no timed launch (e.g. a layout whose steps run no timed kernel): not measured
        roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(wl.tag),
                    "kernel": wl.kernel, "avg_kernel_us": avg_s * 1e6, "kernels_per_step": kernels / launches,
                    "timed_steps": launches, "avg_step_events_us": avg_step_s * 1e6,
                    "timing": "hipExtLaunchKernel start/stop events: each timed kernel's own dispatch begin/end "
                              "(the durations rocprofv3 --kernel-trace reports), summed per step; every "
                              f"{every}-th step of the timed region stamped (timed_steps of {args.steps})",
                    "algorithmic_bytes_per_launch": abytes, **wl.roofline_extra()}
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
        "config": wl.config(),
        "counts_verified": verified,
        "roofline": roofline,
        "cpu_baseline": None,
    }
    alg_flops = wl.algorithmic_flops() if hasattr(wl, "algorithmic_flops") else None
    if alg_flops and avg_s > 0:  # the point-polygon steps: FP64 is not their bound
        pmc_flops = pmc_traffic(wl.tag, "fp64_flops_per_launch")
        result["fp64"] = {
            "bound": "fp64", "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "executed_flops": pmc_flops,
            "achieved": (pmc_flops / avg_s / 1e12) if pmc_flops else None,
            "frac": (pmc_flops / avg_s / 1e12 / FP64_PEAK_TFLOPS) if pmc_flops else None,
            "source": "rocprofv3 SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes of the timed kernels per step (profiles/pmc_"
                      + wl.tag + ".json) / the kernels' time per step: the FP64 work actually executed",
            "reference_work_flops": alg_flops, "candidate_pairs": wl._alg_cand,
            "reference_work_rate_tflops": alg_flops / avg_s / 1e12,
            "reference_work_note": "SURVEY.md 8(d)'s count of the reference's JTS work (candidate pairs x 1850 flop) per "
                                   "second of step time -- a rate, not a roofline fraction: the cell classes decide "
                                   "most pairs without that work"}
    if args.check and world > 1 and hasattr(wl, "check_merged"):
        ok = wl.check_merged(args.warmup + args.steps - 1)
        if rank == 0 and ok is not None:
            result["merged_matches_full_window"] = ok
    if not args.no_cells_line and args.partition == "arrival":
        cells = wl.cells_partition(args.cells_steps)
        if cells is not None and rank == 0:
            result["partition_cells"] = cells
    if args.partition == "cells":
        result["config"]["parallelism"] = f"key-band{world} (north-star layout)"
    if rank == 0 and world == 1 and not args.no_e2e and args.workload == "knn":  # the C2 host path
        e2e = wl.e2e()
        if e2e is not None:
            result["e2e"] = e2e
    if rank == 0 and world == 1 and args.workload == "knn" and not args.no_pipelined:
        result["pipelined"] = wl.pipelined(nstreams=args.pipeline_streams)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = wl.cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
