"""Multi-GPU window evaluation: one process per GPU, torch.distributed over RCCL (xGMI).

Mirrors Flink's data parallelism for the windowed operators (keyBy(gridID) over task slots,
PointPointRangeQuery.java:111-116, PointPointKNNQuery.java:146-151; windowAll merge at
:188-190) the MI355X way:

* a window of N points is sharded by arrival order: rank r holds points
  [r*N/W, (r+1)*N/W) -- for single-query range/kNN this gives the identical result to cell
  sharding and keeps the distance work balanced;
* range: no collective on the data path; each rank's hits are global indices (shard base +
  local index) in ascending order, and the concatenation in rank order is the ascending
  global result.  ``gather_counts`` (one all-gather of W int64) gives each rank its output
  offset when results must land in one buffer;
* kNN: each rank computes its local top-k (k x (f64 dist, u32 idx), <= 3 KB at k = 256) on
  the device, one all-gather moves the W lists over xGMI, and every rank merges them with
  the same device kernel (geohip_knn_merge_async) -> identical results on all ranks.  This
  replaces the reference's parallelism-1 windowAll funnel.

The local engine and the merge are injectable so the orchestration is testable with the
gloo backend on CPU (tests/test_distributed_gloo.py); by default both are libgeohip.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

SENTINEL = 0xFFFFFFFF


def shard_bounds(n_total: int, world: int, rank: int):
    """Arrival-order shard [lo, hi) of rank `rank` in a window of n_total points."""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi


@dataclass
class KnnResult:
    idx: object   # global window indices, ascending (dist, idx)
    dist: object
    count: int


def knn_sharded(x_local, y_local, base: int, qx: float, qy: float, r: float, k: int, *, grid=None, ctx=None,
                group=None, local_knn: Optional[Callable] = None, merge: Optional[Callable] = None) -> KnnResult:
    """kNN of one window sharded over the process group (every rank gets the result).

    local_knn(x, y, qx, qy, r, k) -> (idx int32[k], dist f64[k]) with sentinel padding
    (idx -1 / 0xffffffff, dist all-ones bits); merge(dist[W,k], idx[W,k], k) -> same shape.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if local_knn is None:
        local_knn = _device_local_knn(ctx, grid)
    if merge is None:
        merge = _device_merge(ctx)
    li, ld = local_knn(x_local, y_local, qx, qy, r, k)
    li = li.to(torch.int64)
    valid = li >= 0
    gi = torch.where(valid, li + base, torch.full_like(li, -1)).to(torch.int32)
    gd = ld.contiguous()
    all_d = torch.empty((world, k), dtype=gd.dtype, device=gd.device)
    all_i = torch.empty((world, k), dtype=gi.dtype, device=gi.device)
    if world > 1:
        dist.all_gather_into_tensor(all_d.view(-1), gd, group=group)
        dist.all_gather_into_tensor(all_i.view(-1), gi, group=group)
    else:
        all_d[0] = gd
        all_i[0] = gi
    mi, md = merge(all_d, all_i, k)
    count = int((mi != -1).sum().item())
    return KnnResult(mi[:count], md[:count], count)


def range_sharded(x_local, y_local, base: int, qx: float, qy: float, r: float, approximate: bool = False, *,
                  grid=None, ctx=None, group=None, local_range: Optional[Callable] = None):
    """Range of one window sharded over the group: returns (global_hits_of_this_rank,
    output_offset, total) -- concatenating the ranks' hits in rank order gives the ascending
    global result; no collective touches the hit data (only W int64 counts)."""
    import torch

    if local_range is None:
        local_range = _device_local_range(ctx, grid)
    hits = local_range(x_local, y_local, qx, qy, r, approximate)
    hits = hits.to(torch.int64) + base
    offset, total = gather_counts(len(hits), hits.device, group)
    return hits, offset, total


def gather_counts(count: int, device, group=None):
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    t = torch.tensor([count], dtype=torch.int64, device=device)
    allc = torch.empty(world, dtype=torch.int64, device=device)
    if world > 1:
        dist.all_gather_into_tensor(allc, t, group=group)
    else:
        allc[0] = t[0]
    allc = allc.cpu().tolist()
    return sum(allc[:rank]), sum(allc)


# ------------------------------------------------------------------ default device engine --
def _device_local_knn(ctx, grid):
    import torch

    def f(x, y, qx, qy, r, k):
        oi = torch.empty(k, dtype=torch.int32, device=x.device)
        od = torch.empty(k, dtype=torch.float64, device=x.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=x.device)
        ctx.knn_pp_async(grid, x, y, qx, qy, r, k, oi, od, cnt)
        return oi, od

    return f


def _device_merge(ctx):
    import torch

    def f(all_d, all_i, k):
        w = all_d.shape[0]
        oi = torch.empty(k, dtype=torch.int32, device=all_d.device)
        od = torch.empty(k, dtype=torch.float64, device=all_d.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=all_d.device)
        ctx.knn_merge_async(all_d, all_i, w, k, k, oi, od, cnt)
        return oi, od

    return f


def _device_local_range(ctx, grid):
    def f(x, y, qx, qy, r, approximate):
        return ctx.range_pp(grid, x, y, qx, qy, r, approximate)

    return f
