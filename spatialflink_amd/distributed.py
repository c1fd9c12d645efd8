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

* join (PointPointJoinQuery.java:113-172): the query window is small (C3: 10k x 16 B) and is
  present on every rank.  ``partition="arrival"``: data stays where it arrived and every rank
  joins its shard against all queries (no data exchange; the query block replication of
  JoinQuery.getReplicatedPointQueryStream degenerates to "every rank").  ``partition="cells"``
  mirrors keyBy(gridID) with halo replication: rank s owns the x-major key band of grid columns
  [ceil(s n / W), ceil((s+1) n / W)), data points move to their owner with one all-to-all, and
  each rank keeps only the queries whose Nbr block (cell +- Lc columns, one spare column) meets
  its band.  Both give disjoint per-rank pair sets whose union is the window's result;
* point-polygon range: the polygons (C4: 1k x 51 vertices) are on every rank, points stay.

The local engine and the merge are injectable so the orchestration is testable with the
gloo backend on CPU (tests/test_distributed_gloo.py); by default both are libgeohip.
"""
from __future__ import annotations

import math
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

    world, _ = _world_rank(group)
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
        all_gather_into(all_d.view(-1), gd, group)
        all_gather_into(all_i.view(-1), gi, group)
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


def _java_cell(v, mn: float, l: float):
    """(int)Math.floor((v - mn) / l) per element (HelperClass.java:109-110): fp64 as the
    reference evaluates it, NaN -> 0, saturating int cast."""
    import torch

    t = torch.floor((v - mn) / l)
    t = torch.where(torch.isnan(t), torch.zeros_like(t), t)
    return t.clamp(-2147483648.0, 2147483647.0).to(torch.int64)


def query_block_width(grid_data, qx: float, qy: float, r: float, world: int) -> int:
    """Column block width of the single-query key layout (geohip_band_pack_query_async): at least
    8 blocks per rank across the query's 2 Lc + 1 candidate columns (Lc =
    UniformGrid.getCandidateNeighboringLayers, UniformGrid.java:440-444)."""
    from . import _abi
    try:
        lc = max(_abi.plan_point(grid_data, qx, qy, r)[3], 0)
    except _abi.GeohipError:
        lc = 0
    return max(1, min((2 * lc + 1) // (8 * world), 1 << 20))


def torch_band_pack(grid_data, keep=None, bw: int = 0):
    """band_pack written with torch ops (CPU orchestration tests; the product engine is
    geohip_band_pack_async): same owners, same arrival order inside each owner group.
    keep(x, y) -> bool mask: an extra filter (the query's G u C cells for band_pack_query).
    bw > 0: block-cyclic owners (cx // bw) % world (the single-query layout)."""
    import torch

    def f(x, y, base, nb, world):
        cx = _java_cell(x, grid_data.min_x, grid_data.cell_len)
        cy = _java_cell(y, grid_data.min_y, grid_data.cell_len)
        valid = (cx >= 0) & (cx < nb) & (cy >= 0) & (cy < nb)  # other keys match no Nbr block
        if keep is not None:
            valid = valid & keep(x, y)
        gidx = torch.arange(len(x), dtype=torch.int64, device=x.device) + base
        owner = (cx // bw) % world if bw > 0 else (cx * world) // nb
        sel = torch.nonzero(valid).flatten()
        order = sel[torch.argsort(owner[sel], stable=True)]
        counts = torch.bincount(owner[order], minlength=world).to(torch.int64)
        return x[order], y[order], gidx[order], counts

    return f


def torch_band_pack_query(grid_data, qx: float, qy: float, r: float):
    """band_pack_query with torch ops (CPU tests): the query's G u C membership from the host
    planner's exact boxes (geohip_debug_classify), then torch_band_pack."""
    import torch

    from . import _abi

    def keep(x, y):
        c = _abi.debug_classify(grid_data, qx, qy, r, x.cpu().numpy(), y.cpu().numpy())
        return torch.from_numpy((c & 4) != 0).to(x.device)

    def f(x, y, base, nb, world):
        return torch_band_pack(grid_data, keep, query_block_width(grid_data, qx, qy, r, world))(x, y, base, nb, world)

    return f


def _exchange_records(px, py, pg, send_counts, group):
    """The key-band shuffle: counts exchanged on the device and read once (the only host round
    trip -- all_to_all needs the split sizes), then x, y and the window index as one [m, 3] fp64
    record array in a single all_to_all.  Returns the owner's (x, y, window idx)."""
    import torch

    if _world_rank(group)[0] == 1:  # one owner: the packed points stay (no collective)
        m = int(send_counts.sum().item())
        return px[:m], py[:m], pg[:m]
    recv_counts = torch.empty_like(send_counts)
    all_to_all(recv_counts, send_counts, group=group)
    both = torch.stack([send_counts, recv_counts]).cpu().tolist()
    sc, rc = both[0], both[1]
    nrecv, nsend = sum(rc), sum(sc)
    rec = torch.stack([px[:nsend], py[:nsend], pg[:nsend].view(torch.float64)], dim=1).contiguous()
    got = torch.empty((nrecv, 3), dtype=torch.float64, device=rec.device)
    all_to_all(got, rec, rc, sc, group)
    return got[:, 0].contiguous(), got[:, 1].contiguous(), got[:, 2].contiguous().view(torch.int64)


class CellsBuffers:
    """Preallocated device rows of knn_range_cells' enqueue-only form (one set per window in
    flight): the owner's top-k and range hits with their device counts, the all-gathered lists,
    the merged top-k and the per-rank hit counts."""

    def __init__(self, k: int, hit_cap: int, world: int, device, with_range: bool = True):
        import torch
        i32, i64, f64 = torch.int32, torch.int64, torch.float64
        self.k, self.cap, self.with_range = k, hit_cap, with_range
        self.ki = torch.empty(k, dtype=i32, device=device)
        self.kd = torch.empty(k, dtype=f64, device=device)
        self.kc = torch.zeros(1, dtype=i32, device=device)
        self.hits = torch.empty(max(hit_cap, 1), dtype=i32, device=device)
        self.hc = torch.zeros(1, dtype=i64, device=device)
        self.all_d = torch.empty((world, k), dtype=f64, device=device)
        self.all_i = torch.empty((world, k), dtype=i32, device=device)
        self.mi = torch.empty(k, dtype=i32, device=device)
        self.md = torch.empty(k, dtype=f64, device=device)
        self.mc = torch.zeros(1, dtype=i32, device=device)
        self.counts = torch.zeros(world, dtype=i64, device=device)


@dataclass
class CellsStep:
    """knn_range_cells' enqueue-only result: device tensors, nothing read back yet.  idx / dist:
    the merged top-k (k entries, -1 / sentinel padded), count: its int32 device count; hits: this
    rank's hit buffer (local indices, hit_count of them), mapped to window indices by base or by
    rg; counts: every rank's hit count (device).  result() reads it back as the synchronous form
    returns it."""
    idx: object
    dist: object
    count: object
    hits: object
    hit_count: object
    base: int
    rg: object
    counts: object
    rank: int
    nrecv: int

    def totals(self):
        """(this rank's pair count, its output offset, the total) -- the counts alone, no pairs read."""
        m = int(self.count.item())
        allc = self.counts.cpu().tolist()
        return m, sum(allc[:self.rank]), sum(allc)

    def result(self):
        import torch
        m = int(self.count.item())
        h = int(self.hit_count.item())
        if h > len(self.hits):
            from ._abi import GeohipCapacityError
            raise GeohipCapacityError(f"range hits {h} exceed the hit buffer ({len(self.hits)})")
        lh = self.hits[:h].to(torch.int64)
        hits = lh + self.base if self.rg is None else (self.rg[lh] if h else lh)
        allc = self.counts.cpu().tolist()
        return (KnnResult(self.idx[:m], self.dist[:m], m), (hits, sum(allc[:self.rank]), sum(allc)), self.nrecv)


def _knn_range_cells_enqueue(x_local, y_local, base, qx, qy, r, k, approximate, grid, ctx, group, band_pack,
                             bufs: CellsBuffers) -> CellsStep:
    """knn_range_cells with the device engine into preallocated rows and no host round trip
    except the exchange's split sizes (world > 1; all_to_all takes them on the host)."""
    import torch

    world, rank = _world_rank(group)
    b = bufs
    if world == 1 and band_pack is None:  # one owner: the filter is fused into the kNN pass
        rx, ry, rg, nrecv = x_local, y_local, None, len(x_local)
    else:
        if band_pack is None:
            def band_pack(x, y, bb, nb_, w):
                return ctx.band_pack_query_async(grid, nb_, w, qx, qy, r, x, y, bb)
        px, py, pg, send_counts = band_pack(x_local, y_local, base, int(grid.n), world)
        rx, ry, rg = _exchange_records(px, py, pg, send_counts, group)
        nrecv = len(rx)
    if b.with_range and nrecv > b.cap:  # skewed shuffle: more points than the rows were sized for
        b.hits = torch.empty(nrecv, dtype=torch.int32, device=b.hits.device)
        b.cap = nrecv  # hits <= points received, so the call cannot overflow
    if b.with_range:
        ctx.knn_range_pp_async(grid, rx, ry, qx, qy, r, k, approximate, b.ki, b.kd, b.kc, b.hits, b.cap, b.hc)
    else:
        ctx.knn_pp_async(grid, rx, ry, qx, qy, r, k, b.ki, b.kd, b.kc)
        b.hc.zero_()
    if rg is None and base == 0:
        gi = b.ki  # local positions are window indices: no pass
    else:
        li = b.ki.to(torch.int64)
        if rg is None:
            gi = torch.where(li >= 0, li + base, li).to(torch.int32)
        else:
            gi = torch.where(li >= 0, rg[li.clamp(min=0, max=max(nrecv - 1, 0))] if nrecv else li, li).to(torch.int32)
    if world == 1:  # one list: it is the merged result, its hit count the only count
        return CellsStep(gi, b.kd, b.kc, b.hits, b.hc, base, rg, b.hc, rank, nrecv)
    else:
        all_gather_into(b.all_d.view(-1), b.kd, group)
        all_gather_into(b.all_i.view(-1), gi, group)
        ctx.knn_merge_async(b.all_d, b.all_i, world, k, k, b.mi, b.md, b.mc)
        idx, dist, count = b.mi, b.md, b.mc
        all_gather_into(b.counts, b.hc, group)
    return CellsStep(idx, dist, count, b.hits, b.hc, base, rg, b.counts, rank, nrecv)


def knn_range_cells(x_local, y_local, base: int, qx: float, qy: float, r: float, k: int, approximate: bool = False,
                    *, grid, ctx=None, group=None, band_pack: Optional[Callable] = None,
                    local: Optional[Callable] = None, merge: Optional[Callable] = None,
                    bufs: Optional[CellsBuffers] = None):
    """kNN (k) and range (r) of one point query over a window partitioned by grid-cell key band
    (the north-star layout, mirroring the reference's filter + keyBy(gridID),
    PointPointKNNQuery.java:137-151 / PointPointRangeQuery.java:102-116): every rank packs the
    points of its arrival shard that lie in the query's G u C cells by owner band
    (geohip_band_pack_query_async), one all-to-all moves them to their owner, each owner
    evaluates its band, the top-k lists meet in one all-gather + merge (the windowAll funnel),
    the range hits stay with their owner as window indices.
    local(x, y, qx, qy, r, k, approximate) -> (idx int32 [k] sentinel -1, dist f64 [k], hits int
    [m]), local indices.  Returns (KnnResult, (hits int64 window idx ascending, offset, total),
    points this rank evaluated: the band-packed candidates it received, or at world 1 with the
    default packing its whole shard -- one owner holds every band, the shuffle is the identity and
    the kNN pass applies the G u C filter itself).
    bufs (device engine only: local and merge not given): the enqueue-only form into those
    preallocated rows -- returns a CellsStep (device tensors; .result() reads it back)."""
    import torch

    if bufs is not None:
        if local is not None or merge is not None:
            raise ValueError("knn_range_cells: bufs needs the device engine (no local / merge)")
        return _knn_range_cells_enqueue(x_local, y_local, base, qx, qy, r, k, approximate, grid, ctx, group,
                                        band_pack, bufs)
    world, _ = _world_rank(group)
    nb = int(grid.n)
    shortcut = world == 1 and band_pack is None
    if band_pack is None:
        def band_pack(x, y, b, nb_, w):
            return ctx.band_pack_query_async(grid, nb_, w, qx, qy, r, x, y, b)
    if local is None:
        local = _device_local_knn_range(ctx, grid)
    if merge is None:
        merge = _device_merge(ctx)
    if shortcut:
        # one owner holds every key band: the filter + keyBy shuffle is the identity (the local
        # kernel applies the G u C filter itself), so the shard is evaluated where it lies
        rx, ry = x_local, y_local
        rg = None
        nrecv = len(x_local)
    else:
        px, py, pg, send_counts = band_pack(x_local, y_local, base, nb, world)
        rx, ry, rg = _exchange_records(px, py, pg, send_counts, group)
        nrecv = len(rx)
    li, ld, lh = local(rx, ry, qx, qy, r, k, approximate)
    li64 = li.to(torch.int64)
    if rg is None:
        gi = torch.where(li64 >= 0, li64 + base, torch.full_like(li64, -1)).to(torch.int32)
    else:
        gi = torch.where(li64 >= 0, rg[li64.clamp(min=0)] if nrecv else li64, torch.full_like(li64, -1)).to(torch.int32)
    all_d = torch.empty((world, k), dtype=ld.dtype, device=ld.device)
    all_i = torch.empty((world, k), dtype=torch.int32, device=ld.device)
    if world > 1:
        all_gather_into(all_d.view(-1), ld.contiguous(), group)
        all_gather_into(all_i.view(-1), gi, group)
    else:
        all_d[0] = ld
        all_i[0] = gi
    mi, md = merge(all_d, all_i, k)
    count = int((mi != -1).sum().item())
    if rg is None:
        hits = lh.to(torch.int64) + base
    else:
        hits = rg[lh.to(torch.int64)] if len(lh) else torch.zeros(0, dtype=torch.int64, device=ld.device)
    offset, total = gather_counts(len(hits), hits.device, group)
    return KnnResult(mi[:count], md[:count], count), (hits, offset, total), nrecv


def key_band(world: int, rank: int, nb: int):
    """Grid columns [lo, hi) owned by `rank` when column cx belongs to rank cx * world // nb."""
    return (rank * nb + world - 1) // world, ((rank + 1) * nb + world - 1) // world


def join_sharded(dx_local, dy_local, dbase: int, qx, qy, r: float, approximate: bool = False, *, grid_data,
                 grid_query, ctx=None, group=None, partition: str = "arrival", local_join: Optional[Callable] = None,
                 band_pack: Optional[Callable] = None):
    """Point-point join of one window over the group.  dx/dy_local: this rank's data shard
    (window indices dbase + local position); qx/qy: the whole query window (every rank).
    Returns (pairs int64 [m, 2] = (data window idx, query idx) of this rank, output offset,
    total pairs); the per-rank pair sets are disjoint and their union is the window's join.
    partition="cells": band_pack(x, y, base, nb, world) -> (x, y, window idx, counts[world])
    groups the shard's valid-key points by owner (default: geohip_band_pack_async)."""
    import torch
    import torch.distributed as dist

    if local_join is None:
        local_join = _device_local_join(ctx, grid_data, grid_query)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if partition == "arrival" or world == 1:
        pairs = local_join(dx_local, dy_local, qx, qy, r, approximate).to(torch.int64)
        pairs[:, 0] += dbase
    elif partition == "cells":
        nb = int(grid_query.n)
        if band_pack is None:
            band_pack = _device_band_pack(ctx, grid_data)
        px, py, pg, send_counts = band_pack(dx_local, dy_local, dbase, nb, world)
        rx, ry, rg = _exchange_records(px, py, pg, send_counts, group)
        lo, hi = key_band(world, rank, nb)
        lq = float(grid_query.cell_len)
        qcx = _java_cell(qx, grid_query.min_x, lq)
        lc = math.ceil(r / lq) if r == r and abs(r / lq) < 2.0 ** 31 else nb
        if r == 0 or lc >= nb:  # every cell (UniformGrid.java:264-266) or wider than the grid
            keep = torch.ones(len(qx), dtype=torch.bool, device=qx.device)
        else:
            odd = (qcx < -9999) | (qcx > 99999)  # key round trips of getIntCellIndices: keep
            keep = odd | ((qcx - lc - 1 <= hi - 1) & (qcx + lc + 1 >= lo))
        kq = torch.nonzero(keep).flatten()
        pairs = local_join(rx, ry, qx[kq], qy[kq], r, approximate).to(torch.int64)
        if len(pairs):
            pairs = torch.stack([rg[pairs[:, 0]], kq.to(torch.int64)[pairs[:, 1]]], dim=1)
    else:
        raise ValueError(f"unknown partition {partition!r}")
    offset, total = gather_counts(len(pairs), pairs.device, group)
    return pairs, offset, total


@dataclass
class JoinCellsStep:
    """join_cells_enqueue's result, nothing read back: out[:count] holds this rank's pairs as
    (index into its received records, query index); rg maps a record to its window index;
    counts holds every rank's pair count (device).  result() reads it back as join_sharded
    returns it: (pairs int64 [m, 2] = (data window idx, query idx), output offset, total)."""
    out: object
    count: object
    rg: object
    counts: object
    rank: int

    def totals(self):
        """(this rank's pair count, its output offset, the total) -- the counts alone, no pairs read."""
        m = int(self.count.item())
        allc = self.counts.cpu().tolist()
        return m, sum(allc[:self.rank]), sum(allc)

    def result(self):
        import torch
        m = int(self.count.item())
        if m > self.out.shape[0]:
            from ._abi import GeohipCapacityError
            raise GeohipCapacityError(f"join pairs {m} exceed the pair buffer ({self.out.shape[0]})")
        p = self.out[:m].to(torch.int64)
        if m:
            p = torch.stack([self.rg[p[:, 0]], p[:, 1]], dim=1)
        allc = self.counts.cpu().tolist()
        return p, sum(allc[:self.rank]), sum(allc)


def join_cells_enqueue(dx_local, dy_local, dbase: int, qx, qy, r: float, approximate: bool = False, *, grid_data,
                       grid_query, ctx, out, count, counts, group=None):
    """The key-band join of one window (PointPointJoinQuery.java:137-150) with no host round
    trip but the shuffle's split sizes: data points packed by owner band (geohip_band_pack_async)
    and moved in one all-to-all; the owner joins its band against the whole query window with
    geohip_join_pp_async into the preallocated out ([cap, 2] int32) / count (int64[1]), and the
    ranks' counts meet in one device all-gather into counts (int64[world]).  Every rank takes
    every query: a query whose Nbr block misses a rank's band finds no record there, so the pair
    sets stay disjoint and their union is the window's join; the query window is small (10k
    points in C3), and selecting each band's halo queries on the host cost a synchronisation per
    window."""
    world, rank = _world_rank(group)
    nb = int(grid_query.n)
    px, py, pg, send_counts = ctx.band_pack_async(grid_data, nb, world, dx_local, dy_local, dbase)
    rx, ry, rg = _exchange_records(px, py, pg, send_counts, group)
    ctx.join_pp_async(grid_data, grid_query, rx, ry, qx, qy, r, approximate, out, count)
    if world > 1:
        all_gather_into(counts, count, group)
    else:
        counts.copy_(count)
    return JoinCellsStep(out, count, rg, counts, rank)


def _poly_kw(poly_rings):
    return {} if poly_rings is None else {"poly_rings": poly_rings}


def ppoly_sharded(x_local, y_local, base: int, ring_off, vx, vy, r: float, approximate: bool = False, *, grid=None,
                  ctx=None, group=None, local_ppoly: Optional[Callable] = None, poly_rings=None):
    """Point-polygon range of one window over the group (polygons on every rank, points by
    arrival): returns (pairs int64 [m, 2] = (polygon, point window idx), offset, total).
    poly_rings: rings per polygon (shell + holes), as for Context.range_ppoly."""
    import torch

    if local_ppoly is None:
        local_ppoly = _device_local_ppoly(ctx, grid)
    pairs = local_ppoly(x_local, y_local, ring_off, vx, vy, r, approximate, **_poly_kw(poly_rings)).to(torch.int64)
    if len(pairs):
        pairs[:, 1] += base
    offset, total = gather_counts(len(pairs), pairs.device, group)
    return pairs, offset, total


def join_ppoly_sharded(x_local, y_local, base: int, ring_off, vx, vy, r: float, approximate: bool = False, *,
                       grid_points=None, grid_query=None, ctx=None, group=None,
                       local_join: Optional[Callable] = None, poly_rings=None):
    """Point-polygon join of one window over the group (PointPolygonJoinQuery.java:162-201):
    the polygon stream on every rank, points by arrival; returns (pairs int64 [m, 2] =
    (point window idx, polygon), offset, total).  Per-rank pair sets are disjoint (each point
    lives on one rank) and their union is the window's join; only W counts are exchanged."""
    import torch

    if local_join is None:
        local_join = _device_local_join_ppoly(ctx, grid_points, grid_query)
    pairs = local_join(x_local, y_local, ring_off, vx, vy, r, approximate, **_poly_kw(poly_rings)).to(torch.int64)
    if len(pairs):
        pairs[:, 0] += base
    offset, total = gather_counts(len(pairs), pairs.device, group)
    return pairs, offset, total


def knn_ppoly_sharded(x_local, y_local, base: int, vx, vy, r: float, k: int, approximate: bool = False, *,
                      grid=None, ctx=None, group=None, local_knn: Optional[Callable] = None,
                      merge: Optional[Callable] = None, ring_off=None) -> KnnResult:
    """Point-polygon kNN of one window over the group (PointPolygonKNNQuery.java:162-236 with the
    windowAll merge of KNNQuery.java:204-272 replaced by one all-gather of each rank's top-k):
    local_knn(x, y, vx, vy, r, k, approximate) -> (idx int32[k], dist f64[k]) padded with
    idx -1 / dist all-ones bits; every rank returns the same (idx, dist), ascending."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if local_knn is None:
        local_knn = _device_local_knn_ppoly(ctx, grid)
    if merge is None:
        merge = _device_merge(ctx)
    li, ld = local_knn(x_local, y_local, vx, vy, r, k, approximate, **({} if ring_off is None else {"ring_off": ring_off}))
    li = li.to(torch.int64)
    gi = torch.where(li >= 0, li + base, torch.full_like(li, -1)).to(torch.int32)
    gd = ld.contiguous()
    all_d = torch.empty((world, k), dtype=gd.dtype, device=gd.device)
    all_i = torch.empty((world, k), dtype=gi.dtype, device=gi.device)
    if world > 1:
        all_gather_into(all_d.view(-1), gd, group)
        all_gather_into(all_i.view(-1), gi, group)
    else:
        all_d[0] = gd
        all_i[0] = gi
    mi, md = merge(all_d, all_i, k)
    count = int((mi != -1).sum().item())
    return KnnResult(mi[:count], md[:count], count)


def _world_rank(group=None):
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized():
        return 1, 0  # a single process: the window is one shard
    return dist.get_world_size(group), dist.get_rank(group)


def gather_counts(count: int, device, group=None):
    import torch

    world, rank = _world_rank(group)
    t = torch.tensor([count], dtype=torch.int64, device=device)
    allc = torch.empty(world, dtype=torch.int64, device=device)
    if world > 1:
        all_gather_into(allc, t, group)
    else:
        allc[0] = t[0]
    allc = allc.cpu().tolist()
    return sum(allc[:rank]), sum(allc)


def _host_staged(t, group) -> bool:
    """gloo moves CPU tensors only: device tensors are staged through host memory (the
    multi-process-on-one-GPU test rig); RCCL (backend "nccl") takes them as they are."""
    import torch.distributed as dist

    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_gather_into(out, inp, group=None):
    """dist.all_gather_into_tensor(out, inp), staged through host for gloo."""
    import torch.distributed as dist

    if _host_staged(inp, group):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def all_to_all(out, inp, out_splits=None, in_splits=None, group=None):
    """dist.all_to_all_single, staged through host for gloo."""
    import torch.distributed as dist

    if _host_staged(inp, group):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


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


def _device_band_pack(ctx, grid_data):
    def f(x, y, base, nb, world):
        return ctx.band_pack_async(grid_data, nb, world, x, y, base)

    return f


def _device_local_join(ctx, grid_data, grid_query):
    def f(x, y, qx, qy, r, approximate):
        return ctx.join_pp(grid_data, grid_query, x, y, qx, qy, r, approximate).reshape(-1, 2)

    return f


def _device_local_ppoly(ctx, grid):
    def f(x, y, ring_off, vx, vy, r, approximate, poly_rings=None):
        return ctx.range_ppoly(grid, x, y, ring_off, vx, vy, r, approximate, poly_rings=poly_rings).reshape(-1, 2)

    return f


def _device_local_join_ppoly(ctx, grid_points, grid_query):
    def f(x, y, ring_off, vx, vy, r, approximate, poly_rings=None):
        return ctx.join_ppoly(grid_points, grid_query, x, y, ring_off, vx, vy, r, approximate,
                              poly_rings=poly_rings).reshape(-1, 2)

    return f


def _device_local_knn_ppoly(ctx, grid):
    import torch

    def f(x, y, vx, vy, r, k, approximate, ring_off=None):
        ii, dd = ctx.knn_ppoly(grid, x, y, vx, vy, r, k, approximate, ring_off=ring_off)
        oi = torch.full((k,), -1, dtype=torch.int32, device=x.device)
        od = torch.full((k,), -1, dtype=torch.int64, device=x.device).view(torch.float64)  # all-ones bits
        oi[:len(ii)] = ii
        od[:len(dd)] = dd
        return oi, od

    return f


def _device_local_knn_range(ctx, grid):
    import torch

    def f(x, y, qx, qy, r, k, approximate):
        (ki, kd), ro = ctx.knn_range_pp(grid, x, y, qx, qy, r, k, approximate)
        oi = torch.full((k,), -1, dtype=torch.int32, device=x.device)
        od = torch.full((k,), -1, dtype=torch.int64, device=x.device).view(torch.float64)  # all-ones bits
        oi[:len(ki)] = ki
        od[:len(kd)] = kd
        return oi, od, ro

    return f


def _device_local_range(ctx, grid):
    def f(x, y, qx, qy, r, approximate):
        return ctx.range_pp(grid, x, y, qx, qy, r, approximate)

    return f
