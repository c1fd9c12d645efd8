"""Incremental sliding windows: pane reuse.

A sliding window of size S and slide D (S a multiple of D, QueryConfiguration.java:5-56) is the
union of P = S / D consecutive panes of D.  The reference's incremental range query
(PointPointRangeQuery.queryIncremental, PointPointRangeQuery.java:144-245) evaluates only the
newest slide of each window (``point.timeStampMillisec >= timeWindow.getEnd() - slideStep``,
:215-216) and re-emits the outputs it kept in ListState while their timestamp is still inside the
window (``>= timeWindow.getStart() + slideStep``, :201-208).  Here every pane is evaluated once
on the GPU when it arrives; a window's result is assembled from the last P panes' results:

* range: the panes' hit lists, each computed once by geohip_range_pp_pane with the pane's stream
  position as the index base -- stream positions, ascending; concatenated pane after pane they
  are the window's hits (the range predicate is per point) with no pass over them per window
  (window-local index = stream position - the window's first position);
* kNN: the k smallest of the panes' top-k lists (geohip_knn_merge_async on the device) -- the
  top-k of a union is the top-k of the union of top-ks, so the same (dist, idx) list as a full
  evaluation of the window.

Each point is evaluated once instead of P times (P = 2 for the reference's 10 s / 5 s windows).
The first windows of a stream hold fewer than P panes, as Flink's sliding windows that start
before the first element do.  Panes are device-resident (x, y float64 tensors) or host arrays.
"""
from __future__ import annotations

from collections import deque

from . import _abi


def panes_per_window(window_size: int, slide_step: int) -> int:
    if slide_step <= 0 or window_size <= 0 or window_size % slide_step:
        raise _abi.GeohipArgumentError("incremental windows need window_size a positive multiple of slide_step")
    return window_size // slide_step


class IncrementalRange:
    """Point-point range over sliding windows with pane reuse: each pane's hits are computed once,
    by geohip_range_pp_pane with the pane's stream position as the index base, so they are stream
    positions and serve every window that holds the pane unchanged -- no per-window pass over
    them (the round-4 form added each pane's window offset with a torch pass per window)."""

    def __init__(self, ctx: _abi.Context, grid: _abi.Grid, qx: float, qy: float, r: float,
                 approximate: bool = False, panes: int = 2, start: int = 0):
        self.ctx, self.grid, self.q, self.r, self.approx = ctx, grid, (qx, qy), r, approximate
        self.panes = deque(maxlen=panes)  # (first stream position, pane size, hits as stream positions)
        self.pos = start & 0xFFFFFFFF  # stream position of the next pane's first point (mod 2^32)

    def push(self, x, y):
        """Evaluate the new pane; returns the window's hits (window())."""
        hits = self.ctx.range_pp(self.grid, x, y, self.q[0], self.q[1], self.r, self.approx, point_base=self.pos)
        self.panes.append((self.pos, len(x), hits))
        self.pos = (self.pos + len(x)) & 0xFFFFFFFF
        return self.window()

    @property
    def window_start(self) -> int:
        """Stream position of the window's first point (its local index 0)."""
        return self.panes[0][0] if self.panes else self.pos

    def window(self):
        """The window's hits pane by pane: a list of the panes' hit arrays, nothing recomputed or
        copied.  Each holds stream positions mod 2^32 as uint32 bit patterns (ascending within a
        pane until the stream position wraps, in the ctx's default order; a set in no promised
        order under GEOHIP_ORDER_ANY); a device pane's array is an int32 tensor, so
        positions from 2^31 on read negative -- mask with & 0xFFFFFFFF, or use window_local()."""
        return [hits for _, _, hits in self.panes]

    def window_local(self):
        """The window's hits as window-local indices in one int64 array (a convenience: one pass
        over the hits, (stream position - window_start) mod 2^32)."""
        import numpy as np
        parts, s0 = self.window(), self.window_start
        if parts and _abi._is_device(parts[0]):
            import torch
            return (torch.cat([h.to(torch.int64) for h in parts]) - s0) & 0xFFFFFFFF
        return (np.concatenate([np.zeros(0, np.int64)] + [np.asarray(h).astype(np.int64) for h in parts]) - s0) & 0xFFFFFFFF


class IncrementalPPolyRange:
    """Point-polygon range (many query polygons) over sliding windows with pane reuse: each pane's
    (polygon, point) pairs are computed once, by geohip_range_ppoly_pane with the pane's stream
    position as the point-index base, so the pairs carry stream positions and serve every window
    that holds the pane unchanged -- no per-window pass over them (PointPolygonRangeQuery's
    per-point predicate, PointPolygonRangeQuery.java:104-124, makes pane results independent).
    A window's local point index = stream position - ``window_start`` (mod 2^32).  The polygon
    plan is cached by the context, so panes after the first skip planning and upload."""

    def __init__(self, ctx: _abi.Context, grid: _abi.Grid, ring_off, vx, vy, r: float, approximate: bool = False,
                 panes: int = 2, out_cap: int = 0):
        self.ctx, self.grid, self.r, self.approx = ctx, grid, r, approximate
        self.rings = (ring_off, vx, vy)
        self.panes = deque(maxlen=panes)  # (first stream position, pane size, pairs [m, 2] (polygon, position))
        self.out_cap = out_cap
        self.pos = 0  # stream position of the next pane's first point

    def push(self, x, y, out=None, count=None):
        """Evaluate the new pane; returns the window's pairs (window()).  With ``count`` (one int64
        device tensor) and ``out`` ([cap, 2] int32, device): enqueue-only
        (geohip_range_ppoly_pane_async) -- the pane's entry is (out, count), the pair count stays on
        the device (faults at ctx.sync())."""
        if count is not None:
            self.ctx.range_ppoly_async(self.grid, x, y, *self.rings, self.r, self.approx, out, count,
                                       point_base=self.pos)
            pairs = (out, count)
        else:
            pairs = self.ctx.range_ppoly(self.grid, x, y, *self.rings, self.r, self.approx, out=out,
                                         point_base=self.pos)
        self.panes.append((self.pos, len(x), pairs))
        self.pos = (self.pos + len(x)) & 0xFFFFFFFF
        return self.window()

    @property
    def window_start(self) -> int:
        """Stream position of the window's first point (its local index 0)."""
        return self.panes[0][0] if self.panes else self.pos

    def window(self):
        """Pairs of the window (polygon, stream position), pane by pane (a list: the caller
        concatenates if it needs one array; an enqueue-only pane's entry is its (out, count))."""
        return [pairs for _, _, pairs in self.panes]


class IncrementalKNN:
    """Point-point kNN over sliding windows with pane reuse (device tensors).  Each pane's top-k
    (k indices, -1 padded, and distances) lands in a ring of P slots; a window is one
    geohip_knn_merge_panes_async launch over the ring (the panes' slots oldest first, each
    rebased by its offset in the window) -- no torch kernels between the pass and the merge."""

    def __init__(self, ctx: _abi.Context, grid: _abi.Grid, qx: float, qy: float, r: float, k: int, panes: int = 2):
        if not 1 <= int(panes) <= 16:  # one geohip_knn_merge_panes_async launch merges at most 16 lists
            raise _abi.GeohipArgumentError(f"IncrementalKNN merges 1..16 panes per window, got {panes}")
        self.ctx, self.grid, self.q, self.r, self.k, self.p = ctx, grid, (qx, qy), r, int(k), int(panes)
        self.sizes = deque(maxlen=self.p)  # sizes of the panes in the ring, oldest first
        self.count = 0                     # panes pushed so far
        self._dev = None

    def _alloc(self, dev):
        import torch
        k, p = self.k, self.p
        self.ring_i = torch.full((p, k), -1, dtype=torch.int32, device=dev)
        self.ring_d = torch.empty((p, k), dtype=torch.float64, device=dev)
        self.cnt = torch.zeros(2, dtype=torch.int32, device=dev)
        self.mi = torch.empty(k, dtype=torch.int32, device=dev)
        self.md = torch.empty(k, dtype=torch.float64, device=dev)
        self._dev = dev

    def push(self, x, y, sync: bool = True):
        """Evaluate the new pane and merge the window (on torch's current stream, which the ctx
        follows).  sync=True: (idx, dist) trimmed to the count (one host sync); sync=False: the
        k-long device outputs (idx -1 padded), no sync."""
        if self._dev != x.device:
            self._alloc(x.device)
        slot = self.count % self.p
        self.ctx.knn_pp_async(self.grid, x, y, self.q[0], self.q[1], self.r, self.k, self.ring_i[slot],
                              self.ring_d[slot], self.cnt[0:1])
        self.count += 1
        self.sizes.append(len(x))
        n = len(self.sizes)
        slots = [(self.count - n + j) % self.p for j in range(n)]  # oldest first
        offs = [0]
        for size in list(self.sizes)[:-1]:
            offs.append(offs[-1] + size)
        self.ctx.knn_merge_panes_async(self.ring_d, self.ring_i, slots, offs, self.k, self.mi, self.md, self.cnt[1:2])
        if not sync:
            return self.mi, self.md
        m = int(self.cnt[1].item())
        return self.mi[:m].clone(), self.md[:m].clone()


def run_incremental_range(ctx, grid, panes, qx, qy, r, approximate=False, window_size=10, slide_step=5):
    """Generator over windows: for each pane (x, y) of the stream, the result of the window that
    ends with it as window-local indices (PointPointRangeQuery.queryIncremental semantics)."""
    inc = IncrementalRange(ctx, grid, qx, qy, r, approximate, panes_per_window(window_size, slide_step))
    for x, y in panes:
        inc.push(x, y)
        yield inc.window_local()
