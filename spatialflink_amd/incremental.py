"""Incremental sliding windows: pane reuse.

A sliding window of size S and slide D (S a multiple of D, QueryConfiguration.java:5-56) is the
union of P = S / D consecutive panes of D.  The reference's incremental range query
(PointPointRangeQuery.queryIncremental, PointPointRangeQuery.java:144-245) evaluates only the
newest slide of each window (``point.timeStampMillisec >= timeWindow.getEnd() - slideStep``,
:215-216) and re-emits the outputs it kept in ListState while their timestamp is still inside the
window (``>= timeWindow.getStart() + slideStep``, :201-208).  Here every pane is evaluated once
on the GPU when it arrives; a window's result is assembled from the last P panes' results:

* range: the concatenation of the panes' hit lists, each offset by the pane's position in the
  window -- the window-local indices a full evaluation of the window returns (the range
  predicate is per point, so it is the same set, and ascending);
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
    """Point-point range over sliding windows with pane reuse."""

    def __init__(self, ctx: _abi.Context, grid: _abi.Grid, qx: float, qy: float, r: float,
                 approximate: bool = False, panes: int = 2):
        self.ctx, self.grid, self.q, self.r, self.approx = ctx, grid, (qx, qy), r, approximate
        self.panes = deque(maxlen=panes)  # (pane size, hits of the pane, pane-local indices)

    def push(self, x, y):
        """Evaluate the new pane; returns the window result (window-local indices, ascending)."""
        hits = self.ctx.range_pp(self.grid, x, y, self.q[0], self.q[1], self.r, self.approx)
        self.panes.append((len(x), hits))
        return self.window()

    def window(self):
        import numpy as np
        offs = np.cumsum([0] + [size for size, _ in self.panes])
        if self.panes and _abi._is_device(self.panes[0][1]):
            import torch
            return torch.cat([hits.to(torch.int64) + int(o) for (_, hits), o in zip(self.panes, offs)])
        return np.concatenate([np.zeros(0, np.int64)] +
                              [hits.astype(np.int64) + o for (_, hits), o in zip(self.panes, offs)])


class IncrementalKNN:
    """Point-point kNN over sliding windows with pane reuse (device tensors).  The device kernels
    and the torch plumbing between them (index offsets) run on one private stream; the caller's
    stream waits for it before the results are returned."""

    def __init__(self, ctx: _abi.Context, grid: _abi.Grid, qx: float, qy: float, r: float, k: int, panes: int = 2):
        import torch
        self.ctx, self.grid, self.q, self.r, self.k = ctx, grid, (qx, qy), r, int(k)
        self.panes = deque(maxlen=panes)  # (pane size, top-k idx int32[k] (-1 padded), dist f64[k])
        self.stream = torch.cuda.Stream()

    def push(self, x, y):
        import torch
        caller = torch.cuda.current_stream()
        self.stream.wait_stream(caller)  # the pane's x, y are ready
        prev = self.ctx.stream()
        self.ctx.set_stream(self.stream.cuda_stream)
        try:
            with torch.cuda.stream(self.stream):
                k = self.k
                dev = x.device
                oi = torch.empty(k, dtype=torch.int32, device=dev)
                od = torch.empty(k, dtype=torch.float64, device=dev)
                cnt = torch.zeros(1, dtype=torch.int32, device=dev)
                self.ctx.knn_pp_async(self.grid, x, y, self.q[0], self.q[1], self.r, k, oi, od, cnt)
                self.panes.append((len(x), oi, od))
                mi, md = self._merge()
        finally:
            self.ctx.set_stream(prev)
        caller.wait_stream(self.stream)
        n = int((mi != -1).sum().item())
        return mi[:n], md[:n]

    def _merge(self):
        import torch
        k, p = self.k, len(self.panes)
        dev = self.panes[0][1].device
        all_i = torch.empty((p, k), dtype=torch.int32, device=dev)
        all_d = torch.empty((p, k), dtype=torch.float64, device=dev)
        off = 0
        for j, (size, oi, od) in enumerate(self.panes):
            li = oi.to(torch.int64)
            all_i[j] = torch.where(li >= 0, li + off, torch.full_like(li, -1)).to(torch.int32)
            all_d[j] = od
            off += size
        mi = torch.empty(k, dtype=torch.int32, device=dev)
        md = torch.empty(k, dtype=torch.float64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ctx.knn_merge_async(all_d, all_i, p, k, k, mi, md, cnt)
        return mi, md


def run_incremental_range(ctx, grid, panes, qx, qy, r, approximate=False, window_size=10, slide_step=5):
    """Generator over windows: for each pane (x, y) of the stream, the result of the window that
    ends with it (PointPointRangeQuery.queryIncremental semantics)."""
    inc = IncrementalRange(ctx, grid, qx, qy, r, approximate, panes_per_window(window_size, slide_step))
    for x, y in panes:
        yield inc.push(x, y)
