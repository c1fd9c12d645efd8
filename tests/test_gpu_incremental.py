"""GPU: incremental sliding windows with pane reuse equal full evaluation.

Every window's result, assembled from the per-pane GPU results, must be bit-identical to the C
oracle's evaluation of the whole window (the points of its last window_size / slide_step panes,
concatenated in arrival order): range index sets (ascending), kNN (idx, distance bits).
Pane sizes are ragged and include an empty pane; the first windows hold fewer panes.
"""
import numpy as np
import pytest

import cref
from spatialflink_amd import _abi, synth
from spatialflink_amd.incremental import IncrementalKNN, IncrementalRange
from spatialflink_amd.operators import Point, PointPointRangeQuery, PointWindow, QueryConfiguration, UniformGrid

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING
Q = synth.README_QUERY
SIZES = [50_000, 120_000, 0, 70_001, 200_000, 33_333, 90_000]


def grids(n):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


def pane_stream(seed):
    out, base = [], 0
    for s in SIZES:
        x, y = synth.uniform(s, seed, base=base)
        out.append((x, y))
        base += s
    return out


@pytest.mark.parametrize("p,start", [(2, 0), (3, 0), (2, (1 << 32) - 250_000), (3, (1 << 31) - 100_000)])
def test_incremental_range_equals_full_window(ctx, p, start):
    """Stream positions start at 0, and just below 2^32 / 2^31 (the device pane's int32 hits wrap
    sign and value inside the stream): window-local indices are (position - start) mod 2^32."""
    import torch
    ag, cg = grids(100)
    panes = pane_stream(11)
    inc = IncrementalRange(ctx, ag, Q[0], Q[1], 0.5, False, p, start=start)
    for j, (x, y) in enumerate(panes):
        parts = inc.push(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
        # the panes' hits are stream positions (geohip_range_pp_pane): no per-window pass
        got = (torch.cat([h.to(torch.int64) for h in parts]).cpu().numpy() - inc.window_start) & 0xFFFFFFFF
        assert got.tolist() == inc.window_local().cpu().numpy().tolist()
        win = panes[max(0, j - p + 1):j + 1]
        wx = np.concatenate([w[0] for w in win])
        wy = np.concatenate([w[1] for w in win])
        want = np.sort(cref.range_pp(cg, wx, wy, Q[0], Q[1], 0.5).astype(np.int64))
        assert got.tolist() == want.tolist()


@pytest.mark.parametrize("p,k", [(2, 50), (3, 7)])
def test_incremental_knn_equals_full_window(ctx, p, k):
    import torch
    ag, cg = grids(100)
    panes = pane_stream(12)
    inc = IncrementalKNN(ctx, ag, Q[0], Q[1], 0.5, k, p)
    for j, (x, y) in enumerate(panes):
        gi, gd = inc.push(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
        win = panes[max(0, j - p + 1):j + 1]
        wx = np.concatenate([w[0] for w in win])
        wy = np.concatenate([w[1] for w in win])
        wi, wd = cref.knn_pp(cg, wx, wy, Q[0], Q[1], 0.5, k)
        assert gi.cpu().numpy().tolist() == wi.tolist()
        assert np.array_equal(gd.cpu().numpy().view(np.uint64), wd.view(np.uint64))


def test_query_incremental_operator(ctx):
    """PointPointRangeQuery.queryIncremental mirror: 10 s windows sliding by 5 s (2 panes)."""
    grid = UniformGrid(100, *BJ)
    op = PointPointRangeQuery(QueryConfiguration(window_size=10, slide_step=5), grid, ctx)
    panes = pane_stream(13)
    cg = grids(100)[1]
    windows = list(op.queryIncremental([PointWindow(x, y) for x, y in panes], Point(*Q), 0.5))
    for j, got in enumerate(windows):
        win = panes[max(0, j - 1):j + 1]
        wx = np.concatenate([w[0] for w in win])
        wy = np.concatenate([w[1] for w in win])
        assert np.asarray(got).tolist() == np.sort(cref.range_pp(cg, wx, wy, Q[0], Q[1], 0.5)).tolist()


def test_incremental_ppoly_equals_full_window(ctx):
    import torch
    from helpers import pairs_sorted
    from spatialflink_amd.incremental import IncrementalPPolyRange
    l = (BJ[1] - BJ[0]) / 500
    ag, cg = _abi.make_grid(BJ[0], BJ[2], l, 500), cref.grid(BJ[0], BJ[2], l, 500)
    off, vx, vy = synth.star_polygons(40, 77)
    panes = pane_stream(14)
    inc = IncrementalPPolyRange(ctx, ag, off, vx, vy, 0.01, False, 2)
    for j, (x, y) in enumerate(panes):
        got = inc.push(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
        got = np.concatenate([g.cpu().numpy().astype(np.int64).reshape(-1, 2) & 0xFFFFFFFF for g in got])
        got[:, 1] = (got[:, 1] - inc.window_start) & 0xFFFFFFFF  # stream positions -> window-local
        win = panes[max(0, j - 1):j + 1]
        wx = np.concatenate([w[0] for w in win])
        wy = np.concatenate([w[1] for w in win])
        want = cref.range_ppoly(cg, wx, wy, off, vx, vy, 0.01)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


@pytest.mark.parametrize("p,k", [(16, 40), (5, 300), (2, 2000), (3, 1500)])
def test_pane_merge_many_panes(ctx, p, k):
    """geohip_knn_merge_panes_async over up to 16 panes of a ring (slots rotating, ties across
    panes, panes with fewer candidates than k, the large-k pane pass): every window equals the
    kNN of the window's concatenated panes.  p k <= 4096 takes the one-workgroup LDS merge, (3,
    1500) the global one."""
    import torch
    ag, cg = grids(100)
    rng = np.random.default_rng(p * 31 + k)
    panes = []
    base = 0
    for j in range(p + 4):
        s = int(rng.integers(2000, 60000)) if j % 3 else 900
        x, y = synth.uniform(s, 70 + j, base=base)
        x[:5] = Q[0] + 1e-3  # exact ties across panes (ordered by window index)
        y[:5] = Q[1]
        panes.append((x, y))
        base += s
    inc = IncrementalKNN(ctx, ag, Q[0], Q[1], 0.5, k, p)
    for j, (x, y) in enumerate(panes):
        gi, gd = inc.push(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
        win = panes[max(0, j - p + 1):j + 1]
        wi, wd = cref.knn_pp(cg, np.concatenate([w[0] for w in win]), np.concatenate([w[1] for w in win]),
                             Q[0], Q[1], 0.5, k)
        assert gi.cpu().numpy().tolist() == wi.tolist(), j
        assert np.array_equal(gd.cpu().numpy().view(np.uint64), wd.view(np.uint64)), j


@pytest.mark.parametrize("n", [300_000, 70_000_000])
def test_range_pane_point_base(ctx, n):
    """geohip_range_pp_pane: the hits of geohip_range_pp plus the base (mod 2^32), in the one-kernel
    range path and (70M points) the multi-launch one; a base near 2^32 wraps."""
    import torch
    ag, _ = grids(100)
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_uniform_async(x, y, 0, 41, BJ)
    plain = ctx.range_pp(ag, x, y, Q[0], Q[1], 0.5).to(torch.int64)
    for base in (12345, (1 << 32) - 1000):
        got = ctx.range_pp(ag, x, y, Q[0], Q[1], 0.5, point_base=base).to(torch.int64) & 0xFFFFFFFF
        assert torch.equal(got, (plain + base) & 0xFFFFFFFF)
