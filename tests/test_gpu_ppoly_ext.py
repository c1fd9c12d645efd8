"""GPU parity of the point-polygon join and kNN through the C ABI.

geohip_join_ppoly against the C oracle (pair sets, bit-exact membership) over one and two grids,
radii with and without guaranteed cells, approximate mode, boundary points, NaN points and
polygons whose guaranteed bbox cells leave the grid (out-of-grid points then need the distance
check the join adds); geohip_knn_ppoly against the C oracle: (idx, distance bits) in
ascending (distance, idx), including large ties at distance 0 (points inside the polygon),
k = 1 / 256, fewer candidates than k, an empty window, approximate bbox distances, and the
argument errors where the reference throws.
"""
import math

import numpy as np
import pytest

import cref
from helpers import pairs_sorted
from spatialflink_amd import _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING


def agrid(n):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


def with_edges(x, y, off, vx, vy):
    """Append every vertex, edge midpoints and a NaN point to the window."""
    mx = (vx[:-1] + vx[1:]) / 2
    my = (vy[:-1] + vy[1:]) / 2
    return (np.concatenate([x, vx, mx, [math.nan, 116.0]]), np.concatenate([y, vy, my, [40.0, math.nan]]))


JOIN_CASES = [(500, 500, 0.005, False, 60), (500, 500, 0.03, False, 20), (500, 500, 0.03, True, 20),
              (100, 100, 0.05, False, 10), (200, 500, 0.02, False, 15), (500, 200, 0.04, False, 15),
              (100, 100, 0.0, False, 10)]


@pytest.mark.parametrize("case", range(len(JOIN_CASES)))
def test_join_ppoly_random(ctx, case):
    nu, nq, r, approx, npoly = JOIN_CASES[case]
    x, y = synth.uniform(300000, 70 + case)
    off, vx, vy = synth.star_polygons(npoly, 80 + case)
    x, y = with_edges(x, y, off, vx, vy)
    au, cu = agrid(nu)
    aq, cq = agrid(nq)
    got = ctx.join_ppoly(au, aq, x, y, off, vx, vy, r, approx)
    want = cref.join_ppoly(cu, cq, x, y, off, vx, vy, r, approx)
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


def test_join_ppoly_outside_grid_and_sliver(ctx):
    """Lg == 0: guaranteed bbox cells outside the grid match out-of-grid points, which the join
    then distance-checks; a diagonal sliver whose bbox corners are far from the polygon."""
    l = (BJ[1] - BJ[0]) / 100
    r = l * math.sqrt(2) * 1.2  # Lg == 0
    rings = [[(115.48, 39.58), (115.56, 39.58), (115.56, 39.66), (115.48, 39.66)],
             [(116.0, 40.0), (116.3, 40.3), (116.3, 40.301), (116.0, 40.001)]]
    vx = np.array([c[0] for ring in rings for c in ring])
    vy = np.array([c[1] for ring in rings for c in ring])
    off = np.array([0, 4, 8], np.uint32)
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(115.3, 115.8, 20000), rng.uniform(115.9, 116.4, 20000)])
    y = np.concatenate([rng.uniform(39.4, 39.8, 20000), rng.uniform(39.9, 40.4, 20000)])
    x, y = with_edges(x, y, off, vx, vy)
    au, cu = agrid(100)
    for rr, approx in ((r, False), (r, True), (0.004, False), (0.05, False)):
        got = ctx.join_ppoly(au, au, x, y, off, vx, vy, rr, approx)
        want = cref.join_ppoly(cu, cu, x, y, off, vx, vy, rr, approx)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
        rg = {(p, q) for q, p in cref.range_ppoly(cu, x, y, off, vx, vy, rr, approx).tolist()}
        if not approx:
            assert {tuple(p) for p in got.tolist()} <= rg


def test_join_ppoly_capacity_and_device_buffers(ctx):
    import torch
    x, y = synth.uniform(200000, 91)
    off, vx, vy = synth.star_polygons(30, 92)
    au, cu = agrid(500)
    want = pairs_sorted(cref.join_ppoly(cu, cu, x, y, off, vx, vy, 0.01)).tolist()
    assert len(want) > 10
    with pytest.raises(_abi.GeohipCapacityError):
        ctx.join_ppoly(au, au, x, y, off, vx, vy, 0.01, cap=5)
    tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    got = ctx.join_ppoly(au, au, tx, ty, off, vx, vy, 0.01)
    assert pairs_sorted(got.cpu().numpy()).tolist() == want


KNN_CASES = [(500, 0.005, 50, False), (500, 0.005, 50, True), (100, 0.05, 10, False), (500, 0.02, 256, False),
             (200, 0.03, 1, False), (1000, 0.0, 20, False), (100, 0.5, 100, False)]


@pytest.mark.parametrize("case", range(len(KNN_CASES)))
def test_knn_ppoly_random(ctx, case):
    gn, r, k, approx = KNN_CASES[case]
    x, y = synth.uniform(400000, 110 + case)
    off, vx, vy = synth.star_polygons(3, 120 + case)
    ag, cg = agrid(gn)
    for p in range(3):
        px, py = vx[off[p]:off[p + 1]], vy[off[p]:off[p + 1]]
        wx, wy = with_edges(x, y, np.array([0, len(px)]), px, py)
        gi, gd = ctx.knn_ppoly(ag, wx, wy, px, py, r, k, approx)
        wi, wd = cref.knn_ppoly(cg, wx, wy, px, py, r, k, approx)
        assert gi.tolist() == wi.tolist()
        assert np.array_equal(gd.view(np.uint64), wd.view(np.uint64))


def test_knn_ppoly_ties_small_and_empty(ctx):
    ag, cg = agrid(500)
    ring_x = np.array([116.30, 116.40, 116.40, 116.30])
    ring_y = np.array([40.10, 40.10, 40.20, 40.20])
    rng = np.random.default_rng(5)
    # 5000 points inside (distance 0: the k smallest are the k smallest indices), some outside
    x = np.concatenate([rng.uniform(116.29, 116.41, 3000), rng.uniform(116.31, 116.39, 5000)])
    y = np.concatenate([rng.uniform(40.09, 40.21, 3000), rng.uniform(40.11, 40.19, 5000)])
    perm = rng.permutation(len(x))
    x, y = x[perm], y[perm]
    for k in (1, 64, 256):
        gi, gd = ctx.knn_ppoly(ag, x, y, ring_x, ring_y, 0.005, k)
        wi, wd = cref.knn_ppoly(cg, x, y, ring_x, ring_y, 0.005, k)
        assert gi.tolist() == wi.tolist() and np.array_equal(gd.view(np.uint64), wd.view(np.uint64))
        assert (gd == 0).all()
    # fewer candidates than k
    gi, gd = ctx.knn_ppoly(ag, x[:40], y[:40], ring_x, ring_y, 0.005, 100)
    wi, wd = cref.knn_ppoly(cg, x[:40], y[:40], ring_x, ring_y, 0.005, 100)
    assert gi.tolist() == wi.tolist() and len(gi) <= 40
    # empty window
    gi, gd = ctx.knn_ppoly(ag, np.zeros(0), np.zeros(0), ring_x, ring_y, 0.005, 10)
    assert len(gi) == 0


def test_knn_ppoly_errors(ctx):
    ag, _ = agrid(500)
    x, y = synth.uniform(1000, 1)
    sq_x, sq_y = np.array([116.3, 116.4, 116.4, 116.3]), np.array([40.1, 40.1, 40.2, 40.2])
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.knn_ppoly(ag, x, y, sq_x, sq_y, 0.01, 0)
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.knn_ppoly(ag, x, y, sq_x[:3], sq_y[:3], 0.01, 5)  # <= 3 coordinates (Polygon.java:53)


@pytest.mark.parametrize("approx", [False, True])
def test_knn_ppoly_large_k(ctx, approx):
    """Any k (PointPolygonKNNQuery.java:34): GEOHIP_KNN_PPOLY_MAX_K + 1, 2000 and 60000 take the
    large-k form (radix rounds, gather, sort); a k above the candidate count returns them all.
    Points inside the polygon tie at distance 0 (ordered by index)."""
    ag, cg = agrid(500)
    rng = np.random.default_rng(77)
    x, y = synth.uniform(1_000_000, 78)
    star = np.array(synth._star(rng, 116.4, 40.2, 0.02, 50))
    ring_x, ring_y = star[:, 0].copy(), star[:, 1].copy()
    for k in (_abi.KNN_PPOLY_MAX_K + 1, 2000, 60000):
        gi, gd = ctx.knn_ppoly(ag, x, y, ring_x, ring_y, 0.005, k, approx)
        wi, wd = cref.knn_ppoly(cg, x, y, ring_x, ring_y, 0.005, k, approx)
        assert len(wi) <= k and (k < 50000 or len(wi) < k)
        assert gi.tolist() == wi.tolist()
        assert np.array_equal(gd.view(np.uint64), wd.view(np.uint64))


def test_knn_ppoly_c4_size(ctx):
    """C4 window size (50M uniform points, 500x500) against the C oracle for one polygon."""
    import torch
    n = 50_000_000
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_uniform_async(x, y, 0, 5, BJ)
    torch.cuda.synchronize()
    off, vx, vy = synth.star_polygons(1, 6)
    ag, cg = agrid(500)
    gi, gd = ctx.knn_ppoly(ag, x, y, vx, vy, 0.005, 100)
    hx, hy = synth.uniform(n, 5)
    wi, wd = cref.knn_ppoly(cg, hx, hy, vx, vy, 0.005, 100)
    assert gi.cpu().numpy().tolist() == wi.tolist()
    assert np.array_equal(gd.cpu().numpy().view(np.uint64), wd.view(np.uint64))


def test_knn_ppoly_large_candidate_set(ctx):
    """More than 2^17 candidates: the multi-block radix-select rounds instead of rsel_small."""
    x, y = synth.uniform(1_500_000, 131)
    off, vx, vy = synth.star_polygons(1, 132)
    ag, cg = agrid(100)
    for k, approx in ((256, False), (7, False), (100, True)):
        gi, gd = ctx.knn_ppoly(ag, x, y, vx, vy, 0.5, k, approx)
        wi, wd = cref.knn_ppoly(cg, x, y, vx, vy, 0.5, k, approx)
        assert gi.tolist() == wi.tolist()
        assert np.array_equal(gd.view(np.uint64), wd.view(np.uint64))


def test_sharded_device_paths_world1(ctx):
    """distributed.join_ppoly_sharded / knn_ppoly_sharded with the default device engines
    (geohip_join_ppoly, geohip_knn_ppoly + geohip_knn_merge_async) in a 1-rank group."""
    import socket
    import torch
    import torch.distributed as dist
    from spatialflink_amd import distributed as D
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        au, cu = agrid(200)
        aq, cq = agrid(500)
        x, y = synth.uniform(300_000, 141)
        off, vx, vy = synth.star_polygons(12, 142)
        tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        pairs, o, total = D.join_ppoly_sharded(tx, ty, 0, off, vx, vy, 0.02, grid_points=au, grid_query=aq, ctx=ctx)
        want = cref.join_ppoly(cu, cq, x, y, off, vx, vy, 0.02)
        assert pairs_sorted(pairs.cpu().numpy()).tolist() == pairs_sorted(want).tolist() and total == len(want)
        p0 = slice(off[0], off[1])
        res = D.knn_ppoly_sharded(tx, ty, 0, vx[p0], vy[p0], 0.05, 30, grid=au, ctx=ctx)
        wi, wd = cref.knn_ppoly(cu, x, y, vx[p0], vy[p0], 0.05, 30)
        assert res.idx.cpu().numpy().tolist() == wi.tolist()
        assert np.array_equal(res.dist.cpu().numpy().view(np.uint64), wd.view(np.uint64))
    finally:
        dist.destroy_process_group()


def test_knn_ppoly_async_cached_plan(ctx):
    """geohip_knn_ppoly_async: the polygon plan cached by the ctx across windows and replaced when
    the polygon changes; the selection path guessed from the previous window's candidate count
    (a small window after a huge one and the reverse) -- every result exact vs the oracle."""
    import torch
    ag, cg = agrid(500)
    rng = np.random.default_rng(91)
    small = np.array(synth._star(rng, 116.4, 40.2, 0.01, 30))
    huge = np.array(synth._star(rng, 116.5, 40.3, 0.35, 60))  # > 128K candidates in a 2M window
    oi = torch.empty(64, dtype=torch.int32, device="cuda")
    od = torch.empty(64, dtype=torch.float64, device="cuda")
    oc = torch.zeros(1, dtype=torch.int32, device="cuda")
    for j, (poly, n) in enumerate([(small, 300_000), (small, 2_000_000), (huge, 2_000_000), (huge, 300_000),
                                   (small, 2_000_000), (huge, 2_000_000), (small, 0)]):
        x, y = synth.uniform(n, 92 + j)
        tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        for k in (50, 64):
            ctx.knn_ppoly_async(ag, tx, ty, poly[:, 0].copy(), poly[:, 1].copy(), 0.005, k, False, oi, od, oc)
            wi, wd = cref.knn_ppoly(cg, x, y, poly[:, 0].copy(), poly[:, 1].copy(), 0.005, k)
            m = int(oc.item())
            assert m == len(wi), (j, k)
            assert oi[:m].cpu().numpy().astype(np.uint32).tolist() == wi.tolist(), (j, k)
            assert np.array_equal(od[:m].cpu().numpy().view(np.uint64), wd.view(np.uint64)), (j, k)


def _cell_edges(lo, l, n):
    """Per cell boundary k in 1..n-1 of one grid axis: the first double of cell k and the last
    double of cell k - 1 under Java's (int) Math.floor((v - min) / l) (found by bisection on the
    ordered doubles), plus both ends of the axis."""
    def cell(v):
        return int(math.floor((v - lo) / l))

    def first_at_least(k):
        a, b = lo + (k - 1) * l, lo + (k + 1) * l  # cell(a) < k <= cell(b)
        while True:
            m = (a + b) / 2
            if m in (a, b):
                return b
            if cell(m) >= k:
                b = m
            else:
                a = m

    out = [lo, lo + n * l, np.nextafter(lo + n * l, -np.inf)]
    for k in range(1, n):
        v = first_at_least(k)
        out += [v, np.nextafter(v, -np.inf)]
    for k in range(n):  # the device's 4 x 4 subcell edges (sub_edge: min + (c + i / 4) * l)
        for i in (1, 2, 3):
            v = lo + (k + 0.25 * i) * l
            out += [v, np.nextafter(v, -np.inf)]
    return np.array(out)


@pytest.mark.parametrize("holes", [False, True])
def test_ppoly_cell_class_box_edges(ctx, holes):
    """Per-cell classes (classify_cells) decide whole cells and 4 x 4 subcells from their exact
    coordinate boxes: points at every cell's and subcell's extreme doubles (both sides of each
    boundary, both axes), cell centres, NaN coordinates (cell 0) and random points, for the range
    query and the exact join, against the oracle."""
    n = 500
    l = (BJ[1] - BJ[0]) / n
    ag, cg = agrid(n)
    if holes:
        pr, off, vx, vy, _ = synth.holed_polygons(25, 91)
    else:
        pr = None
        off, vx, vy = synth.star_polygons(40, 90)
    ex = _cell_edges(BJ[0], l, n)
    ey = _cell_edges(BJ[2], l, n)
    # boundary doubles around each polygon (within r_max of its box): their cross product
    px, py = [], []
    for p in range(len(off) - 1 if pr is None else len(pr) - 1):
        a, b = (int(off[p]), int(off[p + 1])) if pr is None else (int(off[pr[p]]), int(off[pr[p + 1]]))
        sx = ex[(ex > vx[a:b].min() - 0.013) & (ex < vx[a:b].max() + 0.013)]
        sy = ey[(ey > vy[a:b].min() - 0.013) & (ey < vy[a:b].max() + 0.013)]
        gx, gy = np.meshgrid(sx, sy, indexing="ij")
        px.append(gx.ravel())
        py.append(gy.ravel())
    gx, gy = np.concatenate(px), np.concatenate(py)
    cx = BJ[0] + (np.arange(n) + 0.5) * l
    cy = BJ[2] + (np.arange(n) + 0.5) * l
    hx, hy = np.meshgrid(cx, cy, indexing="ij")
    rng = np.random.default_rng(5)
    rx, ry = synth.uniform(200000, 93)
    x = np.concatenate([gx.ravel(), hx.ravel(), rx, [math.nan, BJ[0], math.nan], rng.uniform(BJ[0], BJ[1], 10)])
    y = np.concatenate([gy.ravel(), hy.ravel(), ry, [BJ[2], math.nan, math.nan], np.full(10, math.nan)])
    for r in (0.005, 0.012, 0.0):
        got = ctx.range_ppoly(ag, x, y, off, vx, vy, r, poly_rings=pr)
        want = cref.range_ppoly(cg, x, y, off, vx, vy, r, poly_rings=pr)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
        got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, r, poly_rings=pr)
        want = cref.join_ppoly(cg, cg, x, y, off, vx, vy, r, poly_rings=pr)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


@pytest.mark.parametrize("holes", [False, True])
def test_ppoly_refinement_part_edges(ctx, holes):
    """The candidate refinement (ppoly_cand_refine) decides a mixed subcell's candidates by the
    4 x 4 parts the host classified (sub16_edge: min + (c + j / 16) * l) and a mixed part's by its
    4 x 4 sub-parts (sub64_edge: min + (c + j / 64) * l): points at every part and sub-part edge
    double and the double below it, both axes, around each polygon (the parts straddling its
    boundary and its r-contour), for the range query and the exact join, against the oracle."""
    n = 500
    l = (BJ[1] - BJ[0]) / n
    ag, cg = agrid(n)
    if holes:
        pr, off, vx, vy, _ = synth.holed_polygons(4, 95)
        rings = [(int(off[pr[p]]), int(off[pr[p + 1]])) for p in range(len(pr) - 1)]
    else:
        pr = None
        off, vx, vy = synth.star_polygons(6, 94)
        rings = [(int(off[p]), int(off[p + 1])) for p in range(len(off) - 1)]

    def part_edges(lo, a, b):
        k0, k1 = int(math.floor((a - lo) / l)) - 1, int(math.floor((b - lo) / l)) + 2
        out = []
        for k in range(max(k0, 0), min(k1, n)):
            for j in range(1, 64):
                v = lo + (k + 0.015625 * j) * l
                out += [v, np.nextafter(v, -np.inf)]
        return np.array(out)

    px, py = [], []
    for a, b in rings:
        sx = part_edges(BJ[0], vx[a:b].min() - 0.013, vx[a:b].max() + 0.013)
        sy = part_edges(BJ[2], vy[a:b].min() - 0.013, vy[a:b].max() + 0.013)
        # every edge double of x against a thinned set of the y ones, and the reverse (the full
        # cross product of one polygon is ~5e6 points)
        gx, gy = np.meshgrid(sx, sy[::31], indexing="ij")
        hx, hy = np.meshgrid(sx[::31], sy, indexing="ij")
        px += [gx.ravel(), hx.ravel()]
        py += [gy.ravel(), hy.ravel()]
    x, y = np.concatenate(px), np.concatenate(py)
    assert len(x) > 100000
    for r in (0.005, 0.012):
        got = ctx.range_ppoly(ag, x, y, off, vx, vy, r, poly_rings=pr)
        want = cref.range_ppoly(cg, x, y, off, vx, vy, r, poly_rings=pr)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
        got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, r, poly_rings=pr)
        want = cref.join_ppoly(cg, cg, x, y, off, vx, vy, r, poly_rings=pr)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


def test_ppoly_stream_overflow_and_regrow(ctx):
    """The streaming point-polygon path's rare branches: 96 concentric star polygons put ~96
    entries in each central cell, so a wave stages more pairs (and mixed-subcell candidates) than
    its LDS region holds and flushes it before the chunk's end; the candidates of the first call
    exceed the initial candidate buffer (n / 16), so their chunks go to the redo pass (and a wave's
    candidates can pass its spill list: ~96 per point against 16, the redo pass again).
    Range, exact and approximate, and join vs the oracle; a second call reuses the cached plan and
    the grown buffer."""
    ag, cg = agrid(100)
    rng = np.random.default_rng(123)
    off, vx, vy = [0], [], []
    for p in range(96):
        ring = synth._star(rng, 116.4, 40.2, 0.03 + 0.0004 * p, 50)
        vx += [a for a, _ in ring]
        vy += [b for _, b in ring]
        off.append(len(vx))
    off, vx, vy = np.array(off, np.uint32), np.array(vx), np.array(vy)
    x = rng.uniform(116.3, 116.5, 200000)
    y = rng.uniform(40.1, 40.3, 200000)
    x, y = with_edges(x, y, off, vx, vy)
    for r, approx in ((0.01, False), (0.02, True), (0.01, False)):
        got = ctx.range_ppoly(ag, x, y, off, vx, vy, r, approx)
        want = cref.range_ppoly(cg, x, y, off, vx, vy, r, approx)
        assert len(want) > 4096 * 2
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
    got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, 0.01)
    want = cref.join_ppoly(cg, cg, x, y, off, vx, vy, 0.01)
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


def test_join_after_knn_ppoly_scratch(ctx):
    """Regression: the point-polygon kNN's candidate buffer once shared a scratch slot with the
    join's tile counts, so a point join after a large point-polygon kNN on the same ctx read
    leftover counts.  kNN first (a window larger than any tile-count array), then the join."""
    x, y = synth.uniform(400000, 140)
    off, vx, vy = synth.star_polygons(1, 141)
    ag, cg = agrid(500)
    gi, gd = ctx.knn_ppoly(ag, x, y, vx, vy, 0.02, 256)
    wi, wd = cref.knn_ppoly(cg, x, y, vx, vy, 0.02, 256)
    assert gi.tolist() == wi.tolist()
    dx, dy = synth.uniform(200000, 142)
    qx, qy = synth.uniform(2000, 143)
    for _ in range(2):
        got = ctx.join_pp(ag, ag, dx, dy, qx, qy, 0.01, False)
        want = cref.join_pp(cg, cg, dx, dy, qx, qy, 0.01)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
        ctx.knn_ppoly(ag, x, y, vx, vy, 0.02, 256)
