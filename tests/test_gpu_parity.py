"""GPU parity: libgeohip (HIP, gfx950) through the C ABI against the oracles.

Bit-exact everywhere: range/join/ppoly index sets, kNN (idx, distance bits) in ascending
(dist, idx) order.  Small cases against the committed golden vectors and the C oracle;
full BASELINE sizes (C1 range 1M, C2 kNN 10M) against the C oracle too (it finishes in
seconds), plus size-independent properties at larger sizes.
"""
import math

import numpy as np
import pytest

import cref
from helpers import arr, fx, grid_vals, pairs_sorted
from spatialflink_amd import _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING
Q = synth.README_QUERY


def agrid(n):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


# ------------------------------------------------------------------ fp64 primitives -----
def test_fp64_primitives(ctx):
    import torch
    rng = np.random.default_rng(0)
    a = rng.uniform(-1, 1, 200000) * 10.0 ** rng.integers(-8, 3, 200000)
    b = rng.uniform(-1, 1, 200000) * 10.0 ** rng.integers(-8, 3, 200000)
    a[:6] = [0.0, 1e-310, 1e300, math.inf, math.nan, 3 * 2 ** -10]
    b[:6] = [0.0, 3e-310, 1e300, 1.0, 1.0, 4 * 2 ** -10]
    ta = torch.from_numpy(a).cuda()
    tb = torch.from_numpy(b).cuda()
    s, d, h, ms = [t.cpu().numpy() for t in ctx.selftest_fp64(ta, tb)]
    with np.errstate(all="ignore"):
        assert np.array_equal(s.view(np.uint64), np.sqrt(np.abs(a)).view(np.uint64))
        dd = a / b
        same = (d.view(np.uint64) == dd.view(np.uint64)) | (np.isnan(d) & np.isnan(dd))
        assert same.all()
        assert np.array_equal(ms.view(np.uint64), (a * b - b * b).view(np.uint64)) or \
            np.array_equal(np.isnan(ms), np.isnan(a * b - b * b))
    want = np.array([cref.hypot(float(p), float(q)) for p, q in zip(a[:20000], b[:20000])])
    hh = h[:20000]
    assert np.array_equal(hh.view(np.uint64)[~np.isnan(want)], want.view(np.uint64)[~np.isnan(want)])


def test_synth_uniform_bit_identical(ctx):
    import torch
    n = 100003
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_uniform_async(x, y, 12345, 2, BJ)
    torch.cuda.synchronize()
    hx, hy = synth.uniform(n, 2, BJ, base=12345)
    assert np.array_equal(x.cpu().numpy().view(np.uint64), hx.view(np.uint64))
    assert np.array_equal(y.cpu().numpy().view(np.uint64), hy.view(np.uint64))


# ------------------------------------------------------------------ golden vectors ------
def test_range_golden(ctx, golden):
    for c in golden["range_pp"]:
        g = _abi.make_grid(*grid_vals(c["grid"]))
        got = ctx.range_pp(g, arr(c["x"]), arr(c["y"]), fx(c["qx"]), fx(c["qy"]), fx(c["r"]), c["approximate"])
        assert got.tolist() == c["expect"]  # ascending index order


def test_knn_golden(ctx, golden):
    for c in golden["knn_pp"]:
        g = _abi.make_grid(*grid_vals(c["grid"]))
        oi, od = ctx.knn_pp(g, arr(c["x"]), arr(c["y"]), fx(c["qx"]), fx(c["qy"]), fx(c["r"]), c["k"])
        assert oi.tolist() == c["expect_idx"]
        assert [v.hex() for v in od.tolist()] == c["expect_dist"]


# ------------------------------------------------------------------ random vs oracle ----
def _window(rng, n, nan_every=0):
    x = rng.uniform(BJ[0] - 0.1, BJ[1] + 0.1, n)
    y = rng.uniform(BJ[2] - 0.1, BJ[3] + 0.1, n)
    if nan_every:
        x[::nan_every] = np.nan
        y[3::nan_every] = np.nan
    return x, y


RANGE_CASES = [(100, 0.5, Q, False), (100, 0.05, Q, False), (500, 0.05, (116.3, 40.2), False),
               (1000, 0.05, Q, False), (100, 0.5, Q, True), (37, 0.3, (115.45, 39.55), False),
               (100, 0.0, Q, False), (100, -1.0, Q, False), (100, math.nan, Q, False),
               (10, 2.0, (116.5, 40.3), False), (100, 0.03, (117.7, 41.3), False)]


@pytest.mark.parametrize("n", [0, 1, 255, 1024, 1025, 70001])
def test_range_sizes(ctx, n):
    rng = np.random.default_rng(n + 1)
    x, y = _window(rng, n, nan_every=53)
    ag, cg = agrid(100)
    got = ctx.range_pp(ag, x, y, Q[0], Q[1], 0.5)
    want = cref.range_pp(cg, x, y, Q[0], Q[1], 0.5)
    assert got.tolist() == sorted(want.tolist())


@pytest.mark.parametrize("case", range(len(RANGE_CASES)))
def test_range_random(ctx, case):
    gn, r, q, approx = RANGE_CASES[case]
    rng = np.random.default_rng(100 + case)
    x, y = _window(rng, 200000, nan_every=997)
    ag, cg = agrid(gn)
    got = ctx.range_pp(ag, x, y, q[0], q[1], r, approx)
    want = cref.range_pp(cg, x, y, q[0], q[1], r, approx)
    assert got.tolist() == sorted(want.tolist())


def test_range_capacity(ctx):
    rng = np.random.default_rng(5)
    x, y = _window(rng, 50000)
    ag, cg = agrid(100)
    want = sorted(cref.range_pp(cg, x, y, Q[0], Q[1], 0.5).tolist())
    with pytest.raises(_abi.GeohipCapacityError):
        ctx.range_pp(ag, x, y, Q[0], Q[1], 0.5, cap=10)
    got = ctx.range_pp(ag, x, y, Q[0], Q[1], 0.5, cap=len(want))
    assert got.tolist() == want


KNN_CASES = [(100, 0.5, Q, 50), (100, 0.5, Q, 1), (100, 0.05, Q, 64), (100, 0.05, Q, 65), (500, 0.05, Q, 100),
             (1000, 0.05, Q, 128), (1000, 0.05, Q, 129), (100, 0.2, (116.0, 40.5), 256), (37, 0.3, (115.45, 39.55), 10),
             (100, math.nan, Q, 7), (100, 0.0, Q, 5), (100, 0.005, Q, 50)]


@pytest.mark.parametrize("case", range(len(KNN_CASES)))
def test_knn_random(ctx, case):
    gn, r, q, k = KNN_CASES[case]
    rng = np.random.default_rng(200 + case)
    x, y = _window(rng, 300000, nan_every=1009)
    ag, cg = agrid(gn)
    oi, od = ctx.knn_pp(ag, x, y, q[0], q[1], r, k)
    wi, wd = cref.knn_pp(cg, x, y, q[0], q[1], r, k)
    assert oi.tolist() == wi.tolist()
    assert np.array_equal(od.view(np.uint64), wd.view(np.uint64))


@pytest.mark.parametrize("n", [0, 1, 3, 1000, 4097])
def test_knn_small_windows(ctx, n):
    rng = np.random.default_rng(n + 7)
    x, y = _window(rng, n)
    ag, cg = agrid(100)
    oi, od = ctx.knn_pp(ag, x, y, Q[0], Q[1], 0.5, 50)
    wi, wd = cref.knn_pp(cg, x, y, Q[0], Q[1], 0.5, 50)
    assert oi.tolist() == wi.tolist() and np.array_equal(od.view(np.uint64), wd.view(np.uint64))


def test_knn_ties_duplicates(ctx):
    """Many identical coordinates: ties broken by window index (the build contract)."""
    rng = np.random.default_rng(9)
    x, y = _window(rng, 20000)
    x[5000:9000] = 116.40
    y[5000:9000] = 39.93
    ag, cg = agrid(100)
    for k in (1, 50, 200):
        oi, od = ctx.knn_pp(ag, x, y, Q[0], Q[1], 0.5, k)
        wi, wd = cref.knn_pp(cg, x, y, Q[0], Q[1], 0.5, k)
        assert oi.tolist() == wi.tolist() and np.array_equal(od.view(np.uint64), wd.view(np.uint64))


def test_knn_rejects_bad_k(ctx):
    ag, _ = agrid(100)
    x = np.zeros(10)
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.knn_pp(ag, x, x, Q[0], Q[1], 0.5, 0)


# ------------------------------------------------------------------ BASELINE sizes -------
def test_c1_range_1m_full(ctx):
    """BASELINE configs[0]: 1M uniform points, 100x100 grid, r = 0.5, README query."""
    x, y = synth.uniform(1_000_000, 1)
    ag, cg = agrid(100)
    got = ctx.range_pp(ag, x, y, Q[0], Q[1], 0.5)
    want = cref.range_pp(cg, x, y, Q[0], Q[1], 0.5)
    assert got.tolist() == sorted(want.tolist())
    assert 0.20 < len(got) / 1e6 < 0.24  # ~21.9 % hits


def test_c2_knn_10m_full_device(ctx):
    """BASELINE configs[1]: 10M uniform points on device, k = 50, 100x100, r = 0.5."""
    import torch
    n = 10_000_000
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_uniform_async(x, y, 0, 2, BJ)
    torch.cuda.synchronize()
    ag, cg = agrid(100)
    oi, od = ctx.knn_pp(ag, x, y, Q[0], Q[1], 0.5, 50)
    hx, hy = synth.uniform(n, 2)
    wi, wd = cref.knn_pp(cg, hx, hy, Q[0], Q[1], 0.5, 50)
    assert oi.cpu().numpy().astype(np.uint32).tolist() == wi.tolist()
    assert np.array_equal(od.cpu().numpy().view(np.uint64), wd.view(np.uint64))


def test_knn_async_and_merge(ctx):
    """Shard a window in 4 slices, kNN each with the async form, merge with the device merge
    (the cross-GPU path without RCCL): equals the unsharded oracle result."""
    import torch
    rng = np.random.default_rng(3)
    hx, hy = _window(rng, 400000)
    ag, cg = agrid(100)
    k = 50
    S = 4
    per = len(hx) // S
    d_all = torch.empty((S, k), dtype=torch.float64, device="cuda")
    i_all = torch.empty((S, k), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(S + 1, dtype=torch.int32, device="cuda")
    for s in range(S):
        xs = torch.from_numpy(hx[s * per:(s + 1) * per].copy()).cuda()
        ys = torch.from_numpy(hy[s * per:(s + 1) * per].copy()).cuda()
        ctx.knn_pp_async(ag, xs, ys, Q[0], Q[1], 0.5, k, i_all[s], d_all[s], cnt[s:s + 1])
        torch.cuda.synchronize()
        valid = i_all[s] != -1
        i_all[s] = torch.where(valid, i_all[s] + s * per, i_all[s])
    oi = torch.empty(k, dtype=torch.int32, device="cuda")
    od = torch.empty(k, dtype=torch.float64, device="cuda")
    ctx.knn_merge_async(d_all, i_all, S, k, k, oi, od, cnt[S:S + 1])
    torch.cuda.synchronize()
    wi, wd = cref.knn_pp(cg, hx[:S * per], hy[:S * per], Q[0], Q[1], 0.5, k)
    assert oi.cpu().numpy().astype(np.uint32).tolist() == wi.tolist()
    assert np.array_equal(od.cpu().numpy().view(np.uint64), wd.view(np.uint64))


def test_range_device_mode(ctx):
    import torch
    rng = np.random.default_rng(4)
    hx, hy = _window(rng, 123457)
    ag, cg = agrid(500)
    got = ctx.range_pp(ag, torch.from_numpy(hx).cuda(), torch.from_numpy(hy).cuda(), 116.3, 40.2, 0.05)
    want = cref.range_pp(cg, hx, hy, 116.3, 40.2, 0.05)
    assert got.cpu().numpy().astype(np.uint32).tolist() == sorted(want.tolist())


def test_operator_api(ctx):
    from spatialflink_amd import (Point, PointPointKNNQuery, PointPointRangeQuery, PointWindow,
                                  QueryConfiguration, QueryType, UniformGrid)
    grid = UniformGrid(100, *BJ)
    conf = QueryConfiguration(QueryType.WindowBased, 10, 5, 0, False)
    x, y = synth.uniform(50000, 1)
    w = PointWindow(x, y)
    got = PointPointRangeQuery(conf, grid, ctx).run(w, Point(*Q), 0.5)
    cg = cref.grid(grid.minX, grid.minY, grid.cellLength, grid.numGridPartitions)
    assert got.tolist() == sorted(cref.range_pp(cg, x, y, Q[0], Q[1], 0.5).tolist())
    oi, od = PointPointKNNQuery(conf, grid, ctx).run(w, Point(*Q), 0.5, 10)
    wi, _ = cref.knn_pp(cg, x, y, Q[0], Q[1], 0.5, 10)
    assert oi.tolist() == wi.tolist()
