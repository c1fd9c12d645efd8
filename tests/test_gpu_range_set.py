"""Point-point range with unordered-set output (geohip_ctx_set_range_order GEOHIP_ORDER_ANY,
the range_set kernel) against the C oracle.

The reference's window result is a set (PointPointRangeQuery.java:117-136), so these tests compare
SORTED index lists: the same hits, each exactly once, no order promised.  Every case the ascending
mode's parity tests cover (golden vectors, NaN / out-of-grid points, r = 0 / r < 0 / NaN, window
sizes around the 256-point iteration and past one 1024-hit run, approximate mode, two-phase
capacity, panes' point_base) plus what is particular to the set kernel: back-to-back launches on
one ctx (the reservation cursor re-armed by each launch's last block) interleaved with the
ascending mode (shared look-back scratch) and with async calls, and the C1 shape at 10M points
against the ascending mode.
"""
import math

import numpy as np
import pytest

import cref
from helpers import arr, fx, grid_vals
from spatialflink_amd import Context, _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING
Q = synth.README_QUERY


def agrid(n):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


@pytest.fixture(scope="module")
def sctx():
    c = Context(0)
    c.set_range_order(True)
    return c


def _window(rng, n, nan_every=0):
    x = rng.uniform(BJ[0] - 0.1, BJ[1] + 0.1, n)
    y = rng.uniform(BJ[2] - 0.1, BJ[3] + 0.1, n)
    if nan_every:
        x[::nan_every] = np.nan
        y[3::nan_every] = np.nan
    return x, y


def _same_set(got, want):
    g = np.sort(np.asarray(got).astype(np.int64))
    assert len(np.unique(g)) == len(g), "an index emitted twice"
    assert g.tolist() == sorted(np.asarray(want).astype(np.int64).tolist())


def test_range_set_golden(sctx, golden):
    for c in golden["range_pp"]:
        g = _abi.make_grid(*grid_vals(c["grid"]))
        got = sctx.range_pp(g, arr(c["x"]), arr(c["y"]), fx(c["qx"]), fx(c["qy"]), fx(c["r"]), c["approximate"])
        _same_set(got, c["expect"])


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 1024, 4097, 70001, 300_000])
def test_range_set_sizes(sctx, n):
    rng = np.random.default_rng(n + 11)
    x, y = _window(rng, n, nan_every=53)
    ag, cg = agrid(100)
    _same_set(sctx.range_pp(ag, x, y, Q[0], Q[1], 0.5), cref.range_pp(cg, x, y, Q[0], Q[1], 0.5))


RANGE_CASES = [(100, 0.5, Q, False), (100, 0.05, Q, False), (500, 0.05, (116.3, 40.2), False),
               (1000, 0.05, Q, False), (100, 0.5, Q, True), (37, 0.3, (115.45, 39.55), False),
               (100, 0.0, Q, False), (100, -1.0, Q, False), (100, math.nan, Q, False),
               (10, 2.0, (116.5, 40.3), False), (100, 0.03, (117.7, 41.3), False), (10, 2.0, (116.5, 40.3), True)]


@pytest.mark.parametrize("case", range(len(RANGE_CASES)))
def test_range_set_random(sctx, case):
    gn, r, q, approx = RANGE_CASES[case]
    rng = np.random.default_rng(300 + case)
    x, y = _window(rng, 200000, nan_every=997)
    ag, cg = agrid(gn)
    _same_set(sctx.range_pp(ag, x, y, q[0], q[1], r, approx), cref.range_pp(cg, x, y, q[0], q[1], r, approx))


def test_range_set_capacity_and_pane(sctx):
    rng = np.random.default_rng(7)
    x, y = _window(rng, 60000)
    ag, cg = agrid(100)
    want = cref.range_pp(cg, x, y, Q[0], Q[1], 0.5)
    with pytest.raises(_abi.GeohipCapacityError):
        sctx.range_pp(ag, x, y, Q[0], Q[1], 0.5, cap=10)
    _same_set(sctx.range_pp(ag, x, y, Q[0], Q[1], 0.5, cap=len(want)), want)
    base = (1 << 32) - 20000  # pane stream positions wrap inside the pane
    got = sctx.range_pp(ag, x, y, Q[0], Q[1], 0.5, point_base=base)
    _same_set((np.asarray(got).astype(np.int64) - base) & 0xFFFFFFFF, want)


def test_range_set_async_back_to_back_and_mixed_orders(sctx):
    """Async set-mode launches back to back on one ctx (each re-arms the cursor for the next),
    then the ascending mode on the same ctx, then the set mode again."""
    import torch
    ag, cg = agrid(100)
    wins = [synth.uniform(500_000 + 37 * w, 40 + w) for w in range(4)]
    wants = [cref.range_pp(cg, hx, hy, Q[0], Q[1], 0.3) for hx, hy in wins]
    dev = [(torch.from_numpy(hx).cuda(), torch.from_numpy(hy).cuda()) for hx, hy in wins]
    outs = [torch.full((len(w) + 64,), -1, dtype=torch.int32, device="cuda") for w in wants]
    cnt = torch.zeros(4, dtype=torch.int64, device="cuda")
    for rep in range(2):
        for w in range(4):
            sctx.range_pp_async(ag, dev[w][0], dev[w][1], Q[0], Q[1], 0.3, False, outs[w], len(outs[w]),
                                cnt[w:w + 1])
        sctx.sync()
        for w in range(4):
            m = int(cnt[w].item())
            assert m == len(wants[w])
            _same_set(outs[w][:m].cpu().numpy(), wants[w])
            assert (outs[w][m:] == -1).all()  # nothing written past the set
        sctx.set_range_order(False)
        for w in range(4):
            assert sctx.range_pp(ag, *wins[w], Q[0], Q[1], 0.3).tolist() == sorted(wants[w].tolist())
        sctx.set_range_order(True)


def test_range_set_c1_shape_10m(sctx, ctx):
    """BASELINE configs[0]'s query at the bench's 10M points per window: the set equals the
    ascending mode's result (size-independent: same count, same sorted indices)."""
    import torch
    ag, _ = agrid(100)
    n = 10_000_000
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    sctx.synth_uniform_async(x, y, 0, 1, BJ)
    got = sctx.range_pp(ag, x, y, Q[0], Q[1], 0.5)
    want = ctx.range_pp(ag, x, y, Q[0], Q[1], 0.5)
    g = torch.sort(torch.as_tensor(got).to(torch.int64).cuda()).values
    w = torch.as_tensor(want).to(torch.int64).cuda()
    assert len(g) == len(w) > 2_000_000
    assert torch.equal(g, w)


def test_range_set_order_argument():
    c = Context(0)
    with pytest.raises(_abi.GeohipArgumentError):
        _abi.Context._check(c, _abi.lib.geohip_ctx_set_range_order(c.h, 7), "set_range_order")


# ---- the fused kNN + range pass (geohip_knn_range_pp, the C5 step) with the unordered range ----
KR_CASES = [(1000, 0.05, Q, 100, False), (100, 0.5, Q, 50, False), (500, 0.05, (116.3, 40.2), 64, False),
            (100, 0.5, Q, 50, True), (37, 0.3, (115.45, 39.55), 10, False), (100, 0.0, Q, 5, False),
            (100, math.nan, Q, 7, False), (100, 0.03, (117.7, 41.3), 3, False), (100, 0.2, (116.0, 40.5), 1000, False)]


@pytest.mark.parametrize("case", range(len(KR_CASES)))
@pytest.mark.parametrize("n", [300000, 1025, 0])
def test_knn_range_fused_set(sctx, case, n):
    """The unordered fused pass sweeps the window in interleaved fronts (its hit bitmask follows
    each block's fronts): the kNN bits and the range set equal the oracle's."""
    gn, r, q, k, approx = KR_CASES[case]
    rng = np.random.default_rng(500 + case)
    x, y = _window(rng, n, nan_every=1009)
    ag, cg = agrid(gn)
    (oi, od), got = sctx.knn_range_pp(ag, x, y, q[0], q[1], r, k, approx)
    wi, wd = cref.knn_pp(cg, x, y, q[0], q[1], r, k)
    assert oi.tolist() == wi.tolist()
    assert np.array_equal(od.view(np.uint64), wd.view(np.uint64))
    _same_set(got, cref.range_pp(cg, x, y, q[0], q[1], r, approx))


def test_knn_range_fused_set_c5_shard(sctx, ctx):
    """The C5 shard (25M points, 1000 x 1000, k = 100, r = 0.05) through the async form twice on
    one ctx (the reservation cursor re-armed by each launch's last block): the
    kNN equals the ordered pass's bit for bit, the range hits are the same set."""
    import torch
    ag, _ = agrid(1000)
    n = 25_000_000
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    sctx.synth_uniform_async(x, y, 0, 7, BJ)
    (wi, wd), want = ctx.knn_range_pp(ag, x, y, Q[0], Q[1], 0.05, 100)
    want = torch.as_tensor(want).to(torch.int64).cuda()
    ki = torch.empty(100, dtype=torch.int32, device="cuda")
    kd = torch.empty(100, dtype=torch.float64, device="cuda")
    kc = torch.zeros(1, dtype=torch.int32, device="cuda")
    ro = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    rc = torch.zeros(1, dtype=torch.int64, device="cuda")
    for _ in range(2):
        sctx.knn_range_pp_async(ag, x, y, Q[0], Q[1], 0.05, 100, False, ki, kd, kc, ro, n, rc)
        sctx.sync()
        m = int(rc.item())
        assert int(kc.item()) == 100 and m == len(want) > 10_000
        assert torch.equal(ki.cpu().to(torch.int64), torch.as_tensor(wi).cpu().to(torch.int64))
        assert torch.equal(kd.cpu().view(torch.int64), torch.as_tensor(wd).cpu().view(torch.int64))
        assert torch.equal(torch.sort(ro[:m].to(torch.int64)).values, want)
