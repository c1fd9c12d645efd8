"""The enqueue-only join and point-polygon forms (geohip_join_pp_async, geohip_range_ppoly_async,
geohip_join_ppoly_async) against the synchronous forms and the C oracle.

They write the pair total to a device word and return without a host round trip; what a
synchronous call would return as a status surfaces at geohip_ctx_sync: a query key the reference
cannot parse back (PointPointJoinQuery.java:125 -> UniformGrid.getNeighboringCells ->
HelperClass.getIntCellIndices, NumberFormatException).  A point-polygon candidate buffer that
the previous call sized too small is no error: the stream decides the candidates past it, and the
need it reports sizes the next call's buffer.
"""
import numpy as np
import pytest

import cref
from helpers import pair_digest, pairs_sorted
from spatialflink_amd import Context, _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING


def agrid(n):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


def _dev(*arrs):
    import torch
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def test_join_pp_async_back_to_back(ctx):
    """Two windows enqueued back to back (no host synchronisation between them), then one sync:
    each window's pair set equals the oracle's; a short buffer holds a prefix of valid pairs and
    the count still says the total."""
    import torch
    ag, cg = agrid(500)
    wins = [synth.gaussian_clusters(400_000, 51 + w, sigma=0.05) for w in range(2)]
    hqx, hqy = synth.gaussian_clusters(800, 53, sigma=0.05)
    qx, qy = _dev(hqx, hqy)
    want = [cref.join_pp_hash(cg, cg, hx, hy, hqx, hqy, 0.03) for hx, hy in wins]
    outs = [torch.empty((w[0] + 8, 2), dtype=torch.int32, device="cuda") for w in want]
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    dev = [_dev(hx, hy) for hx, hy in wins]
    for w in range(2):
        ctx.join_pp_async(ag, ag, dev[w][0], dev[w][1], qx, qy, 0.03, False, outs[w], cnt[w:w + 1])
    ctx.sync()
    for w in range(2):
        m = int(cnt[w].item())
        assert (m, pair_digest(outs[w][:m])[1]) == want[w]
    short = torch.empty((want[0][0] // 2, 2), dtype=torch.int32, device="cuda")
    ctx.join_pp_async(ag, ag, dev[0][0], dev[0][1], qx, qy, 0.03, False, short, cnt[0:1])
    ctx.sync()
    assert int(cnt[0].item()) == want[0][0]
    full = pairs_sorted(cref.join_pp(cg, cg, *wins[0], hqx, hqy, 0.03))
    got = pairs_sorted(short.cpu().numpy())
    # every written pair is a pair of the window, no pair twice
    assert len(np.unique(got, axis=0)) == len(got)
    keys = full[:, 0] * 100000 + full[:, 1]
    assert np.isin(got[:, 0] * 100000 + got[:, 1], keys).all()


def test_join_pp_async_approx_and_query_key_error(ctx):
    import torch
    ag, cg = agrid(200)
    hx, hy = synth.uniform(200_000, 61)
    hqx, hqy = synth.uniform(300, 62)
    want = cref.join_pp_hash(cg, cg, hx, hy, hqx, hqy, 0.04, True)
    dx, dy, qx, qy = _dev(hx, hy, hqx, hqy)
    out = torch.empty((want[0] + 8, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.join_pp_async(ag, ag, dx, dy, qx, qy, 0.04, True, out, cnt)
    ctx.sync()
    m = int(cnt.item())
    assert (m, pair_digest(out[:m])[1]) == want
    # a query whose key "%05d%05d" does not split back into two ints (cx = 123456, cy = -3):
    # the synchronous join raises, the async one reports at sync (and the ctx stays usable)
    l = (BJ[1] - BJ[0]) / 200
    bad = np.array([BJ[0] + 123456.5 * l]), np.array([BJ[2] - 2.5 * l])
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.join_pp(ag, ag, hx, hy, *bad, 0.04)
    bqx, bqy = _dev(*bad)
    ctx.join_pp_async(ag, ag, dx, dy, bqx, bqy, 0.04, False, out, cnt)
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.sync()
    ctx.sync()  # cleared
    ctx.join_pp_async(ag, ag, dx, dy, qx, qy, 0.04, True, out, cnt)
    ctx.sync()
    assert (int(cnt.item()), pair_digest(out[:int(cnt.item())])[1]) == want


def test_sync_range_leaves_async_fault_for_ctx_sync(ctx):
    """A synchronous range / kNN call consumes only its own look-back fault: an earlier async
    join's query-key fault neither fails it nor is cleared by it; geohip_ctx_sync reports it."""
    ag, cg = agrid(200)
    hx, hy = synth.uniform(100_000, 63)
    dx, dy = _dev(hx, hy)
    import torch
    out = torch.empty((1024, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    l = (BJ[1] - BJ[0]) / 200
    bqx, bqy = _dev(np.array([BJ[0] + 123456.5 * l]), np.array([BJ[2] - 2.5 * l]))
    ctx.join_pp_async(ag, ag, dx, dy, bqx, bqy, 0.04, False, out, cnt)
    q = synth.README_QUERY
    got = ctx.range_pp(ag, hx, hy, q[0], q[1], 0.05)
    assert got.tolist() == sorted(cref.range_pp(cg, hx, hy, q[0], q[1], 0.05).tolist())
    gi, gd = ctx.knn_pp(ag, hx, hy, q[0], q[1], 0.05, 20)
    wi, wd = cref.knn_pp(cg, hx, hy, q[0], q[1], 0.05, 20)
    assert gi.tolist() == wi.tolist()
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.sync()
    ctx.sync()  # cleared


@pytest.mark.parametrize("join,approx", [(False, False), (False, True), (True, False)])
def test_ppoly_async_matches_sync(ctx, join, approx):
    import torch
    ag, cg = agrid(500)
    off, vx, vy = synth.star_polygons(300, 71)
    hx, hy = synth.uniform(2_000_000, 72)
    x, y = _dev(hx, hy)
    if join:
        want = cref.join_ppoly_hash(cg, cg, hx, hy, off, vx, vy, 0.005, approx)
    else:
        want = cref.range_ppoly_hash(cg, hx, hy, off, vx, vy, 0.005, approx)
    out = torch.empty((want[0] + 8, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    for rep in range(2):  # twice without a sync between: the plan cache and the count word
        if join:
            ctx.join_ppoly_async(ag, ag, x, y, off, vx, vy, 0.005, approx, out, cnt[rep:rep + 1])
        else:
            ctx.range_ppoly_async(ag, x, y, off, vx, vy, 0.005, approx, out, cnt[rep:rep + 1])
    ctx.sync()
    assert cnt.cpu().tolist() == [want[0], want[0]]
    assert pair_digest(out[:want[0]]) == want


def test_ppoly_async_candidate_overflow():
    """A fresh ctx sizes the candidate buffer at max(65536, n / 16); a window packed around
    polygon edges needs more.  The chunks whose candidates pass the buffer are decided by the redo
    pass of the same call, so the first call already returns the oracle's pairs in one pass and sync() reports no error; the
    need it reported sizes the next call's buffer (same pairs again)."""
    import torch
    c = Context(0)
    ag, cg = agrid(500)
    off, vx, vy = synth.star_polygons(2000, 81, r_min=0.004, r_max=0.01)
    rng = np.random.default_rng(82)
    # points about r outside each vertex (away from its polygon's centre): their subcells straddle
    # the distance-r curve, so each is a candidate for an exact test
    cx = np.repeat([vx[a:b].mean() for a, b in zip(off[:-1], off[1:])], np.diff(off))
    cy = np.repeat([vy[a:b].mean() for a, b in zip(off[:-1], off[1:])], np.diff(off))
    d = np.hypot(vx - cx, vy - cy)
    ox, oy = vx + (vx - cx) / d * 0.002, vy + (vy - cy) / d * 0.002
    hx = np.concatenate([ox + rng.normal(0, 0.0003, len(vx)) for _ in range(4)])
    hy = np.concatenate([oy + rng.normal(0, 0.0003, len(vy)) for _ in range(4)])
    assert len(hx) // 16 < 65536
    want = cref.range_ppoly_hash(cg, hx, hy, off, vx, vy, 0.002)
    x, y = _dev(hx, hy)
    out = torch.empty((want[0] + 8, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for _ in range(2):
        cnt.zero_()
        c.range_ppoly_async(ag, x, y, off, vx, vy, 0.002, False, out, cnt)
        c.sync()
        assert (int(cnt.item()), pair_digest(out[:int(cnt.item())])[1]) == want
    # the synchronous forms on a fresh ctx: first call over the buffer, one pass, same pairs
    c2 = Context(0)
    got = c2.range_ppoly(ag, hx, hy, off, vx, vy, 0.002)
    assert pairs_sorted(got).tolist() == pairs_sorted(cref.range_ppoly(cg, hx, hy, off, vx, vy, 0.002)).tolist()
    got = c2.join_ppoly(ag, ag, hx, hy, off, vx, vy, 0.002)
    assert pairs_sorted(got).tolist() == pairs_sorted(cref.join_ppoly(cg, cg, hx, hy, off, vx, vy, 0.002)).tolist()


def test_ppoly_pane_async(ctx):
    """geohip_range_ppoly_pane_async: the synchronous pane call's pairs (polygon, base + position),
    a base near 2^32 wrapping; IncrementalPPolyRange's enqueue-only pane."""
    import torch
    from spatialflink_amd.incremental import IncrementalPPolyRange
    ag, cg = agrid(500)
    off, vx, vy = synth.star_polygons(200, 91)
    hx, hy = synth.uniform(1_000_000, 92)
    x, y = _dev(hx, hy)
    want = cref.range_ppoly(cg, hx, hy, off, vx, vy, 0.005)
    base = (1 << 32) - 300_000
    out = torch.empty((len(want) + 8, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.range_ppoly_async(ag, x, y, off, vx, vy, 0.005, False, out, cnt, point_base=base)
    ctx.sync()
    m = int(cnt.item())
    got = out[:m].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    got[:, 1] = (got[:, 1] - base) & 0xFFFFFFFF
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
    inc = IncrementalPPolyRange(ctx, ag, off, vx, vy, 0.005)
    inc.push(x, y, out=out, count=cnt)
    ctx.sync()
    assert int(cnt.item()) == len(want)
