"""Point-polygon range and join on dense overlap: 3000 star polygons of radius 0.02-0.05 deg over
the C4 grid (500 x 500), ~6.5 pairs per point -- the window that made every 4096-point chunk of
the round-5 stream overflow its LDS stage and re-run, and whose candidates overflowed the first
call's candidate buffer (the step ran twice).

Now: a wave whose LDS region fills flushes it early (no chunk re-runs), and candidates past the
buffer are decided by the redo pass of the same call (no second pass).  The first call of a fresh
ctx (candidate buffer at n / 16) and a warm call both match the C oracle's pair count and 64-bit digest
(PointPolygonRangeQuery.java:76-124, PointPolygonJoinQuery.java:162-201).  The window is the C4
window's density at 1.5M points (the oracle finishes in seconds).
"""
import numpy as np
import pytest

import cref
from helpers import pair_digest
from spatialflink_amd import Context, _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING


@pytest.fixture(scope="module")
def dense():
    import torch
    l = (BJ[1] - BJ[0]) / 500
    ag, cg = _abi.make_grid(BJ[0], BJ[2], l, 500), cref.grid(BJ[0], BJ[2], l, 500)
    off, vx, vy = synth.star_polygons(3000, 7, r_min=0.02, r_max=0.05)
    hx, hy = synth.uniform(1_500_000, 5)
    x = torch.from_numpy(hx).cuda()
    y = torch.from_numpy(hy).cuda()
    return ag, cg, off, vx, vy, hx, hy, x, y


@pytest.mark.parametrize("join", [False, True])
def test_dense_overlap_one_pass(dense, join):
    import torch
    ag, cg, off, vx, vy, hx, hy, x, y = dense
    want = (cref.join_ppoly_hash(cg, cg, hx, hy, off, vx, vy, 0.005) if join
            else cref.range_ppoly_hash(cg, hx, hy, off, vx, vy, 0.005))
    assert want[0] > 5 * len(hx)  # the dense shape: ~6.5 pairs per point (3000 polygons)
    c = Context(0)  # fresh: the first call's candidate buffer is n / 16, far too small here
    out = torch.empty((want[0] + 64, 2), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for rep in range(2):
        cnt.zero_()
        if join:
            c.join_ppoly_async(ag, ag, x, y, off, vx, vy, 0.005, False, out, cnt)
        else:
            c.range_ppoly_async(ag, x, y, off, vx, vy, 0.005, False, out, cnt)
        c.sync()
        m = int(cnt.item())
        assert (m, pair_digest(out[:m])[1]) == want, f"call {rep}"
    # the synchronous form on another fresh ctx (host pairs)
    c2 = Context(0)
    got = (c2.join_ppoly(ag, ag, x, y, off, vx, vy, 0.005) if join else c2.range_ppoly(ag, x, y, off, vx, vy, 0.005))
    assert (len(got), pair_digest(got)[1]) == want


def test_stacked_polygons_fill_the_spill_lists():
    """800 star polygons stacked over one small area: each of its cells lists ~800 polygons, far
    more than the 16 entries per point a wave's spill list holds, so the waves' candidates pass
    their spill lists and whole chunks go to the redo pass (besides those past the candidate
    buffer).  Range and join, async twice on one ctx and the synchronous form, against the oracle's
    pair count and digest."""
    import torch
    l = (BJ[1] - BJ[0]) / 500
    ag, cg = _abi.make_grid(BJ[0], BJ[2], l, 500), cref.grid(BJ[0], BJ[2], l, 500)
    cx, cy = 116.40, 39.90
    off, vx, vy = synth.star_polygons(800, 9, n_vert=7, bbox=(cx - 0.005, cx + 0.005, cy - 0.005, cy + 0.005),
                                      r_min=0.03, r_max=0.05)
    rng = np.random.default_rng(10)
    hx = rng.uniform(cx - 0.06, cx + 0.06, 300_000)
    hy = rng.uniform(cy - 0.06, cy + 0.06, 300_000)
    x, y = torch.from_numpy(hx).cuda(), torch.from_numpy(hy).cuda()
    for join in (False, True):
        want = (cref.join_ppoly_hash(cg, cg, hx, hy, off, vx, vy, 0.005) if join
                else cref.range_ppoly_hash(cg, hx, hy, off, vx, vy, 0.005))
        assert want[0] > 50 * len(hx)  # ~hundreds of polygons per point
        c = Context(0)
        out = torch.empty((want[0] + 64, 2), dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        for rep in range(2):
            cnt.zero_()
            if join:
                c.join_ppoly_async(ag, ag, x, y, off, vx, vy, 0.005, False, out, cnt)
            else:
                c.range_ppoly_async(ag, x, y, off, vx, vy, 0.005, False, out, cnt)
            c.sync()
            m = int(cnt.item())
            assert (m, pair_digest(out[:m])[1]) == want, f"join={join} call {rep}"
        c2 = Context(0)
        got = (c2.join_ppoly(ag, ag, x, y, off, vx, vy, 0.005) if join else c2.range_ppoly(ag, x, y, off, vx, vy, 0.005))
        assert (len(got), pair_digest(got)[1]) == want
