"""Full-scale parity: BASELINE.json configs C3, C4 and the C5 shard at their own sizes.

The HIP path (through the C ABI, device-resident windows) against the multithreaded C oracle
(oracle/geohip_oracle.c, OpenMP; test infrastructure only).  Pair sets of up to 4.4e8 pairs are
compared by their exact count and an order-independent 64-bit digest (sum over pairs of
mix64(first << 32 | second) mod 2^64, computed on the device by torch for the product output
and by the oracle for the reference semantics), so no pair list needs sorting or copying.
  C3  point-point join, 10k queries x 10M Gaussian data points (32 centres, sigma 0.1), 500x500,
      r = 0.05  (PointPointJoinQuery.java:113-172)
  C4  point-polygon range, 1k star polygons x 50M uniform points, 500x500, r = 0.005
      (PointPolygonRangeQuery.java:76-124); the join form of the same shape
      (PointPolygonJoinQuery.java:162-201)
  C5  one 25M-point shard, 1000x1000, kNN k = 100 + range r = 0.05 of the README query
      (PointPointKNNQuery.java:125-191, PointPointRangeQuery.java:86-137)
"""
import numpy as np
import pytest

import cref
from helpers import MASK, pair_digest
from spatialflink_amd import _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING
Q = synth.README_QUERY


def agrid(n):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


def test_digest_matches_oracle_mix(ctx):
    """The torch digest is the oracle's mix64, including wrap-around and the top bit."""
    import torch
    rng = np.random.default_rng(7)
    a = rng.integers(0, 1 << 32, 5000, dtype=np.uint64)
    b = rng.integers(0, 1 << 32, 5000, dtype=np.uint64)
    a[:3] = [0, 0xFFFFFFFF, 0x80000000]
    b[:3] = [0, 0xFFFFFFFF, 1]
    want = sum(cref.mix64(int(p) << 32 | int(q)) for p, q in zip(a, b)) & MASK
    t = torch.from_numpy(np.stack([a, b], 1).astype(np.uint32).view(np.int32)).cuda()
    assert pair_digest(t, chunk=1024) == (5000, want)


def _device_uniform(ctx, n, seed):
    import torch
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_uniform_async(x, y, 0, seed, BJ)
    torch.cuda.synchronize()
    return x, y


def test_c3_join_full_scale(ctx):
    """C3 at its own size: 10k queries x 10M Gaussian data points, sigma 0.1, 500x500, r = 0.05."""
    import torch
    hx, hy = synth.gaussian_clusters(10_000_000, 3, sigma=0.1)
    hqx, hqy = synth.gaussian_clusters(10_000, 4, sigma=0.1)
    ag, cg = agrid(500)
    want = cref.join_pp_hash(cg, cg, hx, hy, hqx, hqy, 0.05)
    assert want[0] > 4e8  # ~4.4e8 pairs at sigma 0.1
    dx, dy = torch.from_numpy(hx).cuda(), torch.from_numpy(hy).cuda()
    qx, qy = torch.from_numpy(hqx).cuda(), torch.from_numpy(hqy).cuda()
    out = torch.empty((want[0] + 16, 2), dtype=torch.int32, device="cuda")
    got = ctx.join_pp(ag, ag, dx, dy, qx, qy, 0.05, out=out)
    assert pair_digest(got) == want
    del out, got
    assert ctx.join_pp_count(ag, ag, dx, dy, qx, qy, 0.05) == want[0]


@pytest.fixture(scope="module")
def c4_window(ctx):
    x, y = _device_uniform(ctx, 50_000_000, 5)
    hx, hy = x.cpu().numpy(), y.cpu().numpy()
    off, vx, vy = synth.star_polygons(1000, 6)
    return x, y, hx, hy, off, vx, vy


def test_c4_range_ppoly_full_scale(ctx, c4_window):
    """C4 at its own size: all 1k polygons (50 vertices) x 50M uniform points, 500x500, r = 0.005."""
    import torch
    x, y, hx, hy, off, vx, vy = c4_window
    ag, cg = agrid(500)
    want = cref.range_ppoly_hash(cg, hx, hy, off, vx, vy, 0.005)
    assert want[0] > 1e7
    out = torch.empty((want[0] + 16, 2), dtype=torch.int32, device="cuda")
    got = ctx.range_ppoly(ag, x, y, off, vx, vy, 0.005, out=out)
    assert pair_digest(got) == want


def test_c4_join_ppoly_full_scale(ctx, c4_window):
    """The join form of C4 (PointPolygonJoinQuery): every G u C pair distance-checked."""
    import torch
    x, y, hx, hy, off, vx, vy = c4_window
    ag, cg = agrid(500)
    want = cref.join_ppoly_hash(cg, cg, hx, hy, off, vx, vy, 0.005)
    out = torch.empty((want[0] + 16, 2), dtype=torch.int32, device="cuda")
    got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, 0.005, out=out)
    assert pair_digest(got) == want


def test_c5_shard_knn_and_range_full_scale(ctx):
    """C5 shard: 25M uniform points (rank 0's slice of the 200M window), 1000x1000, kNN k = 100
    and range r = 0.05 of the README query: exact (idx, distance bits) and the exact hit list."""
    x, y = _device_uniform(ctx, 25_000_000, 7)
    hx, hy = x.cpu().numpy(), y.cpu().numpy()
    ag, cg = agrid(1000)
    oi, od = ctx.knn_pp(ag, x, y, Q[0], Q[1], 0.05, 100)
    wi, wd = cref.knn_pp(cg, hx, hy, Q[0], Q[1], 0.05, 100)
    assert len(wi) == 100
    assert oi.cpu().numpy().astype(np.uint32).tolist() == wi.tolist()
    assert np.array_equal(od.cpu().numpy().view(np.uint64), wd.view(np.uint64))
    got = ctx.range_pp(ag, x, y, Q[0], Q[1], 0.05)
    want = cref.range_pp(cg, hx, hy, Q[0], Q[1], 0.05)
    assert got.cpu().numpy().astype(np.uint32).tolist() == want.tolist()
    assert len(want) > 5e4
    # the fused one-pass form of the C5 step (geohip_knn_range_pp)
    (fi, fd), fr = ctx.knn_range_pp(ag, x, y, Q[0], Q[1], 0.05, 100)
    assert fi.cpu().numpy().astype(np.uint32).tolist() == wi.tolist()
    assert np.array_equal(fd.cpu().numpy().view(np.uint64), wd.view(np.uint64))
    assert fr.cpu().numpy().astype(np.uint32).tolist() == want.tolist()


def test_c5_as_configured_200m_window_eight_shards(ctx):
    """BASELINE configs[4] as configured: one 200M-point window (3.2 GB, on one device) split into
    eight 25M-point shards, each evaluated by the fused kNN (k = 100) + range (r = 0.05) pass
    (geohip_knn_range_pp_async, the per-GPU step of the 8-GPU job), the eight top-k lists merged
    by geohip_knn_merge_async (the windowAll merge, KNNQuery.java:204-272) and the range hits
    concatenated in shard order -- against the oracle over the whole window: kNN indices and
    distance bits, the exact range hit list."""
    import torch
    n, S, k, r = 200_000_000, 8, 100, 0.05
    per = n // S
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ctx.synth_uniform_async(x, y, 0, 7, BJ)
    ag, cg = agrid(1000)
    ki = torch.empty((S, k), dtype=torch.int32, device="cuda")
    kd = torch.empty((S, k), dtype=torch.float64, device="cuda")
    kc = torch.zeros(S + 1, dtype=torch.int32, device="cuda")
    cap = 1 << 21
    ro = torch.empty((S, cap), dtype=torch.int32, device="cuda")
    rc = torch.zeros(S, dtype=torch.int64, device="cuda")
    for s in range(S):
        xs, ys = x[s * per:(s + 1) * per], y[s * per:(s + 1) * per]
        ctx.knn_range_pp_async(ag, xs, ys, Q[0], Q[1], r, k, False, ki[s], kd[s], kc[s:s + 1], ro[s], cap,
                               rc[s:s + 1])
    base = (torch.arange(S, dtype=torch.int32, device="cuda") * per).view(S, 1)
    ki = torch.where(ki >= 0, ki + base, ki).contiguous()
    mi = torch.empty(k, dtype=torch.int32, device="cuda")
    md = torch.empty(k, dtype=torch.float64, device="cuda")
    ctx.knn_merge_async(kd, ki, S, k, k, mi, md, kc[S:])
    counts = rc.cpu().tolist()
    assert max(counts) <= cap
    hits = torch.cat([ro[s, :counts[s]].to(torch.int64) + s * per for s in range(S)]).cpu().numpy()
    got_i, got_d = mi.cpu().numpy().astype(np.uint32), md.cpu().numpy()
    assert int(kc[S].item()) == k
    hx, hy = x.cpu().numpy(), y.cpu().numpy()
    del x, y
    wi, wd = cref.knn_pp(cg, hx, hy, Q[0], Q[1], r, k)
    assert got_i.tolist() == wi.tolist()
    assert np.array_equal(got_d.view(np.uint64), wd.view(np.uint64))
    want = cref.range_pp(cg, hx, hy, Q[0], Q[1], r)
    assert len(want) > 4e5
    assert hits.tolist() == want.astype(np.int64).tolist()
