"""GPU: the key-band point-query pieces on the device.

geohip_band_pack_query_async (the reference's G u C filter before keyBy(gridID),
PointPointKNNQuery.java:137-151 / PointPointRangeQuery.java:102-116) against its torch
restatement distributed.torch_band_pack_query (the planner's boxes evaluated on the host through
geohip_debug_classify, the owner of key band (cx * W) // n, arrival order inside each owner):
same points, same owners, same order, same counts -- with NaN points, points on cell edges of the
query's box, out-of-grid points, r = 0 and r < 0 (the planner's cells for a negative radius, as
the range query takes it).  And distributed.knn_range_cells with its
default device callables (band pack, knn_range_pp, merge) at world 1 against the oracle.
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import cref  # noqa: E402  (oracle: the checker)
from spatialflink_amd import _abi, synth  # noqa: E402
from spatialflink_amd import distributed as D  # noqa: E402

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING
Q = synth.README_QUERY


def _window(n, seed, grid_n):
    rng = np.random.default_rng(seed)
    x, y = synth.uniform(n, seed)
    l = (BJ[1] - BJ[0]) / grid_n
    # points exactly on the cell edges around the query (the planner's box boundaries)
    cq = int((Q[0] - BJ[0]) / l)
    edges = BJ[0] + (cq + np.arange(-8, 9)) * l
    k = min(len(x) // 4, 4000)
    x[:k] = rng.choice(edges, k)
    y[:k] = Q[1] + rng.uniform(-0.3, 0.3, k)
    y[k:2 * k] = BJ[2] + (int((Q[1] - BJ[2]) / l) + rng.integers(-8, 9, k)) * l
    x[2 * k:2 * k + 50] = np.nan
    y[2 * k + 50:2 * k + 100] = np.nan
    x[2 * k + 100:2 * k + 150] = BJ[1] + 1.0  # out of the grid
    return x, y


@pytest.mark.parametrize("grid_n,r,world", [(100, 0.5, 4), (1000, 0.05, 8), (100, 0.0, 3), (500, 0.02, 1),
                                            (100, -0.1, 2)])
def test_band_pack_query_matches_torch(ctx, grid_n, r, world):
    import torch
    l = (BJ[1] - BJ[0]) / grid_n
    ag = _abi.make_grid(BJ[0], BJ[2], l, grid_n)
    x, y = _window(200_003, 7 + grid_n, grid_n)
    xd = torch.from_numpy(x).to("cuda:0")
    yd = torch.from_numpy(y).to("cuda:0")
    base = 12345
    ox, oy, oi, cnt = ctx.band_pack_query_async(ag, grid_n, world, Q[0], Q[1], r, xd, yd, base)
    torch.cuda.synchronize()
    tx, ty, ti, tc = D.torch_band_pack_query(ag, Q[0], Q[1], r)(torch.from_numpy(x), torch.from_numpy(y), base,
                                                                 grid_n, world)
    m = int(tc.sum())
    assert cnt.cpu().tolist() == tc.tolist()
    assert np.array_equal(oi[:m].cpu().numpy(), ti.numpy())
    assert np.array_equal(ox[:m].cpu().numpy().view(np.uint64), tx.numpy().view(np.uint64))
    assert np.array_equal(oy[:m].cpu().numpy().view(np.uint64), ty.numpy().view(np.uint64))
    assert m > 0 or r <= 0.0


def test_band_pack_query_empty_window(ctx):
    import torch
    ag = _abi.make_grid(BJ[0], BJ[2], (BJ[1] - BJ[0]) / 100, 100)
    e = torch.empty(0, dtype=torch.float64, device="cuda:0")
    ox, oy, oi, cnt = ctx.band_pack_query_async(ag, 100, 4, Q[0], Q[1], 0.5, e, e, 0)
    torch.cuda.synchronize()
    assert cnt.cpu().tolist() == [0, 0, 0, 0] and len(oi) == 0


@pytest.mark.parametrize("grid_n,r,k", [(100, 0.5, 50), (1000, 0.05, 100)])
def test_knn_range_cells_device_world1(ctx, grid_n, r, k):
    """knn_range_cells with the default device callables (no stand-ins) at world 1 vs the oracle."""
    import torch
    l = (BJ[1] - BJ[0]) / grid_n
    ag = _abi.make_grid(BJ[0], BJ[2], l, grid_n)
    cg = cref.grid(BJ[0], BJ[2], l, grid_n)
    x, y = _window(300_007, 11 + grid_n, grid_n)
    xd, yd = torch.from_numpy(x).to("cuda:0"), torch.from_numpy(y).to("cuda:0")
    res, (hits, off, total), nrecv = D.knn_range_cells(xd, yd, 0, Q[0], Q[1], r, k, grid=ag, ctx=ctx)
    wi, wd = cref.knn_pp(cg, x, y, Q[0], Q[1], r, k)
    assert res.idx.cpu().numpy().astype(np.int64).tolist() == np.asarray(wi, np.int64).tolist()
    assert np.array_equal(res.dist.cpu().numpy().view(np.uint64), np.asarray(wd, np.float64).view(np.uint64))
    want = np.sort(cref.range_pp(cg, x, y, Q[0], Q[1], r)).astype(np.int64)
    assert off == 0 and total == len(want)
    assert np.array_equal(np.sort(hits.cpu().numpy().astype(np.int64)), want)


@pytest.mark.parametrize("grid_n,r,k", [(100, 0.5, 50), (1000, 0.05, 100)])
def test_knn_range_cells_world1_forms(ctx, grid_n, r, k):
    """World 1: the default shortcut (no pack: the kNN pass filters), a caller's band pack (the
    device pack, then the identity exchange) and the enqueue-only form into preallocated rows
    (no host round trip until result()) all give the same top-k, distance bits and hits."""
    import torch
    l = (BJ[1] - BJ[0]) / grid_n
    ag = _abi.make_grid(BJ[0], BJ[2], l, grid_n)
    x, y = _window(300_007, 21 + grid_n, grid_n)
    xd, yd = torch.from_numpy(x).to("cuda:0"), torch.from_numpy(y).to("cuda:0")
    base = 1000

    def packed(xs, ys, b, nb, w):
        return ctx.band_pack_query_async(ag, nb, w, Q[0], Q[1], r, xs, ys, b)
    a = D.knn_range_cells(xd, yd, base, Q[0], Q[1], r, k, grid=ag, ctx=ctx)
    p = D.knn_range_cells(xd, yd, base, Q[0], Q[1], r, k, grid=ag, ctx=ctx, band_pack=packed)
    bufs = D.CellsBuffers(k, len(x), 1, xd.device)
    e = D.knn_range_cells(xd, yd, base, Q[0], Q[1], r, k, grid=ag, ctx=ctx, bufs=bufs).result()
    ra, (ha, _, ta), na = a
    for rb, (hb, _, tb), nbv in (p, e):
        assert rb.count == ra.count
        assert rb.idx.cpu().tolist() == ra.idx.cpu().tolist()
        assert torch.equal(rb.dist.cpu().view(torch.int64), ra.dist.cpu().view(torch.int64))
        assert tb == ta and sorted(hb.cpu().tolist()) == sorted(ha.cpu().tolist())
    assert na == len(x) and e[2] == len(x)
    assert p[2] < len(x)  # the pack kept the G u C candidates only
