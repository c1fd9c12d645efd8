"""GPU parity of polygons with holes (Polygon.java:115-165 createPolygon)
through the C ABI: geohip_range_ppoly / geohip_join_ppoly with poly_rings and geohip_knn_ppoly
with ring_off, against the C oracle (itself checked against the literal restatement in
tests/test_oracle_ppoly.py and the golden holes fixtures).  Points in holes, on hole edges and
vertices, within r of a hole ring, NaN points; holes listed before the shell, padded
degenerate holes, holes crossing or outside the shell, clockwise holes, an open shell; 64, 65
and 201 rings (ring masks in chunks of 64); rings too long for LDS and too many segments for
slab lists; the reference's errors.
Parity unpinned beyond the restatement: the reference ships no holed-polygon test.
"""
import math

import numpy as np
import pytest

import cref
from helpers import arr, fx, golden_polygons, grid_vals, holed_window, pairs_sorted
from spatialflink_amd import _abi, synth

pytestmark = pytest.mark.gpu

BJ = synth.BEIJING


def agrid(n):
    l = (BJ[1] - BJ[0]) / n
    return _abi.make_grid(BJ[0], BJ[2], l, n), cref.grid(BJ[0], BJ[2], l, n)


CASES = [(500, 0.0005, False), (500, 0.003, False), (100, 0.01, False), (500, 0.003, True), (200, 0.0, False),
         (1000, 0.02, False)]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_range_and_join_holes(ctx, case):
    n, r, approx = CASES[case]
    rng = np.random.default_rng(400 + case)
    pr, off, vx, vy, polys = synth.holed_polygons(60, 410 + case)
    x, y = holed_window(rng, 300000, polys, max(r, 0.002))
    ag, cg = agrid(n)
    got = ctx.range_ppoly(ag, x, y, off, vx, vy, r, approx, poly_rings=pr)
    want = cref.range_ppoly(cg, x, y, off, vx, vy, r, approx, poly_rings=pr)
    assert len(want) > 1000 or r == 0
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
    got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, r, approx, poly_rings=pr)
    want = cref.join_ppoly(cg, cg, x, y, off, vx, vy, r, approx, poly_rings=pr)
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()


@pytest.mark.parametrize("case", [0, 1, 2, 3])
def test_knn_holes(ctx, case):
    n, r, approx = CASES[case]
    rng = np.random.default_rng(500 + case)
    pr, off, vx, vy, polys = synth.holed_polygons(6, 510 + case)
    x, y = holed_window(rng, 200000, polys, 0.003)
    ag, cg = agrid(n)
    for p in range(6):
        a, b = pr[p], pr[p + 1]
        ro = off[a:b + 1] - off[a]
        px, py = vx[off[a]:off[b]], vy[off[a]:off[b]]
        for k in (1, 37, 256):
            gi, gd = ctx.knn_ppoly(ag, x, y, px, py, r, k, approx, ring_off=ro)
            wi, wd = cref.knn_ppoly(cg, x, y, px, py, r, k, approx, ring_off=ro)
            assert gi.tolist() == wi.tolist()
            assert np.array_equal(gd.view(np.uint64), wd.view(np.uint64))


def _flat(rings):
    off, vx, vy = [0], [], []
    for ring in rings:
        vx += [c[0] for c in ring]
        vy += [c[1] for c in ring]
        off.append(len(vx))
    return np.array(off, np.uint32), np.array(vx), np.array(vy)


def test_many_and_long_rings(ctx):
    """64 rings (63 holes on a lattice); a 700-vertex shell (rings read from global memory,
    not LDS); a 31000-vertex shell (no slab lists: every segment visited)."""
    rng = np.random.default_rng(9)
    cx, cy, R = 116.4, 40.3, 0.05
    sq = [(cx - R, cy - R), (cx + R, cy - R), (cx + R, cy + R), (cx - R, cy + R)]
    holes = []
    for i in range(63):
        hx_, hy_ = cx - 0.8 * R + (i % 8) * 0.2 * R, cy - 0.8 * R + (i // 8) * 0.2 * R
        holes.append([(hx_, hy_), (hx_ + 0.06 * R, hy_), (hx_ + 0.06 * R, hy_ + 0.06 * R), (hx_, hy_ + 0.06 * R)])
    big = synth._star(rng, 116.8, 40.6, 0.04, 700)
    big_holes = [synth._star(rng, 116.8 + dx, 40.6, 0.006, 12) for dx in (-0.015, 0.0, 0.015)]
    huge = synth._star(rng, 116.0, 40.0, 0.05, 31000)
    huge_holes = [synth._star(rng, 116.0, 40.0 + dy, 0.008, 20) for dy in (-0.02, 0.02)]
    polys = [[sq] + holes, [big] + big_holes, [huge] + huge_holes]
    pr = np.array([0, 64, 68, 71], np.uint32)
    off, vx, vy = _flat([ring for rings in polys for ring in rings])
    x, y = holed_window(rng, 100000, polys[:2] + [huge_holes], 0.002)
    hv = np.array(huge[::97])  # a sample of the long shell's vertices, and points around it
    x = np.concatenate([x, hv[:, 0], rng.uniform(115.94, 116.06, 3000)])
    y = np.concatenate([y, hv[:, 1], rng.uniform(39.94, 40.06, 3000)])
    ag, cg = agrid(500)
    for r in (0.0004, 0.002):
        got = ctx.range_ppoly(ag, x, y, off, vx, vy, r, poly_rings=pr)
        want = cref.range_ppoly(cg, x, y, off, vx, vy, r, poly_rings=pr)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
        got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, r, poly_rings=pr)
        want = cref.join_ppoly(cg, cg, x, y, off, vx, vy, r, poly_rings=pr)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
    for p in range(3):
        a, b = pr[p], pr[p + 1]
        ro = off[a:b + 1] - off[a]
        px, py = vx[off[a]:off[b]], vy[off[a]:off[b]]
        gi, gd = ctx.knn_ppoly(ag, x, y, px, py, 0.002, 200, ring_off=ro)
        wi, wd = cref.knn_ppoly(cg, x, y, px, py, 0.002, 200, ring_off=ro)
        assert gi.tolist() == wi.tolist() and np.array_equal(gd.view(np.uint64), wd.view(np.uint64))


def _lattice_polygon(cx, cy, R, nh, rng):
    """A square shell with nh small holes: a lattice, every 7th hole overlapping its neighbour
    (a point in both is decided by the first in ring order), a few clockwise, some listed
    before the shell is the largest ring anyway."""
    sq = [(cx - R, cy - R), (cx + R, cy - R), (cx + R, cy + R), (cx - R, cy + R)]
    side = int(math.ceil(math.sqrt(nh)))
    step = 1.8 * R / side
    holes = []
    for i in range(nh):
        hx_, hy_ = cx - 0.9 * R + (i % side) * step, cy - 0.9 * R + (i // side) * step
        w = step * (0.9 if i % 7 == 3 else 0.5)
        h = [(hx_, hy_), (hx_ + w, hy_), (hx_ + w, hy_ + w), (hx_, hy_ + w)]
        holes.append(h[::-1] if i % 5 == 1 else h)
    return holes[:3] + [sq] + holes[3:]


def test_two_hundred_holes(ctx):
    """A polygon of 201 rings (4 mask chunks) and one of 130 with a long shell, through range,
    join and kNN (k = 1, 100, 256) against the oracle, with points on hole edges and vertices."""
    rng = np.random.default_rng(21)
    p1 = _lattice_polygon(116.4, 40.3, 0.05, 200, rng)
    big = synth._star(rng, 116.8, 40.6, 0.04, 700)
    p2 = [big] + [synth._star(rng, 116.8 + 0.025 * math.cos(a), 40.6 + 0.025 * math.sin(a), 0.0015, 8)
                  for a in np.linspace(0, 2 * math.pi, 129, endpoint=False)]
    polys = [p1, p2]
    pr = np.array([0, len(p1), len(p1) + len(p2)], np.uint32)
    off, vx, vy = _flat([ring for rings in polys for ring in rings])
    x, y = holed_window(rng, 150000, polys, 0.002)
    # points exactly on hole vertices and edge midpoints of the 200-hole polygon
    hv = np.array([c for ring in p1 for c in ring])
    mid = (hv[:-1] + hv[1:]) / 2
    x = np.concatenate([x, hv[:, 0], mid[:, 0]])
    y = np.concatenate([y, hv[:, 1], mid[:, 1]])
    ag, cg = agrid(500)
    for r in (0.0004, 0.002):
        got = ctx.range_ppoly(ag, x, y, off, vx, vy, r, poly_rings=pr)
        want = cref.range_ppoly(cg, x, y, off, vx, vy, r, poly_rings=pr)
        assert len(want) > 1000
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
        got = ctx.join_ppoly(ag, ag, x, y, off, vx, vy, r, poly_rings=pr)
        want = cref.join_ppoly(cg, cg, x, y, off, vx, vy, r, poly_rings=pr)
        assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
    for p in range(2):
        a, b = pr[p], pr[p + 1]
        ro = off[a:b + 1] - off[a]
        px, py = vx[off[a]:off[b]], vy[off[a]:off[b]]
        for k in (1, 100, 256):
            gi, gd = ctx.knn_ppoly(ag, x, y, px, py, 0.002, k, ring_off=ro)
            wi, wd = cref.knn_ppoly(cg, x, y, px, py, 0.002, k, ring_off=ro)
            assert gi.tolist() == wi.tolist() and np.array_equal(gd.view(np.uint64), wd.view(np.uint64))


def test_holes_device_window_and_repeat(ctx):
    """Device-resident points; the cached plan is reused on a repeat call and replaced when
    only the ring grouping changes (same vertices, other poly_rings)."""
    import torch
    rng = np.random.default_rng(11)
    pr, off, vx, vy, polys = synth.holed_polygons(30, 12)
    x, y = holed_window(rng, 200000, polys, 0.003)
    ag, cg = agrid(500)
    tx, ty = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    want = pairs_sorted(cref.range_ppoly(cg, x, y, off, vx, vy, 0.003, poly_rings=pr)).tolist()
    for _ in range(2):
        got = ctx.range_ppoly(ag, tx, ty, off, vx, vy, 0.003, poly_rings=pr)
        assert pairs_sorted(got.cpu().numpy()).tolist() == want
    # polygons merged pairwise: the second one's rings become holes (or the shell) of the first
    pr2 = np.append(pr[::2], pr[-1]) if len(pr) % 2 == 0 else pr[::2]
    got = ctx.range_ppoly(ag, tx, ty, off, vx, vy, 0.003, poly_rings=pr2)
    want1 = cref.range_ppoly(cg, x, y, off, vx, vy, 0.003, poly_rings=pr2)
    assert pairs_sorted(got.cpu().numpy()).tolist() == pairs_sorted(want1).tolist()
    assert pairs_sorted(want1).tolist() != want
    got = ctx.range_ppoly(ag, tx, ty, off, vx, vy, 0.003, poly_rings=pr)
    assert pairs_sorted(got.cpu().numpy()).tolist() == want


def test_holes_errors_and_empty(ctx):
    ag, cg = agrid(100)
    x, y = synth.uniform(1000, 3)
    shell = [(116.0, 40.0), (116.1, 40.0), (116.1, 40.1), (116.0, 40.1)]
    hole = [(116.04, 40.04), (116.06, 40.04), (116.05, 40.06)]
    # a hole whose first coordinate is NaN: LinearRing not closed (JTS throws)
    off, vx, vy = _flat([shell, [(math.nan, 40.05)] + hole])
    pr = np.array([0, 2], np.uint32)
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.range_ppoly(ag, x, y, off, vx, vy, 0.01, poly_rings=pr)
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.knn_ppoly(ag, x, y, vx, vy, 0.01, 5, ring_off=off)
    with pytest.raises(cref.OracleError):
        cref.range_ppoly(cg, x, y, off, vx, vy, 0.01, poly_rings=pr)
    # an empty ring (IndexOutOfBoundsException)
    off2 = np.array([0, 4, 4], np.uint32)
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.range_ppoly(ag, x, y, off2, vx, vy, 0.01, poly_rings=pr)
    # first ring with <= 3 coordinates: the reference leaves the polygon null
    off3, vx3, vy3 = _flat([hole, shell])
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.range_ppoly(ag, x, y, off3, vx3, vy3, 0.01, poly_rings=pr)
    # a polygon without rings
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.range_ppoly(ag, x, y, off, vx, vy, 0.01, poly_rings=np.array([0, 0, 2], np.uint32))
    # 65 rings (one past a mask chunk): accepted like any ring count (Polygon.java:115-165)
    rings = [shell] + [hole] * 64
    off4, vx4, vy4 = _flat(rings)
    got = ctx.range_ppoly(ag, x, y, off4, vx4, vy4, 0.01, poly_rings=np.array([0, 65], np.uint32))
    want = cref.range_ppoly(cg, x, y, off4, vx4, vy4, 0.01, poly_rings=np.array([0, 65], np.uint32))
    assert pairs_sorted(got).tolist() == pairs_sorted(want).tolist()
    gi, gd = ctx.knn_ppoly(ag, x, y, vx4, vy4, 0.01, 5, ring_off=off4)
    wi, wd = cref.knn_ppoly(cg, x, y, vx4, vy4, 0.01, 5, ring_off=off4)
    assert gi.tolist() == wi.tolist() and np.array_equal(gd.view(np.uint64), wd.view(np.uint64))
    # zero polygons, null arrays
    cnt = _abi.c_uint64(0)
    import ctypes
    rc = _abi.lib.geohip_range_ppoly(ctx.h, ctypes.byref(ag), _abi._ptr(x), _abi._ptr(y), len(x), None, None, None,
                                     None, 0, 0, 0.01, 0, None, 0, ctypes.byref(cnt))
    assert rc == _abi.OK and cnt.value == 0
    rc = _abi.lib.geohip_join_ppoly(ctx.h, ctypes.byref(ag), ctypes.byref(ag), _abi._ptr(x), _abi._ptr(y), len(x),
                                    None, None, None, None, 0, 0, 0.01, 0, None, 0, ctypes.byref(cnt))
    assert rc == _abi.OK and cnt.value == 0
    # ring offsets past the vertex count nv: GEOHIP_ERR_ARG from the C side itself (no host read
    # past the caller's arrays), for every polygon entry point
    off = np.ascontiguousarray(off4, np.uint32)
    vxc, vyc = np.ascontiguousarray(vx4, np.float64), np.ascontiguousarray(vy4, np.float64)
    short = len(vxc) - 1
    rc = _abi.lib.geohip_range_ppoly(ctx.h, ctypes.byref(ag), _abi._ptr(x), _abi._ptr(y), len(x), None, _abi._ptr(off),
                                     _abi._ptr(vxc), _abi._ptr(vyc), short, len(off) - 1, 0.01, 0, None, 0,
                                     ctypes.byref(cnt))
    assert rc == _abi.ERR_ARG and b"past" in _abi.lib.geohip_last_error(ctx.h)
    rc = _abi.lib.geohip_join_ppoly(ctx.h, ctypes.byref(ag), ctypes.byref(ag), _abi._ptr(x), _abi._ptr(y), len(x), None,
                                    _abi._ptr(off), _abi._ptr(vxc), _abi._ptr(vyc), short, len(off) - 1, 0.01, 0, None, 0,
                                    ctypes.byref(cnt))
    assert rc == _abi.ERR_ARG
    k_i = np.zeros(5, np.uint32)
    k_d = np.zeros(5, np.float64)
    kc = _abi.c_uint32(0)
    rc = _abi.lib.geohip_knn_ppoly(ctx.h, ctypes.byref(ag), _abi._ptr(x), _abi._ptr(y), len(x), _abi._ptr(off),
                                   len(off) - 1, _abi._ptr(vxc), _abi._ptr(vyc), short, 0.01, 5, 0, _abi._ptr(k_i),
                                   _abi._ptr(k_d), ctypes.byref(kc))
    assert rc == _abi.ERR_ARG


def test_holes_golden(ctx, golden):
    """The device path against the restatement's holed-polygon vectors (tests/golden)."""
    for c in golden["ppoly_holes"]:
        mx, my, l, n = grid_vals(c["grid"])
        g = _abi.make_grid(mx, my, l, n)
        x, y = arr(c["x"]), arr(c["y"])
        pr, off, vx, vy = golden_polygons(c["polygons"])
        r, approx = fx(c["r"]), c["approximate"]
        assert pairs_sorted(ctx.range_ppoly(g, x, y, off, vx, vy, r, approx, poly_rings=pr)).tolist() == \
            c["expect_range"]
        assert pairs_sorted(ctx.join_ppoly(g, g, x, y, off, vx, vy, r, approx, poly_rings=pr)).tolist() == \
            c["expect_join"]
        a, b = pr[0], pr[1]
        oi, od = ctx.knn_ppoly(g, x, y, vx[off[a]:off[b]], vy[off[a]:off[b]], r, c["k"], approx,
                               ring_off=off[a:b + 1] - off[a])
        assert oi.tolist() == c["expect_knn_idx"]
        assert [v.hex() for v in od.tolist()] == c["expect_knn_dist"]
