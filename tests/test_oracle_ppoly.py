"""CPU: the two oracles of the point-polygon join and kNN agree.

oracle/restate.py restates PointPolygonJoinQuery / PointPolygonKNNQuery literally (gridID
strings, HashSet replication, per-cell heaps); oracle/geohip_oracle.c with packed cell sets and
one global heap.  Small random windows over several grids, both grids of the join, radii with
and without guaranteed cells, approximate mode, boundary points and out-of-grid polygons.
"""
import math

import numpy as np
import pytest

import cref
import restate as R
from helpers import holed_window

BJ = (115.5, 117.6, 39.6, 41.1)


def grids(n):
    l = (BJ[1] - BJ[0]) / n
    return R.UniformGrid(n, *BJ), cref.grid(BJ[0], BJ[2], l, n)


def star(rng, cx, cy, rad, nv=12):
    a = np.arange(nv) * 2 * math.pi / nv
    rr = rad * (1 + 0.3 * rng.random(nv))
    return list(zip((cx + rr * np.cos(a)).tolist(), (cy + rr * np.sin(a)).tolist()))


def window(rng, n, rings):
    x = rng.uniform(BJ[0] - 0.05, BJ[1] + 0.05, n)
    y = rng.uniform(BJ[2] - 0.05, BJ[3] + 0.05, n)
    # points on vertices and edge midpoints (boundary: distance 0) and a NaN point
    extra = [c for ring in rings for c in ring[:3]]
    extra += [((ring[0][0] + ring[1][0]) / 2, (ring[0][1] + ring[1][1]) / 2) for ring in rings]
    x = np.concatenate([x, [e[0] for e in extra], [math.nan]])
    y = np.concatenate([y, [e[1] for e in extra], [40.0]])
    return x, y


def flat(rings):
    off, vx, vy = [0], [], []
    for ring in rings:
        vx += [c[0] for c in ring]
        vy += [c[1] for c in ring]
        off.append(len(vx))
    return np.array(off, np.uint32), np.array(vx), np.array(vy)


JOIN_CASES = [(100, 100, 0.03, False), (500, 500, 0.03, False), (500, 500, 0.03, True), (200, 500, 0.02, False),
              (500, 200, 0.05, False), (100, 100, 0.0, False), (100, 100, 0.0212 * 1.45, False)]


@pytest.mark.parametrize("case", range(len(JOIN_CASES)))
def test_join_ppoly_oracles_agree(case):
    nu, nq, r, approx = JOIN_CASES[case]
    rng = np.random.default_rng(100 + case)
    rings = [star(rng, rng.uniform(*BJ[:2]), rng.uniform(*BJ[2:]), rng.uniform(0.005, 0.03)) for _ in range(4)]
    rings.append([(115.48, 39.58), (115.56, 39.58), (115.56, 39.66), (115.48, 39.66)])  # crosses the grid corner
    x, y = window(rng, 3000, rings)
    ug, cu = grids(nu)
    qg, cq = grids(nq)
    want = sorted(R.join_ppoly(ug, qg, x.tolist(), y.tolist(), rings, r, approx))
    off, vx, vy = flat(rings)
    got = sorted(map(tuple, cref.join_ppoly(cu, cq, x, y, off, vx, vy, r, approx).tolist()))
    assert got == want


def test_join_ppoly_vs_range():
    """Join exact = range exact where G is empty (Lg < 0); with G non-empty the join checks
    the distance of G points too, so it is a subset of the range result (strict for a thin
    diagonal sliver, whose bounding-box corners lie far from the polygon)."""
    rng = np.random.default_rng(7)
    ug, cu = grids(500)
    sliver = [(116.0, 40.0), (116.3, 40.3), (116.3, 40.301), (116.0, 40.001)]
    rings = [star(rng, 116.4, 40.0, 0.02), sliver]
    x, y = window(rng, 20000, rings)
    off, vx, vy = flat(rings)
    for r, equal in ((0.004, True), (0.04, False)):
        j = {(p, q) for p, q in cref.join_ppoly(cu, cu, x, y, off, vx, vy, r).tolist()}
        rg = {(p, q) for q, p in cref.range_ppoly(cu, x, y, off, vx, vy, r).tolist()}
        assert (j == rg) if equal else (j < rg)


KNN_CASES = [(100, 0.03, 10, False), (500, 0.01, 50, False), (500, 0.01, 50, True), (200, 0.05, 1, False),
             (100, 0.0, 5, False), (500, 0.02, 256, False)]


@pytest.mark.parametrize("case", range(len(KNN_CASES)))
def test_knn_ppoly_oracles_agree(case):
    n, r, k, approx = KNN_CASES[case]
    rng = np.random.default_rng(200 + case)
    ring = star(rng, 116.4, 40.2, 0.02)
    x, y = window(rng, 4000, [ring])
    x = np.concatenate([x, rng.uniform(116.38, 116.42, 300)])  # many inside: ties at distance 0
    y = np.concatenate([y, rng.uniform(40.18, 40.22, 300)])
    g, cg = grids(n)
    want = R.knn_ppoly(g, x.tolist(), y.tolist(), ring, r, k, approx)
    vx = np.array([c[0] for c in ring])
    vy = np.array([c[1] for c in ring])
    gi, gd = cref.knn_ppoly(cg, x, y, vx, vy, r, k, approx)
    assert gi.tolist() == [i for i, _ in want]
    wd = np.array([d for _, d in want], dtype=np.float64)
    assert np.array_equal(gd.view(np.uint64), wd.view(np.uint64)) or \
        (np.isnan(gd) == np.isnan(wd)).all() and np.array_equal(gd[~np.isnan(gd)], wd[~np.isnan(wd)])


def test_knn_ppoly_errors():
    _, cg = grids(100)
    with pytest.raises(cref.OracleError):
        cref.knn_ppoly(cg, np.zeros(3), np.zeros(3), np.array([116.0, 116.1, 116.0]), np.array([40.0, 40.0, 40.1]),
                       0.01, 5)  # <= 3 coordinates: Polygon.java:53
    with pytest.raises(cref.OracleError):
        cref.knn_ppoly(cg, np.zeros(3), np.zeros(3), np.array([116.0, 116.1, 116.1, 116.0]),
                       np.array([40.0, 40.0, 40.1, 40.1]), 0.01, 0)  # k = 0


HOLE_CASES = [(500, 0.0005, False), (500, 0.003, False), (100, 0.01, False), (500, 0.003, True)]


@pytest.mark.parametrize("case", range(len(HOLE_CASES)))
def test_holed_polygons_oracles_agree(case):
    """Polygons with holes (createPolygonArray ordering, padding, hole crossing / outside the
    shell): the C oracle's range, join and kNN against the literal restatement."""
    from spatialflink_amd import synth
    n, r, approx = HOLE_CASES[case]
    rng = np.random.default_rng(300 + case)
    pr, off, vx, vy, polys = synth.holed_polygons(6, 310 + case)
    x, y = holed_window(rng, 2000, polys, r)
    g, cg = grids(n)
    want = sorted(R.range_ppoly(g, x.tolist(), y.tolist(), polys, r, approx))
    got = sorted(map(tuple, cref.range_ppoly(cg, x, y, off, vx, vy, r, approx, poly_rings=pr).tolist()))
    assert got == want
    assert len(want) > 500
    want = sorted(R.join_ppoly(g, g, x.tolist(), y.tolist(), polys, r, approx))
    got = sorted(map(tuple, cref.join_ppoly(cg, cg, x, y, off, vx, vy, r, approx, poly_rings=pr).tolist()))
    assert got == want
    for p in (0, 3, 4):
        w = R.knn_ppoly(g, x.tolist(), y.tolist(), polys[p], r, 50, approx)
        a, b = pr[p], pr[p + 1]
        ro = off[a:b + 1] - off[a]
        gi, gd = cref.knn_ppoly(cg, x, y, vx[off[a]:off[b]], vy[off[a]:off[b]], r, 50, approx, ring_off=ro)
        assert gi.tolist() == [i for i, _ in w]
        assert np.array_equal(gd.view(np.uint64), np.array([d for _, d in w]).view(np.uint64))


def test_holed_point_distance_cases():
    """JTS point.distance(polygon) with holes: inside a hole (distance to the hole ring), on a
    hole edge / vertex (0), in the shell outside the holes (0), outside the shell."""
    shell = [(0.0, 0.0), (10.0, 0.0), (10.0, 10.0), (0.0, 10.0)]
    hole = [(4.0, 4.0), (6.0, 4.0), (6.0, 6.0), (4.0, 6.0)]
    off = np.array([0, 4, 8], np.uint32)
    vx = np.array([c[0] for c in shell + hole])
    vy = np.array([c[1] for c in shell + hole])
    for (px, py), want in [((5.0, 5.0), 1.0), ((4.5, 5.0), 0.5), ((6.0, 5.0), 0.0), ((4.0, 4.0), 0.0),
                           ((2.0, 2.0), 0.0), ((12.0, 5.0), 2.0), ((5.0, 4.25), 0.25)]:
        assert cref.point_polygon(px, py, vx, vy, ring_off=off) == want
        assert R.jts_point_polygon_distance(px, py, R.make_polygon([shell, hole])) == want
    # ring order does not matter: the larger ring becomes the shell
    off2 = np.array([0, 4, 8], np.uint32)
    vx2 = np.array([c[0] for c in hole + shell])
    vy2 = np.array([c[1] for c in hole + shell])
    assert cref.point_polygon(5.0, 5.0, vx2, vy2, ring_off=off2) == 1.0
