"""CPU: libgeohip's host planner (the product's plan.cpp, called through the C ABI) against
the literal restatement.

The planner turns the reference's guaranteed / candidate cell sets into rectangles and then
into exact coordinate boxes; the kernels classify points with those boxes only.  These
tests check (1) the rectangles expand to exactly the restatement's string-key sets and
(2) box classification equals cell-set membership for random, boundary-adjacent, NaN, inf
and far-out-of-grid points (geohip_debug_classify evaluates the boxes on the host with the
same predicate as the device).
"""
import math

import numpy as np
import pytest

import restate as R
from spatialflink_amd import _abi

BJ = (115.5, 117.6, 39.6, 41.1)
Q = (116.414899, 39.920374)


def expand(rects):
    s = set()
    for x0, x1, y0, y1 in rects:
        for i in range(x0, x1 + 1):
            for j in range(y0, y1 + 1):
                s.add(R.fmt05(i) + R.fmt05(j))
    return s


QUERIES = [Q, (116.0, 40.5), (115.45, 39.55), (117.7, 41.3), (100.0, 39.0), (116.0, math.nan), (math.nan, math.nan),
           (-1e6, 40.0), (115.5, 39.6), (117.6, 41.1)]
RADII = [0.5, 0.05, 0.005, 0.0, -0.1, math.nan, 0.021 * math.sqrt(2) * 1.0000001, 0.03, 3.0, math.inf]


@pytest.mark.parametrize("n", [1, 7, 100, 500])
def test_rect_sets_equal_restatement(n):
    rg = R.UniformGrid(n, *BJ)
    g = _abi.make_grid(rg.min_x, rg.min_y, rg.cell_len, rg.n)
    for q in QUERIES:
        for r in RADII:
            qkey = rg.key(*q)
            try:
                G = rg.guaranteed_cells(r, qkey)
                C = rg.candidate_cells(r, qkey, G)
                ref_err = None
            except (R.NumberFormatException, RuntimeError) as e:
                ref_err = e
            if ref_err is not None:
                with pytest.raises(_abi.GeohipArgumentError):
                    _abi.plan_point(g, q[0], q[1], r)
                continue
            gr, cr, lg, lc = _abi.plan_point(g, q[0], q[1], r)
            assert (lg, lc) == (rg.guaranteed_layers(r), rg.candidate_layers(r))
            assert expand(gr) == G, (n, q, r)
            assert expand(cr) - G == C, (n, q, r)


def _boundary_points(rg, rng, m=400):
    xs, ys = [], []
    for _ in range(m):
        i = int(rng.integers(-2, rg.n + 3))
        j = int(rng.integers(-2, rg.n + 3))
        bx = rg.min_x + i * rg.cell_len
        by = rg.min_y + j * rg.cell_len
        for dx in (-2, -1, 0, 1, 2):
            x = bx
            for _ in range(abs(dx)):
                x = math.nextafter(x, math.copysign(math.inf, dx))
            xs.append(x)
            ys.append(by if dx % 2 else math.nextafter(by, -math.inf))
    return xs, ys


@pytest.mark.parametrize("n", [7, 100, 500])
def test_box_classification_equals_cell_sets(n):
    rng = np.random.default_rng(n)
    rg = R.UniformGrid(n, *BJ)
    g = _abi.make_grid(rg.min_x, rg.min_y, rg.cell_len, rg.n)
    xs = rng.uniform(115.0, 118.0, 3000).tolist()
    ys = rng.uniform(39.0, 41.7, 3000).tolist()
    bx, by = _boundary_points(rg, rng)
    xs += bx + [math.nan, 116.0, math.nan, math.inf, -math.inf, 1e300, -1e300, rg.min_x, 116.0]
    ys += by + [40.0, math.nan, math.nan, 40.0, 40.0, 40.0, 40.0, rg.min_y, -math.inf]
    x = np.array(xs)
    y = np.array(ys)
    for q in QUERIES[:6]:
        for r in [0.5, 0.05, 0.005, math.nan, 0.021 * math.sqrt(2) * 1.0000001, 0.2]:
            qkey = rg.key(*q)
            try:
                G = rg.guaranteed_cells(r, qkey)
                C = rg.candidate_cells(r, qkey, G)
            except (R.NumberFormatException, RuntimeError):
                continue
            bits = _abi.debug_classify(g, q[0], q[1], r, x, y)
            keys = [rg.key(a, b) for a, b in zip(xs, ys)]
            want_g = np.array([k in G for k in keys])
            want_c = np.array([(k in C) for k in keys])
            assert np.array_equal((bits & 1) == 1, want_g), (q, r)
            assert np.array_equal((bits & 2) == 2, want_c), (q, r)
            assert np.array_equal((bits & 4) == 4, want_g | want_c), (q, r)


def test_planner_cell_matches_restatement():
    rng = np.random.default_rng(11)
    for n in (1, 100, 1000):
        rg = R.UniformGrid(n, *BJ)
        g = _abi.make_grid(rg.min_x, rg.min_y, rg.cell_len, rg.n)
        pts = [(float(a), float(b)) for a, b in zip(rng.uniform(110, 120, 200), rng.uniform(35, 45, 200))]
        pts += [(math.nan, 1.0), (math.inf, -math.inf), (1e300, -1e300), (rg.min_x, rg.min_y)]
        for x, y in pts:
            assert _abi.plan_cell(g, x, y) == rg.cell_indices(x, y)


def test_grid_validation():
    with pytest.raises(_abi.GeohipArgumentError):
        _abi.plan_point(_abi.make_grid(115.5, 39.6, 0.0, 100), 116, 40, 0.1)
    with pytest.raises(_abi.GeohipArgumentError):
        _abi.plan_point(_abi.make_grid(115.5, 39.6, 0.02, 0), 116, 40, 0.1)
    with pytest.raises(_abi.GeohipUnsupportedError):
        _abi.plan_point(_abi.make_grid(115.5, 39.6, 0.02, 100000), 116, 40, 0.1)
