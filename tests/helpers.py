"""Shared helpers for the parity tests."""
import math

import numpy as np


def fx(s):
    return float.fromhex(s)


def arr(lst):
    return np.array([float.fromhex(v) for v in lst], dtype=np.float64)


def grid_vals(gd):
    return fx(gd["min_x"]), fx(gd["min_y"]), fx(gd["cell_len"]), gd["n"]


def pairs_sorted(p):
    p = np.asarray(p, dtype=np.int64).reshape(-1, 2)
    if len(p) == 0:
        return p
    o = np.lexsort((p[:, 1], p[:, 0]))
    return p[o]


def holed_window(rng, n, polys, r):
    """Uniform points plus points around each polygon: its vertices, edge midpoints, hole
    centres, points just inside / outside each hole ring and within r of it."""
    from spatialflink_amd import synth
    x, y = synth.uniform(n, int(rng.integers(1 << 30)))
    xs, ys = [x], [y]
    for rings in polys:
        allv = np.array([c for ring in rings for c in ring])
        lo, hi = allv.min(0), allv.max(0)
        xs.append(rng.uniform(lo[0] - 2 * r, hi[0] + 2 * r, 400))
        ys.append(rng.uniform(lo[1] - 2 * r, hi[1] + 2 * r, 400))
        for ring in rings:
            a = np.array(ring)
            xs += [a[:, 0], (a[:-1, 0] + a[1:, 0]) / 2]
            ys += [a[:, 1], (a[:-1, 1] + a[1:, 1]) / 2]
            c = a.mean(0)
            for f in (0.0, 0.5, 0.97, 1.03, 1.3):
                xs.append(c[0] + f * (a[:, 0] - c[0]))
                ys.append(c[1] + f * (a[:, 1] - c[1]))
    xs.append(np.array([math.nan, 116.0]))
    ys.append(np.array([40.0, math.nan]))
    return np.concatenate(xs), np.concatenate(ys)


def golden_polygons(polys_hex):
    """(poly_rings, ring_off, vx, vy) of a fixture's polygons (rings of [x, y] hex pairs)."""
    pr, off, vx, vy = [0], [0], [], []
    for rings in polys_hex:
        for ring in rings:
            vx += [fx(a) for a, _ in ring]
            vy += [fx(b) for _, b in ring]
            off.append(len(vx))
        pr.append(len(off) - 1)
    return (np.array(pr, np.uint32), np.array(off, np.uint32), np.array(vx, np.float64),
            np.array(vy, np.float64))
