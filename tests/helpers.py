"""Shared helpers for the parity tests."""
import math

import numpy as np

from spatialflink_amd import synth

BJ = synth.BEIJING


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


# ---- order-independent digests of device pair lists (tests/test_gpu_fullscale.py, test_gpu_join_mid.py)
MASK = (1 << 64) - 1


def _s64(c):  # an unsigned 64-bit constant as the int64 torch holds it
    return c - (1 << 64) if c >= 1 << 63 else c


def _lsr(z, s):  # logical right shift of int64 lanes
    import torch
    return torch.bitwise_and(torch.bitwise_right_shift(z, s), (1 << (64 - s)) - 1)


def mix64_torch(v):
    """splitmix64 finaliser on int64 lanes (wrapping arithmetic), = cref.mix64 bit for bit."""
    import torch
    z = v + _s64(0x9E3779B97F4A7C15)
    z = torch.bitwise_xor(z, _lsr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = torch.bitwise_xor(z, _lsr(z, 27)) * _s64(0x94D049BB133111EB)
    return torch.bitwise_xor(z, _lsr(z, 31))


def pair_digest(pairs, chunk=1 << 26):
    """(count, sum of mix64(a << 32 | b) mod 2^64) of an [m, 2] int32 device tensor of pairs."""
    import torch
    m = int(pairs.shape[0])
    h = 0
    for s in range(0, m, chunk):
        p = pairs[s:s + chunk].to(torch.int64)
        v = torch.bitwise_or(torch.bitwise_left_shift(torch.bitwise_and(p[:, 0], 0xFFFFFFFF), 32),
                             torch.bitwise_and(p[:, 1], 0xFFFFFFFF))
        # int64 sums wrap like the oracle's uint64 sum; add the halves exactly in Python
        z = mix64_torch(v)
        lo = int(torch.bitwise_and(z, 0xFFFFFFFF).sum().item())
        hi = int(_lsr(z, 32).sum().item())
        h = (h + lo + (hi << 32)) & MASK
    return m, h


# ---- point-polygon windows around the grid edge (tests/test_gpu_ppoly_tiles.py)
def edge_window(n, seed, off, vx, vy):
    """Uniform points, every vertex and edge midpoint, points around the grid's west edge (in
    and out of the grid), NaN points."""
    x, y = synth.uniform(n, seed)
    rng = np.random.default_rng(seed)
    ex = BJ[0] + rng.uniform(-0.03, 0.03, 4000)
    ey = rng.uniform(39.85, 39.95, 4000)
    mx, my = (vx[:-1] + vx[1:]) / 2, (vy[:-1] + vy[1:]) / 2
    return (np.concatenate([x, vx, mx, ex, [math.nan, 116.0]]), np.concatenate([y, vy, my, ey, [40.0, math.nan]]))


def edge_polygons(npoly, seed, r_min, r_max):
    """Star rings plus three rings across the grid's west edge (their cells leave the grid)."""
    off, vx, vy = synth.star_polygons(npoly, seed, r_min=r_min, r_max=r_max)
    rng = np.random.default_rng(seed + 1)
    xs, ys, o = [vx], [vy], list(off)
    for cy in (39.87, 39.90, 39.93):
        ang = np.arange(24) * (2 * np.pi / 24)
        rad = 0.01 * (1 + 0.3 * rng.uniform(0, 1, 24))
        px, py = BJ[0] + rad * np.cos(ang), cy + rad * np.sin(ang)
        xs.append(np.append(px, px[0]))
        ys.append(np.append(py, py[0]))
        o.append(o[-1] + 25)
    return np.array(o, np.uint32), np.concatenate(xs), np.concatenate(ys)
