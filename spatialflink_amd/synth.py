"""Synthetic window generators: counter-based, so any shard can
regenerate any slice.  ``uniform`` is bit-identical to ``geohip_synth_uniform_async``."""
from __future__ import annotations

import numpy as np

BEIJING = (115.5, 117.6, 39.6, 41.1)  # conf/geoflink-conf.yml:20 gridBBox (minX, maxX, minY, maxY)
README_QUERY = (116.414899, 39.920374)  # README.md:100

_M1 = np.uint64(0x9E3779B97F4A7C15)
_M2 = np.uint64(0xBF58476D1CE4E5B9)
_M3 = np.uint64(0x94D049BB133111EB)
_SEEDMUL = np.uint64(0x632BE59BD9B4E019)


def splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + _M1
        z = (z ^ (z >> np.uint64(30))) * _M2
        z = (z ^ (z >> np.uint64(27))) * _M3
        return z ^ (z >> np.uint64(31))


def unit_uniform(seed: int, k: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        h = splitmix64(np.uint64(seed) * _SEEDMUL + k.astype(np.uint64))
    return (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def uniform(n: int, seed: int, bbox=BEIJING, base: int = 0):
    min_x, max_x, min_y, max_y = bbox
    g = np.arange(base, base + n, dtype=np.uint64)
    ux = unit_uniform(seed, np.uint64(2) * g)
    uy = unit_uniform(seed, np.uint64(2) * g + np.uint64(1))
    return min_x + ux * (max_x - min_x), min_y + uy * (max_y - min_y)


def gaussian_clusters(n: int, seed: int, centres_seed: int = 1000, n_centres: int = 32, sigma: float = 0.1,
                      bbox=BEIJING):
    """32 isotropic Gaussian clusters with centres shared across streams (centres_seed),
    rejection-sampled into the bbox."""
    min_x, max_x, min_y, max_y = bbox
    cr = np.random.default_rng(centres_seed)
    cx = cr.uniform(min_x, max_x, n_centres)
    cy = cr.uniform(min_y, max_y, n_centres)
    rng = np.random.default_rng(seed)
    xs = np.empty(n)
    ys = np.empty(n)
    filled = 0
    while filled < n:
        m = int((n - filled) * 1.3) + 16
        c = rng.integers(0, n_centres, m)
        x = cx[c] + rng.normal(0.0, sigma, m)
        y = cy[c] + rng.normal(0.0, sigma, m)
        ok = (x >= min_x) & (x < max_x) & (y >= min_y) & (y < max_y)
        x, y = x[ok], y[ok]
        t = min(len(x), n - filled)
        xs[filled:filled + t] = x[:t]
        ys[filled:filled + t] = y[:t]
        filled += t
    return xs, ys


def star_polygons(n_poly: int, seed: int, n_vert: int = 50, bbox=BEIJING, r_min=0.005, r_max=0.02):
    """n_poly star-shaped rings: centre uniform, n_vert vertices at equal angles with radius
    R*(1 + 0.3u), R ~ U[r_min, r_max]; ring closed (n_vert + 1 coords).  Returns
    (ring_off, vx, vy)."""
    min_x, max_x, min_y, max_y = bbox
    rng = np.random.default_rng(seed)
    off = [0]
    vx, vy = [], []
    for _ in range(n_poly):
        cx = rng.uniform(min_x, max_x)
        cy = rng.uniform(min_y, max_y)
        R = rng.uniform(r_min, r_max)
        ang = np.arange(n_vert) * (2 * np.pi / n_vert)
        rad = R * (1 + 0.3 * rng.uniform(0, 1, n_vert))
        x = cx + rad * np.cos(ang)
        y = cy + rad * np.sin(ang)
        vx.extend(x.tolist() + [x[0]])
        vy.extend(y.tolist() + [y[0]])
        off.append(len(vx))
    return np.array(off, np.uint32), np.array(vx), np.array(vy)


def _star(rng, cx, cy, R, nv, closed=True, clockwise=False):
    ang = np.arange(nv) * (2 * np.pi / nv)
    if clockwise:
        ang = -ang
    rad = R * (1 + 0.3 * rng.uniform(0, 1, nv))
    x = (cx + rad * np.cos(ang)).tolist()
    y = (cy + rad * np.sin(ang)).tolist()
    if closed:
        x.append(x[0])
        y.append(y[0])
    return list(zip(x, y))


def holed_polygons(n_poly: int, seed: int, n_vert: int = 40, bbox=BEIJING, r_min=0.005, r_max=0.02):
    """n_poly polygons with holes (Polygon(List<List<Coordinate>>) input: rings in the caller's
    order, the largest area becomes the shell).  Star shell of radius R plus 1-3 star holes of
    radius 0.12-0.25 R inside it; by p % 6 the variant: 0 plain, 1 holes listed before the
    shell, 2 an extra degenerate 2-coordinate hole (padded by createPolygonArray), 3 a hole
    crossing the shell's boundary, 4 a "hole" outside the shell (JTS does not validate), 5
    clockwise holes and an open shell.  Returns (poly_rings, ring_off, vx, vy, rings) with
    rings[p] = the list of rings of polygon p."""
    min_x, max_x, min_y, max_y = bbox
    rng = np.random.default_rng(seed)
    polys = []
    for p in range(n_poly):
        v = p % 6
        cx = rng.uniform(min_x + 0.05, max_x - 0.05)
        cy = rng.uniform(min_y + 0.05, max_y - 0.05)
        R = rng.uniform(r_min, r_max)
        shell = _star(rng, cx, cy, R, n_vert, closed=(v != 5))
        holes = []
        for _ in range(int(rng.integers(1, 4))):
            a = rng.uniform(0, 2 * np.pi)
            d = R * rng.uniform(0.0, 0.45)
            holes.append(_star(rng, cx + d * np.cos(a), cy + d * np.sin(a), R * rng.uniform(0.12, 0.25),
                               int(rng.integers(6, 16)), closed=bool(rng.integers(0, 2)), clockwise=(v == 5)))
        if v == 2:
            holes.append([(cx + 0.5 * R, cy), (cx + 0.55 * R, cy + 0.05 * R)])
        if v == 3:
            holes.append(_star(rng, cx + 0.95 * R, cy, 0.2 * R, 10))
        if v == 4:
            holes.append(_star(rng, cx + 1.6 * R, cy + 0.3 * R, 0.2 * R, 10))
        polys.append(holes + [shell] if v == 1 else [shell] + holes)
    pr, off, vx, vy = [0], [0], [], []
    for rings in polys:
        for ring in rings:
            vx.extend(c[0] for c in ring)
            vy.extend(c[1] for c in ring)
            off.append(len(vx))
        pr.append(len(off) - 1)
    return np.array(pr, np.uint32), np.array(off, np.uint32), np.array(vx), np.array(vy), polys


def _digits(v: np.ndarray, width: int) -> np.ndarray:
    """ASCII digits of non-negative int64 v, zero-padded to width: uint8 [len(v), width]."""
    p = np.int64(10) ** np.arange(width - 1, -1, -1, dtype=np.int64)
    return ((v[:, None] // p[None, :]) % 10 + 48).astype(np.uint8)


def csv_text(n: int, seed: int, bbox=BEIJING, frac_digits: int = 13, ts0: int = 1611022449423,
             chunk: int = 1 << 20):
    """CSVTSVToTSpatial records "oid,ts,x,y\\n" (csvTsvSchemaAttr [0, 1, 2, 3]) for the uniform
    window ``uniform(n, seed)`` rounded to frac_digits decimals: oid = record index (no leading
    zeros, so records are ragged), ts = ts0 + index, x/y fixed-point with frac_digits fraction digits.

    Returns (text bytes as a uint8 array, X, Y) where X / 10**frac_digits (an exact int64 over an
    exact power of ten, so one correctly rounded fp64 division) is bit-for-bit the double
    Double.parseDouble returns for the x text; likewise Y."""
    x, y = uniform(n, seed, bbox)
    scale = 10.0 ** frac_digits
    X = np.rint(x * scale).astype(np.int64)
    Y = np.rint(y * scale).astype(np.int64)
    if max(abs(bbox[0]), abs(bbox[1]), abs(bbox[2]), abs(bbox[3])) * scale >= 2.0 ** 53 or min(bbox) < 0:
        raise ValueError("fixed-point synth text needs non-negative coordinates below 2^53 / 10^frac_digits")
    xi_w = len(str(int(bbox[1])))
    yi_w = len(str(int(bbox[3])))
    parts = []
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        idx = np.arange(s, e, dtype=np.int64)
        oid = _digits(idx, 10)
        keep_oid = np.cumsum(oid != 48, axis=1) > 0
        keep_oid[:, -1] = True
        m = e - s
        comma = np.full((m, 1), ord(","), np.uint8)
        dot = np.full((m, 1), ord("."), np.uint8)
        nl = np.full((m, 1), ord("\n"), np.uint8)
        ip = np.int64(10) ** frac_digits
        mat = np.hstack([oid, comma, _digits(ts0 + idx, 13), comma,
                         _digits(X[s:e] // ip, xi_w), dot, _digits(X[s:e] % ip, frac_digits), comma,
                         _digits(Y[s:e] // ip, yi_w), dot, _digits(Y[s:e] % ip, frac_digits), nl])
        keep = np.ones(mat.shape, bool)
        keep[:, :10] = keep_oid
        parts.append(mat[keep])
    return np.concatenate(parts) if parts else np.zeros(0, np.uint8), X, Y
