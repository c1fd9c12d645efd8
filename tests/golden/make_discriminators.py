"""Generate tests/golden/jts_discriminators.json: the parity-pinning kit for SURVEY.md 8(c)'s open
questions about the third-party arithmetic (jts-core 1.16.1, pom.xml:60-64, not vendored).

Every case holds inputs on which the candidate readings of JTS disagree, with the expected answer
under each reading; libgeohip implements reading "A" (oracle/restate.py), and
tests/test_gpu_discriminators.py asserts it does.  jvm/ParityHarness.java reruns the same cases
through the reference's own DistanceFunctions (DistanceFunctions.java:15-36) on a JVM with the
reference's jars and prints which reading each question's cases follow -- one run decides Q1-Q3.

  Q1  Coordinate.distance (DistanceFunctions.java:17 -> Point.distance -> DistanceOp):
        A: Math.hypot(dx, dy) (JDK 8 StrictMath.hypot = fdlibm e_hypot.c)
        B: Math.sqrt(dx * dx + dy * dy)
      cases: point pairs whose distance bits differ, and a kNN window (PointPointKNNQuery,
      k = 16) whose top-k order differs between A and B.
  Q2  RayCrossingCounter.countSegment orientation (PointLocator inside DistanceOp):
        A: RobustDeterminant.signOfDet2x2 of the ROUNDED differences (p1 - p), (p2 - p)
        B: the exact orientation of the original coordinates (Orientation.index, DD)
      cases: points next to a polygon edge (coordinates of mixed magnitude, so the differences
      round) whose containment differs -> point-polygon distance 0 under one reading, > 0 under
      the other.
  Q3  Distance.pointToSegment op order:
        A: |((Ay-py)(Bx-Ax) - (Ax-px)(By-Ay)) / len2| * sqrt(len2)   (the 1.16.1 text recalled)
        B: hypot of p minus the projection A + r (B - A)
      cases: exterior points near star-polygon edges whose point-polygon distance bits differ.

Floats are float.hex strings.  Deterministic (seeded).

    python tests/golden/make_discriminators.py
"""
from __future__ import annotations

import json
import math
import random
import sys
from fractions import Fraction
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import restate as R  # noqa: E402

BJ = (115.5, 117.6, 39.6, 41.1)
Q = (116.414899, 39.920374)


def hx(v: float) -> str:
    return float(v).hex()


def bits(v: float) -> int:
    return R._bits(v)


def naive_dist(ax, ay, bx, by):
    dx, dy = ax - bx, ay - by
    return math.sqrt(dx * dx + dy * dy)


# ------------------------------------------------------------------------------- Q1 --------
def q1(rng):
    pairs = []
    while len(pairs) < 200:
        a = rng.uniform(0, 2 * math.pi)
        rad = rng.uniform(0.001, 0.5)
        px, py = Q[0] + rad * math.cos(a), Q[1] + rad * math.sin(a)
        A = R.jts_point_point_distance(Q[0], Q[1], px, py)
        B = naive_dist(Q[0], Q[1], px, py)
        if bits(A) != bits(B):
            pairs.append({"p": [hx(px), hx(py)], "A": hx(A), "B": hx(B)})
    # a kNN window where the k smallest (dist, idx) differ between the readings: points on a
    # thin annulus around q (radius 0.2, inside the README query's G u C at n = 100, r = 0.5)
    k = 16
    for attempt in range(1000):
        pts = []
        for _ in range(4000):
            a = rng.uniform(0, 2 * math.pi)
            rad = 0.2 + rng.uniform(-1e-15, 1e-15)
            pts.append((Q[0] + rad * math.cos(a), Q[1] + rad * math.sin(a)))
        dA = [R.jts_point_point_distance(Q[0], Q[1], x, y) for x, y in pts]
        dB = [naive_dist(Q[0], Q[1], x, y) for x, y in pts]
        # the 48 nearest by A, then check that the top-k of A and of B differ on that window
        order = sorted(range(len(pts)), key=lambda i: (dA[i], i))[:48]
        win = [pts[i] for i in order]
        wA = [dA[i] for i in order]
        wB = [dB[i] for i in order]
        sa = sorted(range(len(win)), key=lambda i: (bits(wA[i]), i))
        sb = sorted(range(len(win)), key=lambda i: (bits(wB[i]), i))
        # no exact tie at rank k under either reading (the reference's tie order is arrival-order)
        if wA[sa[k - 1]] == wA[sa[k]] or wB[sb[k - 1]] == wB[sb[k]]:
            continue
        if sa[:k] != sb[:k]:
            return pairs, {
                "query": [hx(Q[0]), hx(Q[1])], "r": hx(0.5), "k": k,
                "grid": {"n": 100, "min_x": hx(BJ[0]), "max_x": hx(BJ[1]), "min_y": hx(BJ[2]), "max_y": hx(BJ[3])},
                "x": [hx(p[0]) for p in win], "y": [hx(p[1]) for p in win],
                "A": {"idx": sa[:k], "dist": [hx(wA[i]) for i in sa[:k]]},
                "B": {"idx": sb[:k], "dist": [hx(wB[i]) for i in sb[:k]]},
            }
    raise RuntimeError("no discriminating kNN window found")


# ------------------------------------------------------------------------------- Q2 --------
def orient_exact(p1, p2, p):
    """Sign of the orientation of (p1, p2, p) in exact arithmetic on the original doubles."""
    x1, y1 = Fraction(p1[0]) - Fraction(p[0]), Fraction(p1[1]) - Fraction(p[1])
    x2, y2 = Fraction(p2[0]) - Fraction(p[0]), Fraction(p2[1]) - Fraction(p[1])
    d = x1 * y2 - y1 * x2
    return (d > 0) - (d < 0)


def locate_B(px, py, ring):
    """RayCrossingCounter with the exact orientation of the original coordinates (reading B)."""
    crossings = 0
    for i in range(1, len(ring)):
        p1x, p1y = ring[i]
        p2x, p2y = ring[i - 1]
        if p1x < px and p2x < px:
            continue
        if px == p2x and py == p2y:
            return R.BOUNDARY
        if p1y == py and p2y == py:
            if min(p1x, p2x) <= px <= max(p1x, p2x):
                return R.BOUNDARY
            continue
        if (p1y > py and p2y <= py) or (p2y > py and p1y <= py):
            s = orient_exact((p1x, p1y), (p2x, p2y), (px, py))
            if s == 0:
                return R.BOUNDARY
            if p2y - py < p1y - py:
                s = -s
            if s > 0:
                crossings += 1
    return R.INTERIOR if crossings % 2 == 1 else R.EXTERIOR


def q2(rng):
    # a triangle whose long edge passes 1e-3 from the origin: points near that edge have small
    # coordinates, the vertices large ones, so p1 - p rounds
    ring = [(-6.0, -4.500000000000123), (6.0, 4.5000000000003), (-5.0, 5.25), (-6.0, -4.500000000000123)]
    a, b = ring[0], ring[1]
    cases = []
    seen = set()
    for trial in range(400000):
        t = 0.5 + rng.uniform(-2e-3, 2e-3)
        px = a[0] + t * (b[0] - a[0])
        py = a[1] + t * (b[1] - a[1])
        k = rng.randrange(-40, 41)
        py = py + k * 2.0 ** -60 if rng.random() < 0.5 else py
        px = px + rng.randrange(-40, 41) * 2.0 ** -60
        if (px, py) in seen:
            continue
        seen.add((px, py))
        # the point-polygon distance is 0 when the point is located inside / on the ring, or when
        # its segment distance rounds to 0: compare the distances, not just the locations
        da = R.jts_point_polygon_distance(px, py, ring)
        db = 0.0 if locate_B(px, py, ring) != R.EXTERIOR else min(
            R.point_to_segment(px, py, *ring[i], *ring[i + 1]) for i in range(len(ring) - 1))
        inside_a, inside_b = da == 0.0, db == 0.0
        if inside_a != inside_b:
            cases.append({"p": [hx(px), hx(py)], "A_inside": inside_a, "B_inside": inside_b,
                          "A_dist": hx(da), "B_dist": hx(db)})
            if len(cases) >= 40:
                break
    if len(cases) < 8:
        raise RuntimeError(f"only {len(cases)} Q2 discriminators found")
    return {"ring": [[hx(x), hx(y)] for x, y in ring], "r": hx(1e-300),
            "grid": {"n": 64, "min_x": hx(-8.0), "max_x": hx(8.0), "min_y": hx(-8.0), "max_y": hx(8.0)},
            "cases": cases}


# ------------------------------------------------------------------------------- Q3 --------
def seg_B(px, py, ax, ay, bx, by):
    if ax == bx and ay == by:
        return R.coord_distance(px, py, ax, ay)
    len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay)
    r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2
    if r <= 0.0:
        return R.coord_distance(px, py, ax, ay)
    if r >= 1.0:
        return R.coord_distance(px, py, bx, by)
    cx, cy = ax + r * (bx - ax), ay + r * (by - ay)
    return R.coord_distance(px, py, cx, cy)


def poly_dist_B(px, py, ring):
    if R._ring_location(px, py, ring) != R.EXTERIOR:
        return 0.0
    md = R.DBL_MAX
    for i in range(len(ring) - 1):
        d = seg_B(px, py, ring[i][0], ring[i][1], ring[i + 1][0], ring[i + 1][1])
        if d < md:
            md = d
    return md


def q3(rng):
    c = (116.40, 39.95)
    ring = []
    for j in range(50):
        a = 2 * math.pi * j / 50
        rad = 0.01 * (1 + 0.3 * rng.random())
        ring.append((c[0] + rad * math.cos(a), c[1] + rad * math.sin(a)))
    ring.append(ring[0])
    cases = []
    while len(cases) < 48:
        j = rng.randrange(50)
        (ax, ay), (bx, by) = ring[j], ring[j + 1]
        t = rng.uniform(0.05, 0.95)
        mx, my = ax + t * (bx - ax), ay + t * (by - ay)
        nx, ny = by - ay, -(bx - ax)  # outward-ish normal (counter-clockwise ring)
        s = rng.uniform(1e-4, 2e-3) / math.hypot(nx, ny)
        px, py = mx + s * nx, my + s * ny
        if R._ring_location(px, py, ring) != R.EXTERIOR:
            continue
        A = R.jts_point_polygon_distance(px, py, ring)
        B = poly_dist_B(px, py, ring)
        if bits(A) != bits(B):
            cases.append({"p": [hx(px), hx(py)], "A": hx(A), "B": hx(B)})
    return {"ring": [[hx(x), hx(y)] for x, y in ring], "r": hx(0.005),
            "grid": {"n": 500, "min_x": hx(BJ[0]), "max_x": hx(BJ[1]), "min_y": hx(BJ[2]), "max_y": hx(BJ[3])},
            "cases": cases}


def main():
    rng = random.Random(20261017)
    pairs, knn = q1(rng)
    out = {
        "generator": "tests/golden/make_discriminators.py (oracle/restate.py readings A; alternatives B restated here)",
        "reference": "DistanceFunctions.java:15-36 -> jts-core 1.16.1 (pom.xml:60-64); SURVEY.md 8(c) Q1-Q3",
        "Q1": {"question": "Coordinate.distance: A = Math.hypot (fdlibm), B = Math.sqrt(dx*dx + dy*dy)",
               "pairs_from_query": {"query": [hx(Q[0]), hx(Q[1])], "cases": pairs}, "knn": knn},
        "Q2": {"question": "RayCrossingCounter orientation: A = exact sign of the rounded differences, "
                           "B = exact orientation of the original coordinates", **q2(rng)},
        "Q3": {"question": "Distance.pointToSegment: A = |cross / len2| * sqrt(len2), B = hypot(p - projection)",
               **q3(rng)},
    }
    (HERE / "jts_discriminators.json").write_text(json.dumps(out, indent=1) + "\n")
    print("Q1 pairs", len(pairs), "knn window", len(knn["x"]), "| Q2 cases", len(out["Q2"]["cases"]),
          "| Q3 cases", len(out["Q3"]["cases"]))


if __name__ == "__main__":
    main()
