"""Pure-Python, literal restatement of GeoFlink's windowed spatial query evaluation.

TEST INFRASTRUCTURE ONLY.  This module is an oracle: it may be imported by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg,
never by the product (``spatialflink_amd``), which must run on the HIP library.

It restates, line by line and with Java semantics, the reference path
(``/root/reference/src/main/java/GeoFlink``, abbreviated ``G/``):

* cell keys are real Java-style strings (``String.format("%05d")``
  concatenation, ``HelperClass.java:54-57,104-120``) parsed back exactly like
  ``HelperClass.getIntCellIndices`` (``HelperClass.java:263-276``, with the
  ``removeLeadingZeroesFromString`` regex of ``HelperClass.java:60-63``);
* guaranteed / candidate / neighbouring cell sets are Python ``set``s of those
  strings built by the same loops as ``UniformGrid.java:165-206,261-293,367-444``
  (Java ``int`` wrap-around included);
* distances follow the third-party arithmetic the reference calls
  (``DistanceFunctions.java:15-36`` -> JTS ``jts-core`` 1.16.1, pinned at
  ``pom.xml:60-64``, not vendored): ``Coordinate.distance`` = ``Math.hypot``
  = fdlibm ``e_hypot.c`` (JDK 8 ``StrictMath.hypot``), ``DistanceOp``'s
  ``minDistance`` initialised to ``Double.MAX_VALUE`` with strict ``<`` updates,
  ``Distance.pointToSegment`` and ``RayCrossingCounter`` with an exact
  determinant sign (``RobustDeterminant.signOfDet2x2``);
* kNN per-cell heaps use a literal port of ``java.util.PriorityQueue`` with
  ``Comparators.inTuplePointDistanceComparator`` (``Comparators.java:14-32``) and
  the window-all merge of ``KNNQuery.java:214-272`` including its bookkeeping bug.

Parity status: the reference ships no tests, fixtures or golden vectors
 and cannot be built or run here (Java; no JVM, no Maven
artefacts).  Grid/cell/set semantics are pinned by known-answer values derived
from the Java source (tests/golden/kat_grid.json); distance *bits* depend on
JTS 1.16.1 internals restated from its published algorithm -> "parity unpinned"
for distance bits (Parity).
"""
from __future__ import annotations

import math
import re
import struct
from fractions import Fraction

INT_MIN = -(1 << 31)
INT_MAX = (1 << 31) - 1
DBL_MAX = 1.7976931348623157e308
CELL_STR_LEN = 5  # UniformGrid.java:40


class NumberFormatException(Exception):
    pass


class SystemExit1(Exception):
    """Stands for ``System.exit(1)`` in ``UniformGrid.java:237-241,272-276``."""


# --------------------------------------------------------------------------------------
# Java scalar semantics
# --------------------------------------------------------------------------------------
def wrap32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def d2i(v: float) -> int:
    """Java ``(int)`` cast of a double (JLS 5.1.3): NaN -> 0, saturating."""
    if v != v:
        return 0
    if v >= 2147483647.0:
        return INT_MAX
    if v <= -2147483648.0:
        return INT_MIN
    return int(v)


def jfloor(v: float) -> float:
    if v != v or v in (math.inf, -math.inf):
        return v
    return float(math.floor(v))


def jceil(v: float) -> float:
    if v != v or v in (math.inf, -math.inf):
        return v
    return float(math.ceil(v))


def fmt05(i: int) -> str:
    """``String.format("%05d", i)`` (HelperClass.java:54-57)."""
    return "%05d" % i


_LEADING_ZEROS = re.compile(r"^0+(?!$)")


def parse_java_int(s: str) -> int:
    """``Integer.parseInt(s.replaceFirst("^0+(?!$)", ""))`` (HelperClass.java:60-63)."""
    s = _LEADING_ZEROS.sub("", s, count=1)
    if not s:
        raise NumberFormatException(s)
    body = s
    if s[0] in "+-":
        if len(s) == 1:
            raise NumberFormatException(s)
        body = s[1:]
    if not body.isdigit() or not body.isascii():
        raise NumberFormatException(s)
    v = int(s)
    if v < INT_MIN or v > INT_MAX:
        raise NumberFormatException(s)
    return v


def get_int_cell_indices(key: str):
    """HelperClass.getIntCellIndices (HelperClass.java:263-276)."""
    return parse_java_int(key[0:5]), parse_java_int(key[5:])


# --------------------------------------------------------------------------------------
# fdlibm e_hypot.c (JDK 8 StrictMath.hypot) -- JTS Coordinate.distance
# --------------------------------------------------------------------------------------
def _bits(d: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", d))[0]


def _from_bits(b: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", b & 0xFFFFFFFFFFFFFFFF))[0]


def _hi(d: float) -> int:
    return wrap32(_bits(d) >> 32)


def _lo(d: float) -> int:
    return _bits(d) & 0xFFFFFFFF


def _with_hi(d: float, hi: int) -> float:
    return _from_bits(((hi & 0xFFFFFFFF) << 32) | _lo(d))


def _hi_only(hi: int) -> float:
    return _from_bits((hi & 0xFFFFFFFF) << 32)


def fdlibm_hypot(x: float, y: float) -> float:
    ha = _hi(x) & 0x7FFFFFFF
    hb = _hi(y) & 0x7FFFFFFF
    if hb > ha:
        a, b = y, x
        ha, hb = hb, ha
    else:
        a, b = x, y
    a = _with_hi(a, ha)
    b = _with_hi(b, hb)
    if (ha - hb) > 0x3C00000:
        return a + b
    k = 0
    if ha > 0x5F300000:
        if ha >= 0x7FF00000:
            w = a + b
            if ((ha & 0xFFFFF) | _lo(a)) == 0:
                w = a
            if ((hb ^ 0x7FF00000) | _lo(b)) == 0:
                w = b
            return w
        ha -= 0x25800000
        hb -= 0x25800000
        k += 600
        a = _with_hi(a, ha)
        b = _with_hi(b, hb)
    if hb < 0x20B00000:
        if hb <= 0x000FFFFF:
            if (hb | _lo(b)) == 0:
                return a
            t1 = _hi_only(0x7FD00000)
            b *= t1
            a *= t1
            k -= 1022
        else:
            ha += 0x25800000
            hb += 0x25800000
            k -= 600
            a = _with_hi(a, ha)
            b = _with_hi(b, hb)
    w = a - b
    if w > b:
        t1 = _hi_only(ha)
        t2 = a - t1
        w = math.sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)))
    else:
        a = a + a
        y1 = _hi_only(hb)
        y2 = b - y1
        t1 = _hi_only(ha + 0x00100000)
        t2 = a - t1
        w = math.sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)))
    if k != 0:
        t1 = _hi_only(0x3FF00000 + (k << 20))
        return t1 * w
    return w


def coord_distance(ax, ay, bx, by) -> float:
    """JTS ``Coordinate.distance``: ``Math.hypot(x - c.x, y - c.y)``."""
    return fdlibm_hypot(ax - bx, ay - by)


def jts_point_point_distance(ax, ay, bx, by) -> float:
    """``a.point.distance(b.point)`` (DistanceFunctions.java:15-18) through JTS
    DistanceOp.computeMinDistancePoints: minDistance starts at Double.MAX_VALUE
    and is only replaced by a strictly smaller value (NaN never replaces)."""
    d = coord_distance(ax, ay, bx, by)
    return d if d < DBL_MAX else DBL_MAX


def point_to_segment(px, py, ax, ay, bx, by) -> float:
    """JTS 1.16.1 ``Distance.pointToSegment`` (op order as published)."""
    if ax == bx and ay == by:
        return coord_distance(px, py, ax, ay)
    len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay)
    r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2 if len2 != 0 else (
        math.copysign(math.inf, (px - ax) * (bx - ax) + (py - ay) * (by - ay))
        if ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) != 0 else math.nan)
    if r <= 0.0:
        return coord_distance(px, py, ax, ay)
    if r >= 1.0:
        return coord_distance(px, py, bx, by)
    num = (ay - py) * (bx - ax) - (ax - px) * (by - ay)
    s = num / len2 if len2 != 0 else (math.copysign(math.inf, num) if num != 0 else math.nan)
    return abs(s) * math.sqrt(len2)


def sign_of_det2x2(x1, y1, x2, y2) -> int:
    """Exact sign of x1*y2 - y1*x2 (what RobustDeterminant.signOfDet2x2 computes)."""
    det = Fraction(x1) * Fraction(y2) - Fraction(y1) * Fraction(x2)
    return (det > 0) - (det < 0)


EXTERIOR, BOUNDARY, INTERIOR = 2, 1, 0


def locate_point_in_ring(px, py, ring) -> int:
    """JTS 1.16.1 RayCrossingCounter.locatePointInRing / countSegment."""
    crossings = 0
    for i in range(1, len(ring)):
        p1x, p1y = ring[i]
        p2x, p2y = ring[i - 1]
        if p1x < px and p2x < px:
            continue
        if px == p2x and py == p2y:
            return BOUNDARY
        if p1y == py and p2y == py:
            minx, maxx = p1x, p2x
            if minx > maxx:
                minx, maxx = p2x, p1x
            if px >= minx and px <= maxx:
                return BOUNDARY
            continue
        if (p1y > py and p2y <= py) or (p2y > py and p1y <= py):
            x1 = p1x - px
            y1 = p1y - py
            x2 = p2x - px
            y2 = p2y - py
            s = sign_of_det2x2(x1, y1, x2, y2)
            if s == 0:
                return BOUNDARY
            if y2 < y1:
                s = -s
            if s > 0:
                crossings += 1
    return INTERIOR if crossings % 2 == 1 else EXTERIOR


def ring_envelope(ring):
    """JTS Envelope.expandToInclude over the ring coordinates."""
    minx, maxx, miny, maxy = 0.0, -1.0, 0.0, 0.0
    null = True
    for x, y in ring:
        if null:
            minx = maxx = x
            miny = maxy = y
            null = False
        else:
            if x < minx:
                minx = x
            if x > maxx:
                maxx = x
            if y < miny:
                miny = y
            if y > maxy:
                maxy = y
    return minx, miny, maxx, maxy


def env_point_distance(env, px, py) -> float:
    """JTS Envelope.distance(Envelope) of a ring envelope to a point's (1.16.1), the skip test
    of DistanceOp.computeMinDistance(LineString, Point)."""
    minx, miny, maxx, maxy = env
    if not (px > maxx or px < minx or py > maxy or py < miny):
        return 0.0
    dx = 0.0
    if maxx < px:
        dx = px - maxx
    elif minx > px:
        dx = minx - px
    dy = 0.0
    if maxy < py:
        dy = py - maxy
    elif miny > py:
        dy = miny - py
    if dx == 0.0:
        return dy
    if dy == 0.0:
        return dx
    return math.sqrt(dx * dx + dy * dy)


def _ring_location(px, py, ring) -> int:
    """PointLocator.locateInPolygonRing: envelope test, then RayCrossingCounter."""
    minx, miny, maxx, maxy = ring_envelope(ring)
    if px > maxx or px < minx or py > maxy or py < miny:
        return EXTERIOR
    return locate_point_in_ring(px, py, ring)


def jts_point_polygon_distance(px, py, poly) -> float:
    """``p.point.distance(polygon)`` (DistanceFunctions.java:33-36) via JTS DistanceOp.
    ``poly`` is a closed ring (shell only) or a Polygon from ``make_polygon`` (shell, holes).
    Containment first (PointLocator.locateInPolygon: shell EXTERIOR -> exterior, shell
    BOUNDARY -> boundary, then each hole in order: INTERIOR -> exterior, BOUNDARY ->
    boundary); not exterior -> 0.  Else the minimum over the rings' segments (shell, then
    holes), a ring skipped when its envelope is farther than the current minimum, MAX_VALUE
    start, strict ``<``, stop at 0."""
    rings = [poly] if poly and isinstance(poly[0][0], float) else list(poly)
    loc = _ring_location(px, py, rings[0])
    if loc == BOUNDARY:
        return 0.0
    if loc == INTERIOR:
        for hole in rings[1:]:
            h = _ring_location(px, py, hole)
            if h == INTERIOR:
                loc = EXTERIOR
                break
            if h == BOUNDARY:
                return 0.0
        if loc == INTERIOR:
            return 0.0
    md = DBL_MAX
    for ring in rings:
        if env_point_distance(ring_envelope(ring), px, py) > md:
            continue
        for i in range(len(ring) - 1):
            d = point_to_segment(px, py, ring[i][0], ring[i][1], ring[i + 1][0], ring[i + 1][1])
            if d < md:
                md = d
            if md <= 0.0:
                return md
    return md


def pp_euclid(lon, lat, lon1, lat1) -> float:
    """DistanceFunctions.getPointPointEuclideanDistance (DistanceFunctions.java:60-63):
    sqrt(pow(lat1-lat,2) + pow(lon1-lon,2)); Math.pow(v, 2) == v*v exactly."""
    dy = lat1 - lat
    dx = lon1 - lon
    return math.sqrt(dy * dy + dx * dx)


def bbox_border(x, y, x1, y1, x2, y2) -> float:
    """getPointLineStringNearestBBoxBorderMinEuclideanDistance (DistanceFunctions.java:134-146)."""
    if x1 == x2:
        return pp_euclid(x, y, x1, y)
    elif y1 == y2:
        return pp_euclid(x, y, x, y1)
    return 4.9e-324  # Double.MIN_VALUE


def bbox_distance(x, y, bbox) -> float:
    """getPointPolygonBBoxMinEuclideanDistance (DistanceFunctions.java:150-200)."""
    x1, y1, x2, y2 = bbox
    if x <= x1:
        if y <= y1:
            return pp_euclid(x, y, x1, y1)
        elif y >= y2:
            return pp_euclid(x, y, x1, y2)
        return bbox_border(x, y, x1, y1, x1, y2)
    elif x >= x2:
        if y <= y1:
            return pp_euclid(x, y, x2, y1)
        elif y >= y2:
            return pp_euclid(x, y, x2, y2)
        return bbox_border(x, y, x2, y1, x2, y2)
    else:
        if y <= y1:
            return bbox_border(x, y, x1, y1, x2, y1)
        elif y >= y2:
            return bbox_border(x, y, x1, y2, x2, y2)
        return 0.0


# --------------------------------------------------------------------------------------
# UniformGrid (UniformGrid.java) with string cell keys
# --------------------------------------------------------------------------------------
class UniformGrid:
    def __init__(self, n: int, min_x: float, max_x: float, min_y: float, max_y: float):
        """``UniformGrid(int uniformGridRows, ...)`` (UniformGrid.java:74-85)."""
        self.min_x, self.max_x, self.min_y, self.max_y = min_x, max_x, min_y, max_y
        self.n = n
        self.cell_len = (max_x - min_x) / n

    @classmethod
    def from_cell_length(cls, cell_length, min_x, max_x, min_y, max_y):
        """``UniformGrid(double cellLength, ...)`` (UniformGrid.java:47-72, 114-134)."""
        g = cls.__new__(cls)
        xd, yd = max_x - min_x, max_y - min_y
        if xd > yd:
            diff = xd - yd
            max_y += diff / 2
            min_y -= diff / 2
        elif yd > xd:
            diff = yd - xd
            max_x += diff / 2
            min_x -= diff / 2
        g.min_x, g.max_x, g.min_y, g.max_y = min_x, max_x, min_y, max_y
        grid_len = pp_euclid(min_x, min_y, max_x, min_y)
        rows = grid_len / cell_length
        g.n = 1 if rows < 1 else d2i(jceil(rows))
        g.cell_len = (max_x - min_x) / g.n
        return g

    # HelperClass.assignGridCellID(Coordinate, UniformGrid) (HelperClass.java:104-120)
    def cell_indices(self, x: float, y: float):
        cx = d2i(jfloor((x - self.min_x) / self.cell_len))
        cy = d2i(jfloor((y - self.min_y) / self.cell_len))
        return cx, cy

    def key(self, x: float, y: float) -> str:
        cx, cy = self.cell_indices(x, y)
        return fmt05(cx) + fmt05(cy)

    def valid_key(self, i, j):  # UniformGrid.java:224-229
        return 0 <= i < self.n and 0 <= j < self.n

    def guaranteed_layers(self, r):  # UniformGrid.java:427-438
        diag = self.cell_len * math.sqrt(2)
        return d2i(jfloor((r / diag) - 1))

    def candidate_layers(self, r):  # UniformGrid.java:440-444
        return d2i(jceil(r / self.cell_len))

    def _square(self, ci, cj, layers, exclude=None):
        lo_i, hi_i = wrap32(ci - layers), wrap32(ci + layers)
        lo_j, hi_j = wrap32(cj - layers), wrap32(cj + layers)
        out = set()
        if lo_i > hi_i or lo_j > hi_j:
            return out
        if hi_i == INT_MAX or hi_j == INT_MAX:
            raise RuntimeError("reference loop does not terminate (i <= Integer.MAX_VALUE)")
        # the Java loops visit every (i,j) and keep validKey ones; visiting only the
        # valid sub-range gives the identical set
        for i in range(max(lo_i, 0), min(hi_i, self.n - 1) + 1):
            for j in range(max(lo_j, 0), min(hi_j, self.n - 1) + 1):
                k = fmt05(i) + fmt05(j)
                if exclude is None or k not in exclude:
                    out.add(k)
        return out

    def guaranteed_cells(self, r, qkey):  # UniformGrid.java:165-190
        lg = self.guaranteed_layers(r)
        if lg == 0:
            return {qkey}
        if lg > 0:
            ci, cj = get_int_cell_indices(qkey)
            return self._square(ci, cj, lg)
        return set()

    def guaranteed_cells_poly(self, r, grid_ids):  # UniformGrid.java:193-206
        out = set()
        for cid in grid_ids:
            out |= self.guaranteed_cells(r, cid)
        return out

    def candidate_cells(self, r, qkey, gset):  # UniformGrid.java:367-394
        lc = self.candidate_layers(r)
        if lc > 0:
            ci, cj = get_int_cell_indices(qkey)
            return self._square(ci, cj, lc, exclude=gset)
        return set()

    def candidate_cells_poly(self, r, grid_ids, gset):  # UniformGrid.java:398-410
        out = set()
        for cid in grid_ids:
            out |= self.candidate_cells(r, cid, gset)
        return out

    def all_cells(self):  # UniformGrid.java:87-105 (girdCellsSet)
        return {fmt05(i) + fmt05(j) for i in range(self.n) for j in range(self.n)}

    def neighboring_cells(self, r, qkey):  # UniformGrid.java:261-293
        if r == 0:
            return self.all_cells()
        lc = self.candidate_layers(r)
        if lc <= 0:
            raise SystemExit1("candidateNeighboringLayers cannot be 0 or less")
        ci, cj = get_int_cell_indices(qkey)
        return self._square(ci, cj, lc)


def bbox_grid_ids(grid: UniformGrid, bbox):
    """HelperClass.assignGridCellID(bbox, uGrid) (HelperClass.java:123-143)."""
    minx, miny, maxx, maxy = bbox
    x1 = d2i(jfloor((minx - grid.min_x) / grid.cell_len))
    y1 = d2i(jfloor((miny - grid.min_y) / grid.cell_len))
    x2 = d2i(jfloor((maxx - grid.min_x) / grid.cell_len))
    y2 = d2i(jfloor((maxy - grid.min_y) / grid.cell_len))
    if x2 == INT_MAX or y2 == INT_MAX:
        raise RuntimeError("reference loop does not terminate")
    return {fmt05(x) + fmt05(y) for x in range(x1, x2 + 1) for y in range(y1, y2 + 1)}


def close_ring(coords):
    """Polygon.createPolygon ring closure (Polygon.java:147-155); needs > 3 coords (Polygon.java:53)."""
    ring = [(float(x), float(y)) for x, y in coords]
    if len(ring) <= 3:
        return None
    if not (ring[0][0] == ring[-1][0] and ring[0][1] == ring[-1][1]):
        ring.append(ring[0])
    return ring


def ring_area(ring) -> float:
    """JTS 1.16.1 Polygon.getArea of a shell-only polygon: |Area.ofRingSigned| (shoelace with
    the first x subtracted)."""
    n = len(ring)
    if n < 3:
        return 0.0
    x0 = ring[0][0]
    s = 0.0
    for i in range(1, n - 1):
        s += (ring[i][0] - x0) * (ring[i - 1][1] - ring[i + 1][1])
    return abs(s / 2.0)


def make_polygon(rings_in):
    """Polygon(List<List<Coordinate>>, UniformGrid).createPolygon (Polygon.java:52-66, 115-165):
    one ring -> closed shell; several -> every ring padded (1-3 coords: first coordinate appended
    4 times) and closed, then ordered by area, largest first, with createPolygonArray's insertion
    rule (ties at the tail go after, in the middle before; a NaN area is never inserted); shell =
    first, holes = the rest.  Returns the list of closed rings [shell, holes...] or None when the
    constructor leaves polygon null (first ring <= 3 coords); ValueError where JTS throws
    (an empty ring, a ring whose first coordinate is NaN: not closed)."""
    rings = [[(float(x), float(y)) for x, y in r] for r in rings_in]
    if not rings or len(rings[0]) <= 3:
        return None
    if len(rings) == 1:
        ring = rings[0]
        if not (ring[0][0] == ring[-1][0] and ring[0][1] == ring[-1][1]):
            ring.append(ring[0])
        if not (ring[0][0] == ring[-1][0] and ring[0][1] == ring[-1][1]):
            raise ValueError("Points of LinearRing do not form a closed linestring")
        return [ring]
    ordered = []  # (area, ring)
    for ring in rings:
        if not ring:
            raise ValueError("IndexOutOfBoundsException: empty ring")
        if len(ring) < 4:
            ring = ring + [ring[0]] * 4
        if not (ring[0][0] == ring[-1][0] and ring[0][1] == ring[-1][1]):
            ring.append(ring[0])
        if not (ring[0][0] == ring[-1][0] and ring[0][1] == ring[-1][1]):
            raise ValueError("Points of LinearRing do not form a closed linestring")
        a = ring_area(ring)
        if not ordered or ordered[-1][0] >= a:
            ordered.append((a, ring))
        else:
            for i in range(len(ordered)):
                if ordered[i][0] <= a:
                    ordered.insert(i, (a, ring))
                    break
    return [r for _, r in ordered]


def polygon_of(coords):
    """A query polygon given as one ring (list of (x, y)) or as rings (list of lists)."""
    if coords and isinstance(coords[0][0], (list, tuple)):
        return make_polygon(coords)
    return make_polygon([coords])


# --------------------------------------------------------------------------------------
# Window queries (one window's contents; ids = window-local index)
# --------------------------------------------------------------------------------------
def range_pp(grid, xs, ys, qx, qy, r, approximate=False):
    """PointPointRangeQuery window body (PointPointRangeQuery.java:86-137)."""
    qkey = grid.key(qx, qy)
    G = grid.guaranteed_cells(r, qkey)
    C = grid.candidate_cells(r, qkey, G)
    out = []
    for i, (x, y) in enumerate(zip(xs, ys)):
        k = grid.key(x, y)
        if not (k in C or k in G):  # filter :102-107
            continue
        if k in G:
            out.append(i)
        elif approximate:
            out.append(i)
        elif jts_point_point_distance(qx, qy, x, y) <= r:
            out.append(i)
    return out


class JavaPriorityQueue:
    """Literal java.util.PriorityQueue (binary heap, comparator, array iteration order)."""

    def __init__(self, cmp):
        self.q = []
        self.cmp = cmp

    def size(self):
        return len(self.q)

    def peek(self):
        return self.q[0] if self.q else None

    def offer(self, e):
        self.q.append(e)
        self._sift_up(len(self.q) - 1, e)

    add = offer

    def _sift_up(self, k, x):
        q = self.q
        while k > 0:
            parent = (k - 1) >> 1
            e = q[parent]
            if self.cmp(x, e) >= 0:
                break
            q[k] = e
            k = parent
        q[k] = x

    def _sift_down(self, k, x):
        q = self.q
        n = len(q)
        half = n >> 1
        while k < half:
            child = (k << 1) + 1
            c = q[child]
            right = child + 1
            if right < n and self.cmp(c, q[right]) > 0:
                child = right
                c = q[child]
            if self.cmp(x, c) <= 0:
                break
            q[k] = c
            k = child
        q[k] = x

    def poll(self):
        if not self.q:
            return None
        result = self.q[0]
        x = self.q.pop()
        if self.q:
            self._sift_down(0, x)
        return result

    def remove_at(self, i):
        s = len(self.q) - 1
        if s == i:
            self.q.pop()
        else:
            moved = self.q.pop()
            self._sift_down(i, moved)
            if self.q[i] is moved:
                self._sift_up(i, moved)

    def remove(self, o):
        for i, e in enumerate(self.q):
            if e is o:
                self.remove_at(i)
                return True
        return False

    def __iter__(self):
        return iter(list(self.q))


def _dist_cmp(t1, t2):
    """Comparators.inTuplePointDistanceComparator (Comparators.java:18-31)."""
    d1, d2 = t1[1], t2[1]
    if d1 > d2:
        return -1
    elif d1 == d2:
        return 0
    return 1


def knn_pp_literal(grid, xs, ys, qx, qy, r, k, cell_order=None):
    """Literal RealTime-mode kNN: per-cell PriorityQueue (PointPointKNNQuery.java:86-111)
    then kNNWinAllEvaluationPointStream (KNNQuery.java:214-271).  Returns the merged
    queue's contents in heap (array) order as (idx, dist) tuples.  Cells are merged in
    ``cell_order`` (default: sorted cell key) -- in Flink this order is arrival order."""
    qkey = grid.key(qx, qy)
    G = grid.guaranteed_cells(r, qkey)
    C = grid.candidate_cells(r, qkey, G)
    per_cell = {}
    for i, (x, y) in enumerate(zip(xs, ys)):
        key = grid.key(x, y)
        if key in C or key in G:
            per_cell.setdefault(key, []).append(i)
    heaps = {}
    for key, idxs in per_cell.items():
        pq = JavaPriorityQueue(_dist_cmp)
        for i in idxs:
            d = jts_point_point_distance(qx, qy, xs[i], ys[i])
            if pq.size() < k:
                pq.offer((i, d))
            elif pq.peek()[1] > d:
                pq.poll()
                pq.offer((i, d))
        heaps[key] = pq
    order = cell_order if cell_order is not None else sorted(heaps)
    allpq = JavaPriorityQueue(_dist_cmp)
    ids = set()
    for key in order:
        for cand in heaps[key]:
            if allpq.size() < k:
                if cand[0] not in ids:
                    allpq.add(cand)
                    ids.add(cand[0])
                else:
                    for ex in allpq:
                        if ex[0] == cand[0] and ex[1] > cand[1]:
                            allpq.remove(ex)
                            allpq.add(cand)
                            break
            else:
                if allpq.peek()[1] > cand[1]:
                    if cand[0] not in ids:
                        allpq.poll()
                        head = allpq.peek()  # KNNQuery.java:250-251 (removes the NEW head's id)
                        if head is None:
                            raise RuntimeError("NullPointerException (k == 1) at KNNQuery.java:251")
                        ids.discard(head[0])
                        allpq.offer(cand)
                        ids.add(cand[0])
                    else:
                        for ex in allpq:
                            if ex[0] == cand[0] and ex[1] > cand[1]:
                                allpq.remove(ex)
                                allpq.offer(cand)
                                break
    return list(allpq)


def knn_pp(grid, xs, ys, qx, qy, r, k):
    """Build contract: the k smallest (dist, idx) over G u C,
    ascending.  Equal to knn_pp_literal's set whenever no exact tie straddles rank k."""
    qkey = grid.key(qx, qy)
    G = grid.guaranteed_cells(r, qkey)
    C = grid.candidate_cells(r, qkey, G)
    cand = []
    for i, (x, y) in enumerate(zip(xs, ys)):
        key = grid.key(x, y)
        if key in C or key in G:
            cand.append((jts_point_point_distance(qx, qy, x, y), i))
    cand.sort()
    return [(i, d) for d, i in cand[:k]]


def join_pp(ugrid, qgrid, dxs, dys, qxs, qys, r, approximate=False):
    """PointPointJoinQuery window join (PointPointJoinQuery.java:113-172) with the query
    stream replicated by JoinQuery.getReplicatedPointQueryStream (JoinQuery.java:73-90)."""
    repl = {}
    for qi, (qx, qy) in enumerate(zip(qxs, qys)):
        for key in qgrid.neighboring_cells(r, qgrid.key(qx, qy)):
            repl.setdefault(key, []).append(qi)
    out = []
    for pi, (x, y) in enumerate(zip(dxs, dys)):
        key = ugrid.key(x, y)
        for qi in repl.get(key, ()):
            if approximate or jts_point_point_distance(x, y, qxs[qi], qys[qi]) <= r:
                out.append((pi, qi))
    return out


def range_ppoly(grid, xs, ys, rings, r, approximate=False):
    """PointPolygonRangeQuery window body (PointPolygonRangeQuery.java:76-124), one
    independent query per polygon; returns (poly_idx, point_idx) pairs."""
    out = []
    for pi, coords in enumerate(rings):
        ring = polygon_of(coords)
        if ring is None:
            raise ValueError("polygon needs more than 3 coordinates (Polygon.java:53)")
        bbox = ring_envelope(ring[0])
        ids = bbox_grid_ids(grid, bbox)
        G = grid.guaranteed_cells_poly(r, ids)
        C = grid.candidate_cells_poly(r, ids, G)
        for i, (x, y) in enumerate(zip(xs, ys)):
            key = grid.key(x, y)
            if not (key in C or key in G):
                continue
            if key in G:
                out.append((pi, i))
                continue
            d = bbox_distance(x, y, bbox) if approximate else jts_point_polygon_distance(x, y, ring)
            if d <= r:
                out.append((pi, i))
    return out


def join_ppoly(ugrid, qgrid, xs, ys, rings, r, approximate=False):
    """PointPolygonJoinQuery window join (PointPolygonJoinQuery.java:162-201): each polygon is
    replicated once per cell of G and of C computed on qGrid (JoinQuery.java:93-115); a point
    joins a copy iff its uGrid gridID string equals the copy's gridID; JoinFunction emits when
    approximate or JTS distance <= r (no guaranteed shortcut).  Returns (point_idx, poly_idx)."""
    out = []
    for pi, coords in enumerate(rings):
        ring = polygon_of(coords)
        if ring is None:
            raise ValueError("polygon needs more than 3 coordinates (Polygon.java:53)")
        ids = bbox_grid_ids(qgrid, ring_envelope(ring[0]))
        G = qgrid.guaranteed_cells_poly(r, ids)
        C = qgrid.candidate_cells_poly(r, ids, G)
        replicated = G | C  # disjoint sets: one copy per key
        for i, (x, y) in enumerate(zip(xs, ys)):
            if ugrid.key(x, y) not in replicated:
                continue
            if approximate or jts_point_polygon_distance(x, y, ring) <= r:
                out.append((i, pi))
    return out


def knn_ppoly(grid, xs, ys, coords, r, k, approximate=False):
    """PointPolygonKNNQuery window body (PointPolygonKNNQuery.java:162-236) under the build
    contract of knn_pp: per-cell max-heaps of size k (replace only when the head is larger,
    :199-221) over the points of G u C, then the k smallest (distance, idx) over all cells,
    ascending.  A NaN (approximate bbox distance of a NaN coordinate) ranks last."""
    ring = polygon_of(coords)
    if ring is None:
        raise ValueError("polygon needs more than 3 coordinates (Polygon.java:53)")
    bbox = ring_envelope(ring[0])
    ids = bbox_grid_ids(grid, bbox)
    G = grid.guaranteed_cells_poly(r, ids)
    C = grid.candidate_cells_poly(r, ids, G)
    cells = {}
    for i, (x, y) in enumerate(zip(xs, ys)):
        key = grid.key(x, y)
        if key in C or key in G:
            d = bbox_distance(x, y, bbox) if approximate else jts_point_polygon_distance(x, y, ring)
            cells.setdefault(key, []).append((i, d))

    def rank(e):
        d = e[1]
        return (math.inf, 1, e[0]) if d != d else (d, 0, e[0])
    merged = []
    for pts in cells.values():
        merged += sorted(pts, key=rank)[:k]  # the cell's k smallest (unique idx)
    return sorted(merged, key=rank)[:k]
