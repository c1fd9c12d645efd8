"""Host-side mirror of GeoFlink's operator API for the windowed hot path.

Same names, argument meaning and error behaviour as the Java classes (paths relative to
``/root/reference/src/main/java/GeoFlink``); each ``run`` evaluates ONE window's contents
(the caller assembles windows, as Flink's ``SlidingProcessingTimeWindows`` does) on the
MI355X through libgeohip:

====================================  =========================================================
``UniformGrid``                       ``spatialIndices/UniformGrid.java:47-85`` (both ctors)
``QueryConfiguration`` / ``QueryType`` ``spatialOperators/QueryConfiguration.java:5-56``, ``QueryType.java:3-6``
``Point`` / ``Polygon`` / windows      ``spatialObjects/Point.java:60-111``, ``Polygon.java:52-66``
``PointPointRangeQuery.run``          ``spatialOperators/range/PointPointRangeQuery.java:36-141``
``PointPointKNNQuery.run``            ``spatialOperators/knn/PointPointKNNQuery.java:33-191``
``PointPointJoinQuery.run``           ``spatialOperators/join/PointPointJoinQuery.java:24-172``
``PointPolygonRangeQuery.run``        ``spatialOperators/range/PointPolygonRangeQuery.java:30-128``
====================================  =========================================================

Window contents are columnar (``PointWindow``: x, y and optional object ids); results are
window-local indices (mapping back to the caller's Point objects, the way the JNI shim in
INTEGRATION.md maps them back to Java ``Point`` instances).
"""
from __future__ import annotations

import enum
import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import _abi


class QueryType(enum.Enum):  # QueryType.java:3-6
    RealTime = "RealTime"
    WindowBased = "WindowBased"
    CountBased = "CountBased"


@dataclass
class QueryConfiguration:  # QueryConfiguration.java:5-56
    query_type: QueryType = QueryType.WindowBased
    window_size: int = 10
    slide_step: int = 5
    allowed_lateness: int = 0
    approximate_query: bool = False

    def isApproximateQuery(self) -> bool:
        return self.approximate_query

    def getQueryType(self) -> QueryType:
        return self.query_type


class UniformGrid:
    """UniformGrid (UniformGrid.java).  Only its numeric state crosses the ABI."""

    CELLINDEXSTRLENGTH = 5

    def __init__(self, uniform_grid_rows: int, min_x: float, max_x: float, min_y: float, max_y: float):
        # UniformGrid(int uniformGridRows, ...) (UniformGrid.java:74-85)
        self.minX, self.maxX, self.minY, self.maxY = float(min_x), float(max_x), float(min_y), float(max_y)
        self.numGridPartitions = int(uniform_grid_rows)
        self.cellLength = (self.maxX - self.minX) / uniform_grid_rows

    @classmethod
    def from_cell_length(cls, cell_length: float, min_x, max_x, min_y, max_y) -> "UniformGrid":
        """UniformGrid(double cellLength, ...) (UniformGrid.java:47-72, adjust :114-134)."""
        g = cls.__new__(cls)
        min_x, max_x, min_y, max_y = float(min_x), float(max_x), float(min_y), float(max_y)
        xd, yd = max_x - min_x, max_y - min_y
        if xd > yd:
            diff = xd - yd
            max_y += diff / 2
            min_y -= diff / 2
        elif yd > xd:
            diff = yd - xd
            max_x += diff / 2
            min_x -= diff / 2
        g.minX, g.maxX, g.minY, g.maxY = min_x, max_x, min_y, max_y
        dy, dx = min_y - min_y, max_x - min_x
        grid_length = math.sqrt(dy * dy + dx * dx)  # getPointPointEuclideanDistance
        rows = grid_length / cell_length
        g.numGridPartitions = 1 if rows < 1 else int(math.ceil(rows))
        g.cellLength = (g.maxX - g.minX) / g.numGridPartitions
        return g

    def getMinX(self): return self.minX
    def getMinY(self): return self.minY
    def getMaxX(self): return self.maxX
    def getMaxY(self): return self.maxY
    def getCellLength(self): return self.cellLength
    def getNumGridPartitions(self): return self.numGridPartitions
    def getCellIndexStrLength(self): return self.CELLINDEXSTRLENGTH

    def abi(self) -> _abi.Grid:
        return _abi.make_grid(self.minX, self.minY, self.cellLength, self.numGridPartitions)

    def cell_of(self, x: float, y: float):
        """HelperClass.assignGridCellID as integer indices (computed by libgeohip's planner)."""
        return _abi.plan_cell(self.abi(), x, y)

    def grid_id(self, x: float, y: float) -> str:
        cx, cy = self.cell_of(x, y)
        return "%05d%05d" % (cx, cy)


@dataclass
class Point:
    """Query point (Point.java:60-67 computes gridID at construction)."""
    x: float
    y: float
    objID: Optional[str] = None
    timeStampMillisec: int = 0


@dataclass
class Polygon:
    """Query polygon as given to Polygon(List<List<Coordinate>>, UniformGrid): either one ring
    ([(x, y), ...]) or a list of rings ([[(x, y), ...], ...]; the largest JTS area becomes the
    shell, the others its holes -- Polygon.createPolygon, Polygon.java:115-165)."""
    coordinates: Sequence
    objID: Optional[str] = None

    def __post_init__(self):
        rings = self.rings
        if not rings or len(rings[0]) <= 3:  # Polygon.java:53 leaves polygon == null
            raise _abi.GeohipArgumentError("Polygon needs more than 3 coordinates (Polygon.java:53)")

    @property
    def rings(self):
        c = self.coordinates
        if len(c) and len(c[0]) and isinstance(c[0][0], (list, tuple, np.ndarray)):
            return [list(r) for r in c]
        return [list(c)]


@dataclass
class PointWindow:
    """One window's points, columnar (x, y float64; host numpy or device torch)."""
    x: object
    y: object
    obj_ids: Optional[np.ndarray] = None
    start: int = 0
    end: int = 0

    def __len__(self):
        return len(self.x)


_ctx_cache: dict = {}


def default_context(device: int = 0) -> _abi.Context:
    ctx = _ctx_cache.get(device)
    if ctx is None:
        ctx = _ctx_cache[device] = _abi.Context(device)
    return ctx


class _Operator:
    def __init__(self, conf: QueryConfiguration, index: UniformGrid, ctx: Optional[_abi.Context] = None):
        self.conf = conf
        self.index = index
        self.ctx = ctx

    def _ctx(self) -> _abi.Context:
        return self.ctx or default_context()

    def getQueryConfiguration(self):
        return self.conf

    def getSpatialIndex(self):
        return self.index

    def _check_type(self):
        qt = self.conf.query_type
        if qt not in (QueryType.RealTime, QueryType.WindowBased):
            raise _abi.GeohipArgumentError("Not yet support")  # IllegalArgumentException in run()


class PointPointRangeQuery(_Operator):
    """PointPointRangeQuery.run (PointPointRangeQuery.java:36-141): indices of window points
    in guaranteed cells, or in candidate cells within ``query_radius`` (``<=``; all candidate
    points when the configuration is approximate)."""

    def run(self, window: PointWindow, query_point: Point, query_radius: float):
        self._check_type()
        return self._ctx().range_pp(self.index.abi(), window.x, window.y, query_point.x, query_point.y,
                                    float(query_radius), self.conf.approximate_query)


    def queryIncremental(self, panes, query_point: Point, query_radius: float):
        """PointPointRangeQuery.queryIncremental (PointPointRangeQuery.java:144-245): ``panes`` is
        the stream cut into slides (PointWindow each); yields each sliding window's result
        (window-local indices) with every point evaluated once (spatialflink_amd.incremental)."""
        from .incremental import IncrementalRange, panes_per_window
        self._check_type()
        inc = IncrementalRange(self._ctx(), self.index.abi(), query_point.x, query_point.y, float(query_radius),
                               self.conf.approximate_query,
                               panes_per_window(self.conf.window_size, self.conf.slide_step))
        for pane in panes:
            inc.push(pane.x, pane.y)
            yield inc.window_local()


class PointPointKNNQuery(_Operator):
    """PointPointKNNQuery.run (PointPointKNNQuery.java:33-191): the window's k nearest
    points among guaranteed u candidate cells, ascending (distance, index); no radius filter
    (r only selects the cells)."""

    def run(self, window: PointWindow, query_point: Point, query_radius: float, k: int):
        self._check_type()
        return self._ctx().knn_pp(self.index.abi(), window.x, window.y, query_point.x, query_point.y,
                                  float(query_radius), int(k))

    def queryIncremental(self, panes, query_point: Point, query_radius: float, k: int):
        """Sliding-window kNN with pane reuse (device panes): yields each window's (idx, dist),
        the k smallest (dist, idx) over the window's last window_size / slide_step panes."""
        from .incremental import IncrementalKNN, panes_per_window
        self._check_type()
        inc = IncrementalKNN(self._ctx(), self.index.abi(), query_point.x, query_point.y, float(query_radius), int(k),
                             panes_per_window(self.conf.window_size, self.conf.slide_step))
        for pane in panes:
            yield inc.push(pane.x, pane.y)


class PointPointJoinQuery(_Operator):
    """PointPointJoinQuery.run (PointPointJoinQuery.java:24-172): (data index, query index)
    pairs with the data point's uGrid cell in the query's qGrid neighbourhood and
    distance <= r (all such pairs when approximate)."""

    def __init__(self, conf: QueryConfiguration, index1: UniformGrid, index2: UniformGrid,
                 ctx: Optional[_abi.Context] = None):
        super().__init__(conf, index1, ctx)
        self.index2 = index2

    def run(self, ordinary: PointWindow, queries: PointWindow, query_radius: float):
        self._check_type()
        return self._ctx().join_pp(self.index.abi(), self.index2.abi(), ordinary.x, ordinary.y, queries.x,
                                   queries.y, float(query_radius), self.conf.approximate_query)


class PointPolygonRangeQuery(_Operator):
    """PointPolygonRangeQuery.run (PointPolygonRangeQuery.java:30-128) for one or many
    independent query polygons; returns (polygon index, point index) pairs."""

    def run(self, window: PointWindow, query_polygons, query_radius: float):
        self._check_type()
        polys = [query_polygons] if isinstance(query_polygons, Polygon) else list(query_polygons)
        pr, off, vx, vy = _rings(polys)
        return self._ctx().range_ppoly(self.index.abi(), window.x, window.y, off, vx, vy, float(query_radius),
                                       self.conf.approximate_query, poly_rings=pr)


def _rings(polys):
    """(poly_rings, ring_off, vx, vy) of a polygon list: polygon i = rings
    [poly_rings[i], poly_rings[i+1]), ring j = vertices [ring_off[j], ring_off[j+1])."""
    pr, off, vx, vy = [0], [0], [], []
    for p in polys:
        for ring in p.rings:
            for c in ring:
                vx.append(float(c[0]))
                vy.append(float(c[1]))
            off.append(len(vx))
        pr.append(len(off) - 1)
    return np.array(pr, np.uint32), np.array(off, np.uint32), np.array(vx), np.array(vy)


class PointPolygonJoinQuery(_Operator):
    """PointPolygonJoinQuery.run (PointPolygonJoinQuery.java:27-201): the polygon stream is
    replicated to each polygon's guaranteed and candidate cells on the query grid
    (JoinQuery.getReplicatedPolygonQueryStream, JoinQuery.java:93-115) and joined with the
    points' gridIDs; returns (point index, polygon index) pairs with JTS distance <= r (every
    such pair when approximate)."""

    def __init__(self, conf: QueryConfiguration, index1: UniformGrid, index2: UniformGrid,
                 ctx: Optional[_abi.Context] = None):
        super().__init__(conf, index1, ctx)
        self.index2 = index2

    def run(self, points: PointWindow, query_polygons, query_radius: float):
        self._check_type()
        polys = [query_polygons] if isinstance(query_polygons, Polygon) else list(query_polygons)
        pr, off, vx, vy = _rings(polys)
        return self._ctx().join_ppoly(self.index.abi(), self.index2.abi(), points.x, points.y, off, vx, vy,
                                      float(query_radius), self.conf.approximate_query, poly_rings=pr)


class PointPolygonKNNQuery(_Operator):
    """PointPolygonKNNQuery.run (PointPolygonKNNQuery.java:34-236): the window's k nearest
    points to one query polygon among its guaranteed u candidate cells, ascending
    (distance, index); distance = JTS point.distance(polygon) or, when approximate, the
    bounding-box distance (DistanceFunctions.java:150-200)."""

    def run(self, window: PointWindow, query_polygon: Polygon, query_radius: float, k: int):
        self._check_type()
        _, off, vx, vy = _rings([query_polygon])
        return self._ctx().knn_ppoly(self.index.abi(), window.x, window.y, vx, vy, float(query_radius), int(k),
                                     self.conf.approximate_query, ring_off=off)
