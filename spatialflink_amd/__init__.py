"""spatialflink_amd -- MI355X-native (gfx950 HIP) evaluation of GeoFlink's windowed spatial
queries behind a C ABI (include/geohip.h, libgeohip.so), with a host-side mirror of the
reference operator API (spatialflink_amd.operators).  See DESIGN.md."""
from . import _abi
from ._abi import Context, GeohipError, GeohipArgumentError, GeohipCapacityError, GeohipDeviceError
from .operators import (QueryConfiguration, QueryType, UniformGrid, Point, Polygon, PointWindow,
                        PointPointRangeQuery, PointPointKNNQuery, PointPointJoinQuery, PointPolygonRangeQuery,
                        PointPolygonJoinQuery, PointPolygonKNNQuery)

__all__ = ["Context", "GeohipError", "GeohipArgumentError", "GeohipCapacityError", "GeohipDeviceError",
           "QueryConfiguration", "QueryType", "UniformGrid", "Point", "Polygon", "PointWindow",
           "PointPointRangeQuery", "PointPointKNNQuery", "PointPointJoinQuery", "PointPolygonRangeQuery",
           "PointPolygonJoinQuery", "PointPolygonKNNQuery"]
