"""ctypes binding of the C oracle (oracle/geohip_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by spatialflink_amd.
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "libgeohip_oracle.so"


class Grid(ctypes.Structure):
    _fields_ = [("min_x", c_double), ("min_y", c_double), ("cell_len", c_double), ("n", c_int32)]


class IngestSpec(ctypes.Structure):
    _fields_ = [("format", c_int32), ("delim", c_int32), ("fx", c_int32), ("fy", c_int32), ("fts", c_int32),
                ("foid", c_int32)]


class TrajSpec(ctypes.Structure):
    _fields_ = [("date_format", c_int32), ("utc_offset_min", c_int32), ("prop_ts", ctypes.c_char * 60),
                ("prop_oid", ctypes.c_char * 60)]


def _load():
    if not LIB.exists():
        import subprocess
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    lib = ctypes.CDLL(str(LIB))
    sig = {
        "geohip_oracle_hypot": (c_double, [c_double, c_double]),
        "geohip_oracle_pp_distance": (c_double, [c_double] * 4),
        "geohip_oracle_point_segment": (c_double, [c_double] * 6),
        "geohip_oracle_point_polygon": (c_double, [c_double, c_double, c_void_p, c_void_p, c_int]),
        "geohip_oracle_bbox_distance": (c_double, [c_double] * 6),
        "geohip_oracle_d2i": (c_int32, [c_double]),
        "geohip_oracle_cell": (None, [POINTER(Grid), c_double, c_double, POINTER(c_int32), POINTER(c_int32)]),
        "geohip_oracle_layers_guaranteed": (c_int32, [POINTER(Grid), c_double]),
        "geohip_oracle_layers_candidate": (c_int32, [POINTER(Grid), c_double]),
        "geohip_oracle_key_roundtrip": (c_int, [c_int32, c_int32, POINTER(c_int32), POINTER(c_int32)]),
        "geohip_oracle_key_matches": (c_int, [c_int32, c_int32, c_void_p, c_int]),
        "geohip_oracle_range_pp": (c_int64, [POINTER(Grid), c_void_p, c_void_p, c_uint64, c_double, c_double,
                                             c_double, c_int, c_void_p, c_uint64, POINTER(c_uint64)]),
        "geohip_oracle_knn_pp": (c_int, [POINTER(Grid), c_void_p, c_void_p, c_uint64, c_double, c_double, c_double,
                                         c_uint32, c_void_p, c_void_p, POINTER(c_uint32)]),
        "geohip_oracle_join_pp": (c_int64, [POINTER(Grid), POINTER(Grid), c_void_p, c_void_p, c_uint64, c_void_p,
                                            c_void_p, c_uint64, c_double, c_int, c_void_p, c_uint64,
                                            POINTER(c_uint64)]),
        "geohip_oracle_ingest_record": (c_int, [POINTER(IngestSpec), POINTER(Grid), ctypes.c_char_p, c_uint64,
                                                POINTER(c_double), POINTER(c_double), POINTER(c_int64),
                                                POINTER(c_uint32)]),
        "geohip_oracle_ingest": (c_int64, [POINTER(IngestSpec), POINTER(Grid), c_void_p, c_uint64, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_uint64]),
        "geohip_oracle_ingest_traj": (c_int64, [POINTER(IngestSpec), POINTER(TrajSpec), POINTER(Grid), c_void_p,
                                                c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64,
                                                c_void_p, c_uint64]),
        "geohip_oracle_range_ppoly": (c_int64, [POINTER(Grid), c_void_p, c_void_p, c_uint64, c_void_p, c_void_p,
                                                c_void_p, c_void_p, c_uint32, c_double, c_int, c_void_p, c_uint64,
                                                POINTER(c_uint64)]),
        "geohip_oracle_join_ppoly": (c_int64, [POINTER(Grid), POINTER(Grid), c_void_p, c_void_p, c_uint64, c_void_p,
                                               c_void_p, c_void_p, c_void_p, c_uint32, c_double, c_int, c_void_p,
                                               c_uint64, POINTER(c_uint64)]),
        "geohip_oracle_knn_ppoly": (c_int, [POINTER(Grid), c_void_p, c_void_p, c_uint64, c_void_p, c_uint32, c_void_p,
                                            c_void_p, c_double, c_uint32, c_int, c_void_p, c_void_p,
                                            POINTER(c_uint32)]),
        "geohip_oracle_point_polygon_rings": (c_double, [c_double, c_double, c_void_p, c_uint32, c_void_p, c_void_p,
                                                         POINTER(c_int)]),
        "geohip_oracle_set_threads": (None, [c_int]),
        "geohip_oracle_threads": (c_int, []),
        "geohip_oracle_mix64": (c_uint64, [c_uint64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


class OracleError(RuntimeError):
    pass


def grid(min_x, min_y, cell_len, n) -> Grid:
    return Grid(float(min_x), float(min_y), float(cell_len), int(n))


def _p(a):
    return a.ctypes.data_as(c_void_p)


def hypot(x, y):
    return lib.geohip_oracle_hypot(x, y)


def cell(g: Grid, x, y):
    cx, cy = c_int32(0), c_int32(0)
    lib.geohip_oracle_cell(ctypes.byref(g), x, y, ctypes.byref(cx), ctypes.byref(cy))
    return cx.value, cy.value


def layers(g: Grid, r):
    return lib.geohip_oracle_layers_guaranteed(ctypes.byref(g), r), lib.geohip_oracle_layers_candidate(ctypes.byref(g), r)


def range_pp(g: Grid, x, y, qx, qy, r, approximate=False) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.empty(max(len(x), 1), np.uint32)
    c = lib.geohip_oracle_range_pp(ctypes.byref(g), _p(x), _p(y), len(x), qx, qy, r, int(approximate), _p(out), len(out),
                                   None)
    if c < 0:
        raise OracleError(f"oracle range_pp error {c}")
    return out[:c].copy()


def range_pp_hash(g: Grid, x, y, qx, qy, r, approximate=False):
    """(hit count, sum of mix64(idx) mod 2^64) without materialising the hits."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    h = c_uint64(0)
    c = lib.geohip_oracle_range_pp(ctypes.byref(g), _p(x), _p(y), len(x), qx, qy, r, int(approximate), None, 0,
                                   ctypes.byref(h))
    if c < 0:
        raise OracleError(f"oracle range_pp error {c}")
    return c, h.value


def knn_pp(g: Grid, x, y, qx, qy, r, k):
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    oi = np.empty(k, np.uint32)
    od = np.empty(k, np.float64)
    cnt = c_uint32(0)
    rc = lib.geohip_oracle_knn_pp(ctypes.byref(g), _p(x), _p(y), len(x), qx, qy, r, k, _p(oi), _p(od),
                                  ctypes.byref(cnt))
    if rc != 0:
        raise OracleError(f"oracle knn_pp error {rc}")
    return oi[:cnt.value].copy(), od[:cnt.value].copy()


def join_pp(gd: Grid, gq: Grid, dx, dy, qx, qy, r, approximate=False, cap=None) -> np.ndarray:
    dx = np.ascontiguousarray(dx, np.float64)
    dy = np.ascontiguousarray(dy, np.float64)
    qx = np.ascontiguousarray(qx, np.float64)
    qy = np.ascontiguousarray(qy, np.float64)
    if cap is None:
        c = lib.geohip_oracle_join_pp(ctypes.byref(gd), ctypes.byref(gq), _p(dx), _p(dy), len(dx), _p(qx), _p(qy),
                                      len(qx), r, int(approximate), None, 0, None)
        if c < 0:
            raise OracleError(f"oracle join_pp error {c}")
        cap = c
    out = np.empty((max(cap, 1), 2), np.uint32)
    c = lib.geohip_oracle_join_pp(ctypes.byref(gd), ctypes.byref(gq), _p(dx), _p(dy), len(dx), _p(qx), _p(qy),
                                  len(qx), r, int(approximate), _p(out), cap, None)
    if c < 0:
        raise OracleError(f"oracle join_pp error {c}")
    return out[:c].copy()


def join_pp_hash(gd: Grid, gq: Grid, dx, dy, qx, qy, r, approximate=False):
    """(pair count, sum of mix64(p << 32 | q) mod 2^64) without materialising the pairs."""
    dx = np.ascontiguousarray(dx, np.float64)
    dy = np.ascontiguousarray(dy, np.float64)
    qx = np.ascontiguousarray(qx, np.float64)
    qy = np.ascontiguousarray(qy, np.float64)
    h = c_uint64(0)
    c = lib.geohip_oracle_join_pp(ctypes.byref(gd), ctypes.byref(gq), _p(dx), _p(dy), len(dx), _p(qx), _p(qy),
                                  len(qx), r, int(approximate), None, 0, ctypes.byref(h))
    if c < 0:
        raise OracleError(f"oracle join_pp error {c}")
    return c, h.value


def _rings(ring_off, vx, vy, poly_rings):
    ring_off = np.ascontiguousarray(ring_off, np.uint32)
    vx = np.ascontiguousarray(vx, np.float64)
    vy = np.ascontiguousarray(vy, np.float64)
    if poly_rings is None:
        return ring_off, vx, vy, None, len(ring_off) - 1
    pr = np.ascontiguousarray(poly_rings, np.uint32)
    return ring_off, vx, vy, pr, len(pr) - 1


def _ppoly(fn, grids, x, y, ring_off, vx, vy, r, approximate, poly_rings, want_hash):
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    ring_off, vx, vy, pr, npoly = _rings(ring_off, vx, vy, poly_rings)
    args = (*grids, _p(x), _p(y), len(x), None if pr is None else _p(pr), _p(ring_off), _p(vx), _p(vy), npoly, r,
            int(approximate))
    if want_hash:
        h = c_uint64(0)
        c = fn(*args, None, 0, ctypes.byref(h))
        if c < 0:
            raise OracleError(f"oracle polygon query error {c}")
        return c, h.value
    c = fn(*args, None, 0, None)
    if c < 0:
        raise OracleError(f"oracle polygon query error {c}")
    out = np.empty((max(c, 1), 2), np.uint32)
    assert fn(*args, _p(out), c, None) == c
    return out[:c].copy()


def range_ppoly(g: Grid, x, y, ring_off, vx, vy, r, approximate=False, poly_rings=None) -> np.ndarray:
    """PointPolygonRangeQuery window body: pairs (polygon, point).  Ring j = vertices
    [ring_off[j], ring_off[j+1]); polygon p = rings [poly_rings[p], poly_rings[p+1])
    (poly_rings None: one ring per polygon)."""
    return _ppoly(lib.geohip_oracle_range_ppoly, (ctypes.byref(g),), x, y, ring_off, vx, vy, r, approximate,
                  poly_rings, False)


def range_ppoly_hash(g: Grid, x, y, ring_off, vx, vy, r, approximate=False, poly_rings=None):
    """(pair count, sum of mix64(poly << 32 | point) mod 2^64)."""
    return _ppoly(lib.geohip_oracle_range_ppoly, (ctypes.byref(g),), x, y, ring_off, vx, vy, r, approximate,
                  poly_rings, True)


def join_ppoly(gp: Grid, gq: Grid, x, y, ring_off, vx, vy, r, approximate=False, poly_rings=None) -> np.ndarray:
    """PointPolygonJoinQuery window join: pairs (point, polygon), oracle order."""
    return _ppoly(lib.geohip_oracle_join_ppoly, (ctypes.byref(gp), ctypes.byref(gq)), x, y, ring_off, vx, vy, r,
                  approximate, poly_rings, False)


def join_ppoly_hash(gp: Grid, gq: Grid, x, y, ring_off, vx, vy, r, approximate=False, poly_rings=None):
    """(pair count, sum of mix64(point << 32 | poly) mod 2^64)."""
    return _ppoly(lib.geohip_oracle_join_ppoly, (ctypes.byref(gp), ctypes.byref(gq)), x, y, ring_off, vx, vy, r,
                  approximate, poly_rings, True)


def knn_ppoly(g: Grid, x, y, vx, vy, r, k, approximate=False, ring_off=None):
    """PointPolygonKNNQuery window body: (idx, dist) ascending by (dist bits, idx).  One query
    polygon: rings ring_off[0..] of vx/vy (None: vx/vy is one ring)."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    vx = np.ascontiguousarray(vx, np.float64)
    vy = np.ascontiguousarray(vy, np.float64)
    ro = np.array([0, len(vx)], np.uint32) if ring_off is None else np.ascontiguousarray(ring_off, np.uint32)
    oi = np.empty(k, np.uint32)
    od = np.empty(k, np.float64)
    cnt = c_uint32(0)
    rc = lib.geohip_oracle_knn_ppoly(ctypes.byref(g), _p(x), _p(y), len(x), _p(ro), len(ro) - 1, _p(vx), _p(vy), r, k,
                                     int(approximate), _p(oi), _p(od), ctypes.byref(cnt))
    if rc != 0:
        raise OracleError(f"oracle knn_ppoly error {rc}")
    return oi[:cnt.value].copy(), od[:cnt.value].copy()


def point_polygon(px, py, vx, vy, ring_off=None):
    """JTS point.distance(polygon): one closed ring, or the polygon built from rings ring_off."""
    vx = np.ascontiguousarray(vx, np.float64)
    vy = np.ascontiguousarray(vy, np.float64)
    if ring_off is None:
        return lib.geohip_oracle_point_polygon(px, py, _p(vx), _p(vy), len(vx))
    ro = np.ascontiguousarray(ring_off, np.uint32)
    st = c_int(0)
    d = lib.geohip_oracle_point_polygon_rings(px, py, _p(ro), len(ro) - 1, _p(vx), _p(vy), ctypes.byref(st))
    if st.value:
        raise OracleError(f"oracle polygon error {st.value}")
    return d


def set_threads(t: int) -> None:
    lib.geohip_oracle_set_threads(int(t))


def threads() -> int:
    return lib.geohip_oracle_threads()


MASK64 = (1 << 64) - 1


def mix64(z: int) -> int:
    return lib.geohip_oracle_mix64(z & MASK64)


# ---- ingest codec (oracle/ingest_oracle.c) -------------------------------------------------
CSV, GEOJSON, WKT = 0, 1, 2


class IngestRejected(OracleError):
    """The reference throws on record ``bad`` (NumberFormatException, IndexOutOfBounds, ...)."""

    def __init__(self, bad):
        super().__init__(f"record {bad} rejected by the reference grammar")
        self.bad = bad


def ingest_spec(fmt, delimiter=",", fx=0, fy=1, fts=-1, foid=-1) -> IngestSpec:
    return IngestSpec(fmt, delimiter.encode()[0] if delimiter else 0, fx, fy, fts, foid)


def traj_spec(prop_ts="timestamp", prop_oid="oID", date_format=1, utc_offset_min=0) -> TrajSpec:
    return TrajSpec(date_format, utc_offset_min, prop_ts.encode(), prop_oid.encode())


def ingest_traj(spec: IngestSpec, traj: TrajSpec | None, text: bytes, g: Grid | None = None):
    """TrajectoryStream batch -> dict(x, y, ts, cell, oid): oid = list of bytes / None per record
    (quotes deleted); IngestRejected(bad) for the first record thrown or not restated."""
    g = g if g is not None else grid(0.0, 0.0, 1.0, 1)
    cap = text.count(b"\n") + 1
    x, y = np.empty(cap), np.empty(cap)
    ts, cell = np.empty(cap, dtype=np.int64), np.empty(cap, dtype=np.uint32)
    off = np.empty(cap + 1, dtype=np.uint64)
    ob = np.empty(len(text) + 1, dtype=np.uint8)
    buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, dtype=np.uint8)
    n = lib.geohip_oracle_ingest_traj(ctypes.byref(spec), ctypes.byref(traj) if traj is not None else None,
                                      ctypes.byref(g), _p(buf), len(text), _p(x), _p(y), _p(ts), _p(cell), _p(ob),
                                      len(ob), _p(off), cap)
    if n < 0:
        raise IngestRejected(-n - 1)
    mask = (1 << 63) - 1
    oids = []
    for i in range(n):
        o = int(off[i])
        oids.append(None if o >> 63 else bytes(ob[o & mask:int(off[i + 1]) & mask]))
    return {"x": x[:n], "y": y[:n], "ts": ts[:n], "cell": cell[:n], "oid": oids,
            "oid_text": bytes(ob[:int(off[n]) & mask]), "oid_off": off[:n + 1]}


def ingest_record(spec: IngestSpec, rec: bytes, g: Grid | None = None):
    """One record -> (x, y, ts, cell) or None where the reference throws."""
    g = g if g is not None else grid(0.0, 0.0, 1.0, 1)
    x, y, ts, c = c_double(), c_double(), c_int64(), c_uint32()
    rc = lib.geohip_oracle_ingest_record(ctypes.byref(spec), ctypes.byref(g), rec, len(rec), ctypes.byref(x),
                                         ctypes.byref(y), ctypes.byref(ts), ctypes.byref(c))
    return None if rc else (x.value, y.value, ts.value, c.value)


def ingest(spec: IngestSpec, text: bytes, g: Grid | None = None):
    """A '\n'-separated batch -> dict(x, y, ts, cell) (numpy); IngestRejected(bad) where it throws."""
    g = g if g is not None else grid(0.0, 0.0, 1.0, 1)
    cap = text.count(b"\n") + 1
    x, y = np.empty(cap), np.empty(cap)
    ts, cell = np.empty(cap, dtype=np.int64), np.empty(cap, dtype=np.uint32)
    buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, dtype=np.uint8)
    n = lib.geohip_oracle_ingest(ctypes.byref(spec), ctypes.byref(g), _p(buf), len(text), _p(x), _p(y), _p(ts),
                                 _p(cell), cap)
    if n < 0:
        raise IngestRejected(-n - 1)
    return {"x": x[:n], "y": y[:n], "ts": ts[:n], "cell": cell[:n]}
