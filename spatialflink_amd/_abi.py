"""ctypes binding of libgeohip.so (include/geohip.h).

The product path: every query call goes to the gfx950 HIP library.  There is no CPU
fallback -- if the shared library is missing this module raises at import time, and if no
device is present ``Context()`` raises ``GeohipDeviceError``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_uint32, c_uint64, c_void_p
from pathlib import Path

import numpy as np

LIB_PATH = Path(os.environ.get("GEOHIP_LIB", Path(__file__).resolve().parent / "libgeohip.so"))

OK, ERR_ARG, ERR_CAPACITY, ERR_DEVICE, ERR_OOM, ERR_UNSUPPORTED = 0, 1, 2, 3, 4, 5
MEM_HOST, MEM_DEVICE = 0, 1
ORDER_ASCENDING, ORDER_ANY = 0, 1  # geohip_ctx_set_range_order
KNN_MAX_K = 1024
KNN_PPOLY_MAX_K = 256
SENTINEL_IDX = 0xFFFFFFFF


class GeohipError(RuntimeError):
    code = -1


class GeohipArgumentError(GeohipError, ValueError):
    """Where the reference calls System.exit(1) or throws (IllegalArgument/NumberFormat)."""
    code = ERR_ARG


class GeohipCapacityError(GeohipError):
    code = ERR_CAPACITY


class GeohipDeviceError(GeohipError):
    code = ERR_DEVICE


class GeohipOOMError(GeohipError, MemoryError):
    code = ERR_OOM


class GeohipUnsupportedError(GeohipError, NotImplementedError):
    code = ERR_UNSUPPORTED


_ERRORS = {ERR_ARG: GeohipArgumentError, ERR_CAPACITY: GeohipCapacityError, ERR_DEVICE: GeohipDeviceError,
           ERR_OOM: GeohipOOMError, ERR_UNSUPPORTED: GeohipUnsupportedError}


class Grid(ctypes.Structure):
    _fields_ = [("min_x", c_double), ("min_y", c_double), ("cell_len", c_double), ("n", c_int32),
                ("reserved", c_int32)]


FMT_CSV, FMT_GEOJSON, FMT_WKT = 0, 1, 2


class IngestSpec(ctypes.Structure):
    """geohip_ingest_spec: format, delimiter byte, csvTsvSchemaAttr x/y/ts/objID indices."""
    _fields_ = [("format", c_int32), ("delim", c_int32), ("attr_x", c_int32), ("attr_y", c_int32),
                ("attr_ts", c_int32), ("attr_oid", c_int32)]


def make_ingest_spec(fmt: int, delimiter: str = ",", attr_x: int = 0, attr_y: int = 1, attr_ts: int = -1,
                     attr_oid: int = 0) -> IngestSpec:
    d = delimiter.encode() if delimiter else b"\0"
    if len(d) != 1:
        raise GeohipUnsupportedError("delimiter must be one byte")
    return IngestSpec(fmt, d[0], attr_x, attr_y, attr_ts, attr_oid)


class TrajSpec(ctypes.Structure):
    """geohip_traj_spec: the TrajectoryStream's DateFormat and GeoJSON property names."""
    _fields_ = [("date_format", c_int32), ("utc_offset_min", c_int32), ("prop_ts", ctypes.c_char * 60),
                ("prop_oid", ctypes.c_char * 60)]


def make_traj_spec(prop_ts: str = "timestamp", prop_oid: str = "oID", date_format: int = 1,
                   utc_offset_min: int = 0) -> TrajSpec:
    """Defaults: conf/geoflink-conf.yml's propertyTimeStamp / propertyObjID and
    "yyyy-MM-dd HH:mm:ss" (GEOHIP_DATE_YMD_HMS) in UTC."""
    a, b = prop_ts.encode(), prop_oid.encode()
    if len(a) > 59 or len(b) > 59:
        raise GeohipArgumentError("property names of at most 59 bytes")
    return TrajSpec(date_format, utc_offset_min, a, b)


OID_NULL = (1 << 24) - 1  # the length field of a null objID span


def oid_spans_to_strings(text: bytes, spans) -> list:
    """Host view of objID spans (tests, small batches): the str / None per record, quotes deleted."""
    out = []
    for v in (int(s) for s in spans):
        off, ln = v >> 24, v & OID_NULL
        out.append(None if ln == OID_NULL else text[off:off + ln].replace(b'"', b"").decode("utf-8", "replace"))
    return out


class CsvOutSpec(ctypes.Structure):
    """geohip_csv_out_spec: csvTsvSchemaAttr positions of objID, ts, x, y and the delimiter."""
    _fields_ = [("attr_oid", c_int32), ("attr_ts", c_int32), ("attr_x", c_int32), ("attr_y", c_int32),
                ("delim_len", c_int32), ("delim", ctypes.c_char * 8), ("reserved", c_int32)]


def _separation(delimiter: str) -> bytes:
    """The schemas' SEPARATION: the config string `\\\\t` (backslash, backslash, t) becomes the two
    characters `\\t` (Serialization.java:62-66, 110-114); UTF-8, 1..8 bytes."""
    if delimiter == "\\\\t":
        delimiter = "\\t"
    d = delimiter.encode()
    if not 1 <= len(d) <= 8:
        raise GeohipUnsupportedError("delimiter must be 1..8 bytes")
    return d


def make_csv_out_spec(attrs=(0, 1, 2, 3), delimiter: str = ",") -> CsvOutSpec:
    d = _separation(delimiter)
    return CsvOutSpec(attrs[0], attrs[1], attrs[2], attrs[3], len(d), d, 0)


DATE_NONE, DATE_YMD_HMS = 0, 1


class TextOutSpec(ctypes.Structure):
    """geohip_text_out_spec: output schema (FMT_CSV / FMT_WKT / FMT_GEOJSON), CSV positions,
    delimiter, date formatter and its zone offset."""
    _fields_ = [("format", c_int32), ("attr_oid", c_int32), ("attr_ts", c_int32), ("attr_x", c_int32),
                ("attr_y", c_int32), ("delim_len", c_int32), ("delim", ctypes.c_char * 8), ("date_format", c_int32),
                ("utc_offset_min", c_int32)]


def make_text_out_spec(fmt: int, attrs=(0, 1, 2, 3), delimiter: str = ",", date_format: int = DATE_NONE,
                       utc_offset_min: int = 0) -> TextOutSpec:
    """Serialization.PointToCSVTSVOutputSchema / PointToWKTOutputSchema / PointToGeoJSONOutputSchema
    (Serialization.java:17-152); date_format DATE_YMD_HMS = SimpleDateFormat("yyyy-MM-dd HH:mm:ss")
    in a fixed-offset zone."""
    d = _separation(delimiter) if fmt != FMT_GEOJSON else b","
    return TextOutSpec(fmt, attrs[0], attrs[1], attrs[2], attrs[3], len(d), d, date_format, utc_offset_min)


class Rect(ctypes.Structure):
    _fields_ = [("x0", c_int32), ("x1", c_int32), ("y0", c_int32), ("y1", c_int32)]


# One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 (SONAME
# libamdhip64.so.7, loaded under the file name libamdhip64.so).  Loading torch first lets
# libgeohip's NEEDED libamdhip64.so.7 bind to that same instance; loading libgeohip first
# would bring /opt/rocm's copy and leave torch with a second runtime that sees no GPU.
try:  # pragma: no cover - torch is optional for the C-ABI user
    import torch  # noqa: F401
except Exception:  # noqa: BLE001
    torch = None

if not LIB_PATH.exists():
    raise ImportError(f"{LIB_PATH} not built: run `python -m spatialflink_amd.build` (hipcc, gfx950)")

lib = ctypes.CDLL(str(LIB_PATH))

_P = c_void_p
_SIGS = {
    "geohip_version": (c_char_p, []),
    "geohip_abi_version": (c_int, []),
    "geohip_device_count": (c_int, [POINTER(c_int)]),
    "geohip_ctx_create": (c_int, [c_uint32, POINTER(c_void_p)]),
    "geohip_ctx_destroy": (c_int, [_P]),
    "geohip_last_error": (c_char_p, [_P]),
    "geohip_ctx_set_mem": (c_int, [_P, c_int]),
    "geohip_ctx_set_stream": (c_int, [_P, _P]),
    "geohip_ctx_reset_stream": (c_int, [_P]),
    "geohip_ctx_stream": (c_void_p, [_P]),
    "geohip_ctx_set_timing": (c_int, [_P, c_int]),
    "geohip_ctx_set_range_order": (c_int, [_P, c_int]),
    "geohip_ctx_sync": (c_int, [_P]),
    "geohip_debug_lookback_inject": (c_int, [_P, c_int]),
    "geohip_ctx_timing": (c_int, [_P, POINTER(c_double), POINTER(c_uint64), c_int]),
    "geohip_ctx_timing_kernels": (c_int, [_P, POINTER(c_double), POINTER(c_uint64), POINTER(c_double),
                                          POINTER(c_uint64), c_int]),
    "geohip_range_pp": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_double, c_double, c_double, c_int, _P,
                                c_uint64, POINTER(c_uint64)]),
    "geohip_range_pp_pane": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_uint32, c_double, c_double, c_double, c_int,
                                     _P, c_uint64, POINTER(c_uint64)]),
    "geohip_range_pp_async": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_double, c_double, c_double, c_int,
                                      _P, c_uint64, _P]),
    "geohip_knn_pp": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_double, c_double, c_double, c_uint32, _P, _P,
                              POINTER(c_uint32)]),
    "geohip_knn_pp_async": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_double, c_double, c_double, c_uint32,
                                    _P, _P, _P]),
    "geohip_knn_merge_async": (c_int, [_P, _P, _P, c_uint32, c_uint32, c_uint32, _P, _P, _P]),
    "geohip_knn_merge_panes_async": (c_int, [_P, _P, _P, c_uint32, _P, _P, c_uint32, c_uint32, _P, _P, _P]),
    "geohip_format_points_csv": (c_int, [_P, POINTER(CsvOutSpec), _P, _P, c_uint64, _P, _P, _P, _P, c_uint64, _P,
                                         c_uint64, POINTER(c_uint64), _P]),
    "geohip_format_points": (c_int, [_P, POINTER(TextOutSpec), _P, _P, c_uint64, _P, _P, _P, _P, c_uint64, _P, c_uint64,
                                     POINTER(c_uint64), _P]),
    "geohip_band_pack_async": (c_int, [_P, POINTER(Grid), c_int32, c_uint32, _P, _P, c_uint64, ctypes.c_int64, _P, _P,
                                       _P, _P]),
    "geohip_band_pack_query_async": (c_int, [_P, POINTER(Grid), c_int32, c_uint32, c_double, c_double, c_double, _P, _P,
                                             c_uint64, ctypes.c_int64, _P, _P, _P, _P]),
    "geohip_knn_range_pp": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_double, c_double, c_double, c_uint32,
                                    c_int, _P, _P, POINTER(c_uint32), _P, c_uint64, POINTER(c_uint64)]),
    "geohip_knn_range_pp_async": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_double, c_double, c_double,
                                          c_uint32, c_int, _P, _P, _P, _P, c_uint64, _P]),
    "geohip_join_pp": (c_int, [_P, POINTER(Grid), POINTER(Grid), _P, _P, c_uint64, _P, _P, c_uint64, c_double,
                               c_int, _P, c_uint64, POINTER(c_uint64)]),
    "geohip_join_pp_count_only": (c_int, [_P, POINTER(Grid), POINTER(Grid), _P, _P, c_uint64, _P, _P, c_uint64,
                                          c_double, c_int, POINTER(c_uint64)]),
    "geohip_join_pp_async": (c_int, [_P, POINTER(Grid), POINTER(Grid), _P, _P, c_uint64, _P, _P, c_uint64, c_double,
                                     c_int, _P, c_uint64, _P]),
    "geohip_range_ppoly_async": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, _P, _P, _P, _P, c_uint64, c_uint32,
                                         c_double, c_int, _P, c_uint64, _P]),
    "geohip_range_ppoly_pane_async": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_uint32, _P, _P, _P, _P, c_uint64,
                                              c_uint32, c_double, c_int, _P, c_uint64, _P]),
    "geohip_join_ppoly_async": (c_int, [_P, POINTER(Grid), POINTER(Grid), _P, _P, c_uint64, _P, _P, _P, _P, c_uint64,
                                        c_uint32, c_double, c_int, _P, c_uint64, _P]),
    "geohip_range_ppoly": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, _P, _P, _P, _P, c_uint64, c_uint32, c_double, c_int,
                                   _P, c_uint64, POINTER(c_uint64)]),
    "geohip_range_ppoly_pane": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_uint32, _P, _P, _P, _P, c_uint64, c_uint32,
                                        c_double, c_int, _P, c_uint64, POINTER(c_uint64)]),
    "geohip_join_ppoly": (c_int, [_P, POINTER(Grid), POINTER(Grid), _P, _P, c_uint64, _P, _P, _P, _P, c_uint64, c_uint32,
                                  c_double, c_int, _P, c_uint64, POINTER(c_uint64)]),
    "geohip_knn_ppoly": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, _P, c_uint32, _P, _P, c_uint64, c_double, c_uint32, c_int,
                                 _P, _P, POINTER(c_uint32)]),
    "geohip_knn_ppoly_async": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, _P, c_uint32, _P, _P, c_uint64, c_double, c_uint32,
                                       c_int, _P, _P, _P]),
    "geohip_plan_point": (c_int, [POINTER(Grid), c_double, c_double, c_double, POINTER(Rect), POINTER(c_uint32),
                                  POINTER(Rect), POINTER(c_uint32), POINTER(c_int32), POINTER(c_int32)]),
    "geohip_plan_cell": (c_int, [POINTER(Grid), c_double, c_double, POINTER(c_int32), POINTER(c_int32)]),
    "geohip_synth_uniform_async": (c_int, [_P, _P, _P, c_uint64, c_uint64, c_uint64, c_double, c_double, c_double,
                                           c_double]),
    "geohip_ingest_points": (c_int, [_P, POINTER(Grid), POINTER(IngestSpec), _P, c_uint64, _P, _P, _P, _P, c_uint64,
                                     POINTER(c_uint64), POINTER(c_uint64)]),
    "geohip_debug_ingest_record": (c_int, [POINTER(IngestSpec), c_char_p, c_uint64, POINTER(c_double),
                                           POINTER(c_double), POINTER(ctypes.c_int64)]),
    "geohip_debug_ingest_traj_record": (c_int, [POINTER(IngestSpec), POINTER(TrajSpec), c_char_p, c_uint64,
                                                POINTER(c_double), POINTER(c_double), POINTER(ctypes.c_int64),
                                                POINTER(c_uint64)]),
    "geohip_ingest_trajectory": (c_int, [_P, POINTER(Grid), POINTER(IngestSpec), POINTER(TrajSpec), _P, c_uint64, _P,
                                         _P, _P, _P, _P, c_uint64, POINTER(c_uint64), POINTER(c_uint64)]),
    "geohip_ingest_oid_compact": (c_int, [_P, _P, c_uint64, _P, c_uint64, _P, c_uint64, _P, POINTER(c_uint64)]),
    "geohip_debug_selftest_fp64": (c_int, [_P, _P, _P, c_uint64, _P, _P, _P, _P]),
    "geohip_debug_classify": (c_int, [POINTER(Grid), c_double, c_double, c_double, _P, _P, c_uint64, _P]),
    "geohip_debug_knn_pass_stats": (c_int, [_P, _P]),
    "geohip_debug_knn_pass_trace": (c_int, [_P, POINTER(Grid), _P, _P, c_uint64, c_double, c_double, c_double,
                                            c_uint32, c_int, _P, c_uint64, POINTER(c_uint32)]),
}
for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

# symbols of include/geohip.h (tests check the library exports every one)
HEADER_SYMBOLS = [n for n in _SIGS if not n.startswith("geohip_debug_")]


def version() -> str:
    return lib.geohip_version().decode()


def device_count() -> int:
    c = c_int(0)
    lib.geohip_device_count(ctypes.byref(c))
    return c.value


def make_grid(min_x: float, min_y: float, cell_len: float, n: int) -> Grid:
    return Grid(float(min_x), float(min_y), float(cell_len), int(n), 0)


def plan_point(grid: Grid, qx: float, qy: float, r: float):
    """Planner introspection (host only): (g_rects, c_rects, Lg, Lc) as lists of (x0,x1,y0,y1)."""
    g = (Rect * 16)()
    c = Rect()
    ng, nc = c_uint32(0), c_uint32(0)
    lg, lc = c_int32(0), c_int32(0)
    rc = lib.geohip_plan_point(ctypes.byref(grid), qx, qy, r, g, ctypes.byref(ng), ctypes.byref(c),
                               ctypes.byref(nc), ctypes.byref(lg), ctypes.byref(lc))
    if rc:
        raise _ERRORS.get(rc, GeohipError)(f"plan_point failed ({rc})")
    gl = [(g[i].x0, g[i].x1, g[i].y0, g[i].y1) for i in range(ng.value)]
    cl = [(c.x0, c.x1, c.y0, c.y1)] if nc.value else []
    return gl, cl, lg.value, lc.value


def debug_classify(grid: Grid, qx: float, qy: float, r: float, x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """Host evaluation of the planner's boxes (test hook): bit0 inG, bit1 inC, bit2 in G u C."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.empty(len(x), np.uint8)
    rc = lib.geohip_debug_classify(ctypes.byref(grid), qx, qy, r, x.ctypes.data_as(c_void_p),
                                   y.ctypes.data_as(c_void_p), len(x), out.ctypes.data_as(c_void_p))
    if rc:
        raise _ERRORS.get(rc, GeohipError)(f"debug_classify failed ({rc})")
    return out


def plan_cell(grid: Grid, x: float, y: float):
    cx, cy = c_int32(0), c_int32(0)
    lib.geohip_plan_cell(ctypes.byref(grid), x, y, ctypes.byref(cx), ctypes.byref(cy))
    return cx.value, cy.value


def debug_ingest_record(spec: IngestSpec, rec: bytes):
    """The device record parser (ingest_parse.h) run on the host: (x, y, ts) or None if rejected."""
    x, y, ts = c_double(), c_double(), ctypes.c_int64()
    rc = lib.geohip_debug_ingest_record(ctypes.byref(spec), rec, len(rec), ctypes.byref(x), ctypes.byref(y),
                                        ctypes.byref(ts))
    if rc == ERR_ARG:
        raise GeohipArgumentError("bad ingest spec")
    return None if rc else (x.value, y.value, ts.value)


def debug_ingest_traj_record(spec: IngestSpec, traj: TrajSpec | None, rec: bytes):
    """The device trajectory parse on the host: (x, y, ts, oid span relative to rec) or None if
    rejected."""
    x, y, ts, oid = c_double(), c_double(), ctypes.c_int64(), c_uint64()
    rc = lib.geohip_debug_ingest_traj_record(ctypes.byref(spec), ctypes.byref(traj) if traj is not None else None, rec,
                                             len(rec), ctypes.byref(x), ctypes.byref(y), ctypes.byref(ts),
                                             ctypes.byref(oid))
    if rc == ERR_ARG:
        raise GeohipArgumentError("bad ingest spec")
    return None if rc else (x.value, y.value, ts.value, oid.value)


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(c_void_p)
    return c_void_p(a.data_ptr())  # torch tensor on the ctx device (checked by Context._dev)


def _is_device(a) -> bool:
    return not isinstance(a, np.ndarray) and getattr(a, "is_cuda", False)


def _f64(a):
    if isinstance(a, np.ndarray):
        return np.ascontiguousarray(a, dtype=np.float64)
    return a


def _host(a, dtype):
    """Host array of dtype (polygon rings and other planning inputs are host memory)."""
    if a is not None and not isinstance(a, np.ndarray) and hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(a, dtype=dtype)


def _poly_arrays(poly_rings, ring_off, vx, vy):
    """(poly_rings or None, ring_off, vx, vy, npoly) as host arrays for the point-polygon calls."""
    ring_off = _host(ring_off, np.uint32)
    pr = None if poly_rings is None else _host(poly_rings, np.uint32)
    npoly = (len(ring_off) if pr is None else len(pr)) - 1
    if npoly < 0:
        raise GeohipArgumentError("ring_off / poly_rings need at least one entry")
    vx, vy = _host(vx, np.float64), _host(vy, np.float64)
    _check_rings(ring_off, vx, vy)
    if pr is not None and npoly and (int(pr[-1]) >= len(ring_off) or int(pr.max()) >= len(ring_off)):
        raise GeohipArgumentError("poly_rings refers past the end of ring_off")
    return pr, ring_off, vx, vy, npoly


def _check_rings(ring_off, vx, vy):
    """Python-side argument check (the C side checks ring offsets against the vertex count too)."""
    if len(vx) != len(vy):
        raise GeohipArgumentError(f"vx and vy differ in length ({len(vx)} vs {len(vy)})")
    if len(ring_off) and int(ring_off.max()) > len(vx):
        raise GeohipArgumentError(f"ring_off refers past the end of vx/vy ({int(ring_off.max())} > {len(vx)})")


class Context:
    """One geohip_ctx (one device, one stream).  Not shared between threads."""

    def __init__(self, device: int = 0):
        h = c_void_p()
        rc = lib.geohip_ctx_create(1 << device, ctypes.byref(h))
        if rc:
            raise _ERRORS.get(rc, GeohipError)(f"geohip_ctx_create(device={device}) failed ({rc}); "
                                               "libgeohip needs an MI355X (gfx950) device")
        self.h = h
        self.device = device
        self._mem = MEM_HOST
        self._follow = True   # device calls enqueue on torch's current stream of the inputs' device
        self._bound = None    # stream handle the C ctx enqueues on (None: its own stream)

    def close(self):
        if self.h:
            lib.geohip_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc:
            msg = lib.geohip_last_error(self.h).decode(errors="replace")
            raise _ERRORS.get(rc, GeohipError)(f"{what}: {msg}")

    def set_mem(self, kind: int):
        if kind != self._mem:
            self._check(lib.geohip_ctx_set_mem(self.h, kind), "set_mem")
            self._mem = kind

    def set_stream(self, stream_ptr: int | None):
        """Enqueue on this hipStream_t (0 = the null stream, PyTorch's default); None = the ctx's
        own stream.  Stops following torch's current stream (follow_torch_stream)."""
        self._follow = False
        self._bind(stream_ptr)

    def _bind(self, stream_ptr):
        if stream_ptr is None:
            self._check(lib.geohip_ctx_reset_stream(self.h), "reset_stream")
        else:
            self._check(lib.geohip_ctx_set_stream(self.h, c_void_p(stream_ptr) if stream_ptr else None), "set_stream")
        self._bound = stream_ptr

    def follow_torch_stream(self, on: bool = True):
        """Default: calls on device tensors run on torch.cuda.current_stream() of their device, so
        torch kernels that produced the inputs finish first and torch work queued after an
        *_async call sees its results."""
        self._follow = bool(on)

    def stream(self) -> int:
        return lib.geohip_ctx_stream(self.h) or 0

    @contextlib.contextmanager
    def using_stream(self, stream_ptr):
        """Bind a stream for a block, then restore the previous binding and follow mode."""
        prev, follow = self._bound, self._follow
        self._follow = False
        self._bind(stream_ptr)
        try:
            yield self
        finally:
            self._bind(prev)
            self._follow = follow

    def _dev(self, t, what="array", dtype="float64"):
        """Validate a device tensor argument (dtype, contiguity, ctx device) and, in follow mode,
        bind torch's current stream of its device."""
        import torch
        if t.dtype != getattr(torch, dtype):
            raise GeohipArgumentError(f"{what}: expected a {dtype} tensor, got {t.dtype}")
        if not t.is_contiguous():
            raise GeohipArgumentError(f"{what}: tensor must be contiguous")
        if t.device.index != self.device:
            raise GeohipArgumentError(f"{what}: tensor on {t.device}, ctx on cuda:{self.device}")
        if self._follow:
            s = torch.cuda.current_stream(t.device).cuda_stream
            if s != self._bound:
                self._bind(s)

    def sync(self):
        """Wait for this ctx's queued work; raises GeohipDeviceError if a kernel gave up a look-back
        wait since the last check (geohip_ctx_sync)."""
        self._check(lib.geohip_ctx_sync(self.h), "sync")

    def debug_lookback_inject(self, on: bool):
        """Test knob: range look-back waits give up (the fault path)."""
        self._check(lib.geohip_debug_lookback_inject(self.h, int(on)), "debug_lookback_inject")

    def set_range_order(self, unordered: bool):
        """geohip_ctx_set_range_order: False = ascending hit indices (the default), True = the
        same set in any order (one pass, no ordered emission; the reference's window result is
        a set)."""
        self._check(lib.geohip_ctx_set_range_order(self.h, ORDER_ANY if unordered else ORDER_ASCENDING),
                    "set_range_order")

    def set_timing(self, on: bool):
        self._check(lib.geohip_ctx_set_timing(self.h, int(on)), "set_timing")

    def timing(self, reset: bool = True):
        ms, n = c_double(0), c_uint64(0)
        self._check(lib.geohip_ctx_timing(self.h, ctypes.byref(ms), ctypes.byref(n), int(reset)), "timing")
        return ms.value, n.value

    def timing_kernels(self, reset: bool = True):
        """(step_ms, steps, kernel_ms, kernels) since the last reset: step_ms sums the timed steps
        (a multi-launch step from its first launch to its last, gaps included), kernel_ms the
        kernels of those steps as their own dispatches stamp them (what rocprofv3 reports)."""
        sm, sn, km, kn = c_double(0), c_uint64(0), c_double(0), c_uint64(0)
        self._check(lib.geohip_ctx_timing_kernels(self.h, ctypes.byref(sm), ctypes.byref(sn), ctypes.byref(km),
                                                  ctypes.byref(kn), int(reset)), "timing_kernels")
        return sm.value, sn.value, km.value, kn.value

    def _mem_for(self, *arrays, dtype="float64"):
        dev = [_is_device(a) for a in arrays if a is not None]
        if any(dev) and not all(dev):
            raise GeohipArgumentError("mix of host and device arrays")
        on_dev = bool(dev and dev[0])
        if on_dev:
            for a in arrays:
                if a is not None:
                    self._dev(a, dtype=dtype)
        self.set_mem(MEM_DEVICE if on_dev else MEM_HOST)
        return on_dev

    # ---- queries -------------------------------------------------------------------------
    def range_pp(self, grid: Grid, x, y, qx, qy, r, approximate=False, cap=None, point_base=None):
        """Hit indices, ascending.  ``point_base`` (geohip_range_pp_pane): indices are point_base +
        position (mod 2^32), a pane's stream positions."""
        x, y = _f64(x), _f64(y)
        n = len(x)
        dev = self._mem_for(x, y)
        if dev:
            import torch
            cap = n if cap is None else cap
            out = torch.empty(max(cap, 1), dtype=torch.int32, device=x.device)
        else:
            cap = n if cap is None else cap
            out = np.empty(max(cap, 1), dtype=np.uint32)
        cnt = c_uint64(0)
        if point_base is None:
            rc = lib.geohip_range_pp(self.h, ctypes.byref(grid), _ptr(x), _ptr(y), n, qx, qy, r, int(approximate),
                                     _ptr(out), cap, ctypes.byref(cnt))
        else:
            rc = lib.geohip_range_pp_pane(self.h, ctypes.byref(grid), _ptr(x), _ptr(y), n, int(point_base) & 0xFFFFFFFF,
                                          qx, qy, r, int(approximate), _ptr(out), cap, ctypes.byref(cnt))
        self._check(rc, "range_pp")
        return out[:cnt.value]

    def knn_pp(self, grid: Grid, x, y, qx, qy, r, k):
        x, y = _f64(x), _f64(y)
        n = len(x)
        dev = self._mem_for(x, y)
        if dev:
            import torch
            oi = torch.empty(k, dtype=torch.int32, device=x.device)
            od = torch.empty(k, dtype=torch.float64, device=x.device)
        else:
            oi = np.empty(k, dtype=np.uint32)
            od = np.empty(k, dtype=np.float64)
        cnt = c_uint32(0)
        rc = lib.geohip_knn_pp(self.h, ctypes.byref(grid), _ptr(x), _ptr(y), n, qx, qy, r, k, _ptr(oi), _ptr(od),
                               ctypes.byref(cnt))
        self._check(rc, "knn_pp")
        return oi[:cnt.value], od[:cnt.value]

    def knn_range_pp(self, grid: Grid, x, y, qx, qy, r, k, approximate=False, cap=None):
        """kNN (k) and range (r) of one query point over one window in one pass:
        ((knn_idx, knn_dist), range_idx) -- the results of knn_pp and range_pp."""
        x, y = _f64(x), _f64(y)
        n = len(x)
        dev = self._mem_for(x, y)
        cap = n if cap is None else cap
        if dev:
            import torch
            oi = torch.empty(k, dtype=torch.int32, device=x.device)
            od = torch.empty(k, dtype=torch.float64, device=x.device)
            ro = torch.empty(max(cap, 1), dtype=torch.int32, device=x.device)
        else:
            oi = np.empty(k, dtype=np.uint32)
            od = np.empty(k, dtype=np.float64)
            ro = np.empty(max(cap, 1), dtype=np.uint32)
        kc, rc_ = c_uint32(0), c_uint64(0)
        rc = lib.geohip_knn_range_pp(self.h, ctypes.byref(grid), _ptr(x), _ptr(y), n, qx, qy, r, k, int(approximate),
                                     _ptr(oi), _ptr(od), ctypes.byref(kc), _ptr(ro), cap, ctypes.byref(rc_))
        self._check(rc, "knn_range_pp")
        return (oi[:kc.value], od[:kc.value]), ro[:rc_.value]

    def knn_range_pp_async(self, grid: Grid, x, y, qx, qy, r, k, approximate, knn_idx, knn_dist, knn_count,
                           range_idx, cap, range_count):
        self._dev(x, "x")
        self._dev(y, "y")
        self._dev(knn_idx, "knn_idx", "int32")
        self._dev(knn_dist, "knn_dist")
        self._dev(knn_count, "knn_count", "int32")
        self._dev(range_idx, "range_idx", "int32")
        self._dev(range_count, "range_count", "int64")
        if range_idx.numel() < cap:
            raise GeohipArgumentError("knn_range_pp_async: range_idx shorter than cap")
        if knn_idx.numel() < k or knn_dist.numel() < k:
            raise GeohipArgumentError("knn_range_pp_async: knn_idx / knn_dist shorter than k")
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_knn_range_pp_async(self.h, ctypes.byref(grid), x.data_ptr(), y.data_ptr(), x.numel(), qx, qy, r,
                                           k, int(approximate), knn_idx.data_ptr(), knn_dist.data_ptr(),
                                           knn_count.data_ptr(), range_idx.data_ptr(), cap, range_count.data_ptr())
        if rc:
            self._check(rc, "knn_range_pp_async")

    # async forms: device tensors only, no host sync; the hot per-window path, so the pointers
    # go to ctypes as plain ints (argtypes c_void_p) without wrapper objects
    def knn_pp_async(self, grid: Grid, x, y, qx, qy, r, k, out_idx, out_dist, out_count):
        self._dev(x, "x")
        self._dev(y, "y")
        self._dev(out_idx, "out_idx", "int32")
        self._dev(out_dist, "out_dist")
        self._dev(out_count, "out_count", "int32")
        if out_idx.numel() < k or out_dist.numel() < k:
            raise GeohipArgumentError("knn_pp_async: out_idx / out_dist shorter than k")
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_knn_pp_async(self.h, ctypes.byref(grid), x.data_ptr(), y.data_ptr(), x.numel(), qx, qy, r, k,
                                     out_idx.data_ptr(), out_dist.data_ptr(), out_count.data_ptr())
        if rc:
            self._check(rc, "knn_pp_async")

    def knn_merge_async(self, dist, idx, nlists, list_len, k, out_idx, out_dist, out_count):
        self._dev(dist, "dist")
        self._dev(idx, "idx", "int32")
        if dist.numel() < nlists * list_len or idx.numel() < nlists * list_len:
            raise GeohipArgumentError("knn_merge_async: lists shorter than nlists * list_len")
        self._dev(out_idx, "out_idx", "int32")
        self._dev(out_dist, "out_dist")
        self._dev(out_count, "out_count", "int32")
        if out_idx.numel() < k or out_dist.numel() < k:
            raise GeohipArgumentError("knn_merge_async: out_idx / out_dist shorter than k")
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_knn_merge_async(self.h, dist.data_ptr(), idx.data_ptr(), nlists, list_len, k,
                                        out_idx.data_ptr(), out_dist.data_ptr(), out_count.data_ptr())
        if rc:
            self._check(rc, "knn_merge_async")

    def knn_merge_panes_async(self, ring_d, ring_i, slots, offsets, k, out_idx, out_dist, out_count):
        """geohip_knn_merge_panes_async: the window's k smallest from the panes' top-k lists in a
        ring (ring_d / ring_i: [slots, list_len] device tensors), pane b = ring slot slots[b]
        (oldest first) rebased by offsets[b].  One launch, no host sync."""
        self._dev(ring_d, "ring_d")
        self._dev(ring_i, "ring_i", "int32")
        self._dev(out_idx, "out_idx", "int32")
        self._dev(out_dist, "out_dist")
        self._dev(out_count, "out_count", "int32")
        if ring_d.dim() != 2 or ring_d.shape != ring_i.shape:
            raise GeohipArgumentError("knn_merge_panes_async: ring_d / ring_i must be [slots, list_len]")
        if out_idx.numel() < k or out_dist.numel() < k:
            raise GeohipArgumentError("knn_merge_panes_async: outputs shorter than k")
        nslot, L = int(ring_d.shape[0]), int(ring_d.shape[1])
        sl = (ctypes.c_uint32 * len(slots))(*[int(v) for v in slots])
        of = (ctypes.c_uint64 * len(offsets))(*[int(v) for v in offsets])
        if len(slots) != len(offsets) or any(not 0 <= int(v) < nslot for v in slots):
            raise GeohipArgumentError("knn_merge_panes_async: bad slot list")
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_knn_merge_panes_async(self.h, ring_d.data_ptr(), ring_i.data_ptr(), L, sl, of, len(slots), k,
                                              out_idx.data_ptr(), out_dist.data_ptr(), out_count.data_ptr())
        if rc:
            self._check(rc, "knn_merge_panes_async")

    def format_points_csv(self, spec: CsvOutSpec, x, y, ts=None, oid_text=None, oid_off=None, idx=None, cap=None):
        """geohip_format_points_csv (Serialization.PointToCSVTSVOutputSchema over result points):
        device tensors in (x, y float64; ts int64; oid_text uint8 + oid_off int64 [n + 1]; idx
        int32 record -> point), -> (text uint8 device tensor, record offsets int64 [m + 1])."""
        return self._format(lib.geohip_format_points_csv, spec, x, y, ts, oid_text, oid_off, idx, cap)

    def format_points(self, spec: TextOutSpec, x, y, ts=None, oid_text=None, oid_off=None, idx=None, cap=None):
        """geohip_format_points: the CSV/TSV, WKT or GeoJSON point schema (spec.format), arguments
        as for format_points_csv."""
        return self._format(lib.geohip_format_points, spec, x, y, ts, oid_text, oid_off, idx, cap)

    def _format(self, fn, spec, x, y, ts, oid_text, oid_off, idx, cap):
        import torch
        self._dev(x, "x")
        self._dev(y, "y")
        if y.numel() != x.numel():
            raise GeohipArgumentError("format: x and y differ in length")
        if ts is not None:
            self._dev(ts, "ts", "int64")
            if ts.numel() < x.numel():
                raise GeohipArgumentError("format: ts shorter than x")
        if (oid_text is None) != (oid_off is None):
            raise GeohipArgumentError("oid_text and oid_off go together")
        if oid_text is not None:
            self._dev(oid_text, "oid_text", "uint8")
            self._dev(oid_off, "oid_off", "int64")
            if oid_off.numel() < x.numel() + 1:
                raise GeohipArgumentError("format: oid_off needs n + 1 entries")
        if idx is not None:
            self._dev(idx, "idx", "int32")
        n = x.numel()
        m = idx.numel() if idx is not None else n
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        off = torch.empty(m + 1, dtype=torch.int64, device=x.device)
        ln = c_uint64(0)
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        if cap is None:  # size pass
            rc = fn(self.h, ctypes.byref(spec), x.data_ptr(), y.data_ptr(), n, ptr(ts), ptr(oid_text), ptr(oid_off),
                    ptr(idx), m, None, 0, ctypes.byref(ln), off.data_ptr())
            if rc not in (OK, ERR_CAPACITY):
                self._check(rc, "format_points")
            cap = ln.value
        out = torch.empty(max(cap, 1), dtype=torch.uint8, device=x.device)
        rc = fn(self.h, ctypes.byref(spec), x.data_ptr(), y.data_ptr(), n, ptr(ts), ptr(oid_text), ptr(oid_off),
                ptr(idx), m, out.data_ptr(), cap, ctypes.byref(ln), off.data_ptr())
        self._check(rc, "format_points")
        return out[:ln.value], off

    def band_pack_async(self, grid_data: Grid, nb: int, world: int, x, y, base: int = 0):
        """geohip_band_pack_async: this shard's valid-key points grouped by key-band owner rank
        (column cx -> rank cx * world // nb), arrival order inside a group.  Returns device
        tensors (x, y, idx int64 = base + position) of length len(x) (the first counts.sum()
        entries are filled) and counts (uint64 as int64, [world])."""
        import torch
        self._dev(x, "x")
        self._dev(y, "y")
        n = x.numel()
        if y.numel() != n:
            raise GeohipArgumentError("band_pack_async: x and y differ in length")
        ox = torch.empty(max(n, 1), dtype=torch.float64, device=x.device)
        oy = torch.empty_like(ox)
        oi = torch.empty(max(n, 1), dtype=torch.int64, device=x.device)
        cnt = torch.empty(max(world, 1), dtype=torch.int64, device=x.device)
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_band_pack_async(self.h, ctypes.byref(grid_data), int(nb), int(world), x.data_ptr(),
                                        y.data_ptr(), n, int(base), ox.data_ptr(), oy.data_ptr(), oi.data_ptr(),
                                        cnt.data_ptr())
        if rc:
            self._check(rc, "band_pack_async")
        return ox[:n], oy[:n], oi[:n], cnt[:world]

    def band_pack_query_async(self, grid_data: Grid, nb: int, world: int, qx: float, qy: float, r: float, x, y,
                              base: int = 0):
        """geohip_band_pack_query_async: as band_pack_async, keeping only the points of the point
        query's G u C cells (the reference's filter before keyBy(gridID))."""
        import torch
        self._dev(x, "x")
        self._dev(y, "y")
        n = x.numel()
        if y.numel() != n:
            raise GeohipArgumentError("band_pack_query_async: x and y differ in length")
        ox = torch.empty(max(n, 1), dtype=torch.float64, device=x.device)
        oy = torch.empty_like(ox)
        oi = torch.empty(max(n, 1), dtype=torch.int64, device=x.device)
        cnt = torch.empty(max(world, 1), dtype=torch.int64, device=x.device)
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_band_pack_query_async(self.h, ctypes.byref(grid_data), int(nb), int(world), qx, qy, r,
                                              x.data_ptr(), y.data_ptr(), n, int(base), ox.data_ptr(), oy.data_ptr(),
                                              oi.data_ptr(), cnt.data_ptr())
        if rc:
            self._check(rc, "band_pack_query_async")
        return ox[:n], oy[:n], oi[:n], cnt[:world]

    def range_pp_async(self, grid: Grid, x, y, qx, qy, r, approximate, out_idx, cap, out_count):
        self._dev(x, "x")
        self._dev(y, "y")
        self._dev(out_idx, "out_idx", "int32")
        self._dev(out_count, "out_count", "int64")
        if out_idx.numel() < cap:
            raise GeohipArgumentError("range_pp_async: out_idx shorter than cap")
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_range_pp_async(self.h, ctypes.byref(grid), x.data_ptr(), y.data_ptr(), x.numel(), qx, qy, r,
                                       int(approximate), out_idx.data_ptr(), cap, out_count.data_ptr())
        if rc:
            self._check(rc, "range_pp_async")

    def join_pp_async(self, grid_data: Grid, grid_query: Grid, dx, dy, qx, qy, r, approximate, out, out_count):
        """geohip_join_pp_async: pairs into ``out`` ([cap, 2] int32, device), the pair total into
        ``out_count`` (one int64, device); nothing is read back (pairs past cap are not written;
        query-key errors surface at sync())."""
        for t, nm in ((dx, "dx"), (dy, "dy"), (qx, "qx"), (qy, "qy")):
            self._dev(t, nm)
        self._dev(out, "out", "int32")
        self._dev(out_count, "out_count", "int64")
        if out.dim() != 2 or out.shape[1] != 2:
            raise GeohipArgumentError("join_pp_async: out must be [cap, 2]")
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_join_pp_async(self.h, ctypes.byref(grid_data), ctypes.byref(grid_query), dx.data_ptr(),
                                      dy.data_ptr(), dx.numel(), qx.data_ptr(), qy.data_ptr(), qx.numel(), r,
                                      int(approximate), out.data_ptr(), out.shape[0], out_count.data_ptr())
        if rc:
            self._check(rc, "join_pp_async")

    def range_ppoly_async(self, grid: Grid, x, y, ring_off, vx, vy, r, approximate, out, out_count, poly_rings=None,
                          point_base=None):
        """geohip_range_ppoly_async: (polygon, point) pairs into ``out`` ([cap, 2] int32, device),
        the pair total into ``out_count`` (one int64, device); a candidate-buffer overflow surfaces
        at sync().  ``point_base`` (geohip_range_ppoly_pane_async): point indices point_base +
        position (mod 2^32)."""
        if point_base is None:
            self._ppoly_async(lib.geohip_range_ppoly_async, "range_ppoly_async", (ctypes.byref(grid),), x, y, ring_off,
                              vx, vy, r, approximate, out, out_count, poly_rings)
        else:
            base = int(point_base) & 0xFFFFFFFF
            fn = lambda h, g, px, py, n, *rest: lib.geohip_range_ppoly_pane_async(h, g, px, py, n, base, *rest)  # noqa: E731
            self._ppoly_async(fn, "range_ppoly_pane_async", (ctypes.byref(grid),), x, y, ring_off, vx, vy, r,
                              approximate, out, out_count, poly_rings)

    def join_ppoly_async(self, grid_points: Grid, grid_query: Grid, x, y, ring_off, vx, vy, r, approximate, out,
                         out_count, poly_rings=None):
        """geohip_join_ppoly_async: (point, polygon) pairs, as range_ppoly_async."""
        self._ppoly_async(lib.geohip_join_ppoly_async, "join_ppoly_async",
                          (ctypes.byref(grid_points), ctypes.byref(grid_query)), x, y, ring_off, vx, vy, r,
                          approximate, out, out_count, poly_rings)

    def _ppoly_async(self, fn, what, grids, x, y, ring_off, vx, vy, r, approximate, out, out_count, poly_rings):
        self._dev(x, "x")
        self._dev(y, "y")
        self._dev(out, "out", "int32")
        self._dev(out_count, "out_count", "int64")
        if out.dim() != 2 or out.shape[1] != 2:
            raise GeohipArgumentError(f"{what}: out must be [cap, 2]")
        pr, ring_off, vx, vy, npoly = _poly_arrays(poly_rings, ring_off, vx, vy)
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = fn(self.h, *grids, x.data_ptr(), y.data_ptr(), x.numel(), _ptr(pr), _ptr(ring_off), _ptr(vx), _ptr(vy),
                len(vx), npoly, r, int(approximate), out.data_ptr(), out.shape[0], out_count.data_ptr())
        if rc:
            self._check(rc, what)

    def join_pp(self, grid_data: Grid, grid_query: Grid, dx, dy, qx, qy, r, approximate=False, cap=None, out=None):
        """Pairs (data idx, query idx).  ``out`` (optional): a preallocated [cap, 2] u32/i32 buffer on
        the same side as the inputs (one pass, no count-only pass)."""
        dx, dy, qx, qy = _f64(dx), _f64(dy), _f64(qx), _f64(qy)
        dev = self._mem_for(dx, dy, qx, qy)
        cnt = c_uint64(0)
        if cap is None and out is None:
            rc = lib.geohip_join_pp_count_only(self.h, ctypes.byref(grid_data), ctypes.byref(grid_query), _ptr(dx),
                                               _ptr(dy), len(dx), _ptr(qx), _ptr(qy), len(qx), r, int(approximate),
                                               ctypes.byref(cnt))
            self._check(rc, "join_pp_count_only")
            cap = cnt.value
        if out is not None:
            cap = len(out) if cap is None else min(cap, len(out))
        elif dev:
            import torch
            out = torch.empty((max(cap, 1), 2), dtype=torch.int32, device=dx.device)
        else:
            out = np.empty((max(cap, 1), 2), dtype=np.uint32)
        rc = lib.geohip_join_pp(self.h, ctypes.byref(grid_data), ctypes.byref(grid_query), _ptr(dx), _ptr(dy),
                                len(dx), _ptr(qx), _ptr(qy), len(qx), r, int(approximate), _ptr(out), cap,
                                ctypes.byref(cnt))
        self._check(rc, "join_pp")
        return out[:cnt.value]

    def join_pp_count(self, grid_data: Grid, grid_query: Grid, dx, dy, qx, qy, r, approximate=False) -> int:
        dx, dy, qx, qy = _f64(dx), _f64(dy), _f64(qx), _f64(qy)
        self._mem_for(dx, dy, qx, qy)
        cnt = c_uint64(0)
        rc = lib.geohip_join_pp_count_only(self.h, ctypes.byref(grid_data), ctypes.byref(grid_query), _ptr(dx),
                                           _ptr(dy), len(dx), _ptr(qx), _ptr(qy), len(qx), r, int(approximate),
                                           ctypes.byref(cnt))
        self._check(rc, "join_pp_count_only")
        return cnt.value

    def range_ppoly(self, grid: Grid, x, y, ring_off, vx, vy, r, approximate=False, cap=None, out=None,
                    poly_rings=None, point_base=None):
        """Pairs (polygon idx, point idx).  ``out``: optional preallocated [cap, 2] buffer.
        ``poly_rings``: polygon i = rings [poly_rings[i], poly_rings[i+1]) of ``ring_off``
        (shell and holes, Polygon.createPolygon); None = one ring per polygon.  ``point_base``
        (geohip_range_ppoly_pane): point indices are point_base + position (mod 2^32)."""
        x, y = _f64(x), _f64(y)
        self._mem_for(x, y)
        pr, ring_off, vx, vy, npoly = _poly_arrays(poly_rings, ring_off, vx, vy)
        cnt = c_uint64(0)
        if point_base is None:
            call = lib.geohip_range_ppoly
        else:
            base = int(point_base) & 0xFFFFFFFF
            call = lambda h, g, px, py, n, *rest: lib.geohip_range_ppoly_pane(h, g, px, py, n, base, *rest)  # noqa: E731
        if out is not None:
            cap = len(out) if cap is None else min(cap, len(out))
        if cap is None:
            rc = call(self.h, ctypes.byref(grid), _ptr(x), _ptr(y), len(x), _ptr(pr),
                      _ptr(ring_off), _ptr(vx), _ptr(vy), len(vx), npoly, r, int(approximate), None, 0,
                      ctypes.byref(cnt))
            if rc not in (OK, ERR_CAPACITY):
                self._check(rc, "range_ppoly")
            cap = cnt.value
        if out is not None:
            pass
        elif _is_device(x):
            import torch
            out = torch.empty((max(cap, 1), 2), dtype=torch.int32, device=x.device)
        else:
            out = np.empty((max(cap, 1), 2), dtype=np.uint32)
        rc = call(self.h, ctypes.byref(grid), _ptr(x), _ptr(y), len(x), _ptr(pr), _ptr(ring_off),
                  _ptr(vx), _ptr(vy), len(vx), npoly, r, int(approximate), _ptr(out), cap, ctypes.byref(cnt))
        self._check(rc, "range_ppoly")
        return out[:cnt.value]

    def join_ppoly(self, grid_points: Grid, grid_query: Grid, x, y, ring_off, vx, vy, r, approximate=False, cap=None,
                   out=None, poly_rings=None):
        """Point-polygon join: pairs (point idx, polygon idx).  ``out``: optional [cap, 2] buffer.
        ``poly_rings`` as for range_ppoly."""
        x, y = _f64(x), _f64(y)
        self._mem_for(x, y)
        pr, ring_off, vx, vy, npoly = _poly_arrays(poly_rings, ring_off, vx, vy)
        cnt = c_uint64(0)
        args = (self.h, ctypes.byref(grid_points), ctypes.byref(grid_query), _ptr(x), _ptr(y), len(x), _ptr(pr),
                _ptr(ring_off), _ptr(vx), _ptr(vy), len(vx), npoly, r, int(approximate))
        if out is not None:
            cap = len(out) if cap is None else min(cap, len(out))
        if cap is None:
            rc = lib.geohip_join_ppoly(*args, None, 0, ctypes.byref(cnt))
            if rc not in (OK, ERR_CAPACITY):
                self._check(rc, "join_ppoly")
            cap = cnt.value
        if out is None:
            if _is_device(x):
                import torch
                out = torch.empty((max(cap, 1), 2), dtype=torch.int32, device=x.device)
            else:
                out = np.empty((max(cap, 1), 2), dtype=np.uint32)
        rc = lib.geohip_join_ppoly(*args, _ptr(out), cap, ctypes.byref(cnt))
        self._check(rc, "join_ppoly")
        return out[:cnt.value]

    def knn_ppoly(self, grid: Grid, x, y, vx, vy, r, k, approximate=False, ring_off=None):
        """Point-polygon kNN of one polygon: (idx, dist) ascending by (dist, idx).  ``ring_off``:
        its rings (shell and holes) as vertex offsets into vx/vy; None = one ring."""
        x, y = _f64(x), _f64(y)
        dev = self._mem_for(x, y)
        vx = _host(vx, np.float64)
        vy = _host(vy, np.float64)
        ring_off = _host([0, len(vx)] if ring_off is None else ring_off, np.uint32)
        _check_rings(ring_off, vx, vy)
        if dev:
            import torch
            oi = torch.empty(k, dtype=torch.int32, device=x.device)
            od = torch.empty(k, dtype=torch.float64, device=x.device)
        else:
            oi = np.empty(k, dtype=np.uint32)
            od = np.empty(k, dtype=np.float64)
        cnt = c_uint32(0)
        rc = lib.geohip_knn_ppoly(self.h, ctypes.byref(grid), _ptr(x), _ptr(y), len(x), _ptr(ring_off),
                                  len(ring_off) - 1, _ptr(vx), _ptr(vy), len(vx), r, k, int(approximate), _ptr(oi), _ptr(od),
                                  ctypes.byref(cnt))
        self._check(rc, "knn_ppoly")
        return oi[:cnt.value], od[:cnt.value]

    def knn_ppoly_async(self, grid: Grid, x, y, vx, vy, r, k, approximate, out_idx, out_dist, out_count, ring_off=None):
        """geohip_knn_ppoly_async: device window, k-long device outputs (sentinel-padded), count
        on the device; no host synchronisation (the polygon plan is cached by the ctx)."""
        self._dev(x, "x")
        self._dev(y, "y")
        self._dev(out_idx, "out_idx", "int32")
        self._dev(out_dist, "out_dist")
        self._dev(out_count, "out_count", "int32")
        if out_idx.numel() < k or out_dist.numel() < k:
            raise GeohipArgumentError("knn_ppoly_async: outputs shorter than k")
        vx = _host(vx, np.float64)
        vy = _host(vy, np.float64)
        ring_off = _host([0, len(vx)] if ring_off is None else ring_off, np.uint32)
        _check_rings(ring_off, vx, vy)
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        rc = lib.geohip_knn_ppoly_async(self.h, ctypes.byref(grid), x.data_ptr(), y.data_ptr(), x.numel(),
                                        _ptr(ring_off), len(ring_off) - 1, _ptr(vx), _ptr(vy), len(vx), r, k, int(approximate),
                                        out_idx.data_ptr(), out_dist.data_ptr(), out_count.data_ptr())
        if rc:
            self._check(rc, "knn_ppoly_async")

    def ingest_points(self, spec: IngestSpec, text, grid: Grid | None = None, with_ts=False, with_cell=False,
                      cap=None, out=None):
        """geohip_ingest_points: text (bytes / uint8 numpy on the host, uint8 torch on the device)
        -> dict(x, y[, ts][, cell]) trimmed to the record count.  Raises GeohipUnsupportedError
        (attribute ``bad`` = first rejected record) where the device grammar rejects a record."""
        if isinstance(text, (bytes, bytearray)):
            text = np.frombuffer(text, dtype=np.uint8)
        dev = self._mem_for(text, dtype="uint8")
        nbytes = int(text.numel()) if dev else int(text.size)
        if cap is None:
            cap = nbytes // 2 + 1  # a record has at least one byte plus its '\n'
        if out is None:
            if dev:
                import torch
                mk = lambda dt: torch.empty(max(cap, 1), dtype=dt, device=text.device)  # noqa: E731
                out = {"x": mk(torch.float64), "y": mk(torch.float64)}
                if with_ts:
                    out["ts"] = mk(torch.int64)
                if with_cell:
                    out["cell"] = mk(torch.int32)
            else:
                out = {"x": np.empty(max(cap, 1)), "y": np.empty(max(cap, 1))}
                if with_ts:
                    out["ts"] = np.empty(max(cap, 1), dtype=np.int64)
                if with_cell:
                    out["cell"] = np.empty(max(cap, 1), dtype=np.uint32)
        cnt, bad = c_uint64(0), c_uint64(0)
        rc = lib.geohip_ingest_points(self.h, ctypes.byref(grid) if grid is not None else None, ctypes.byref(spec),
                                      _ptr(text), nbytes, _ptr(out["x"]), _ptr(out["y"]), _ptr(out.get("ts")),
                                      _ptr(out.get("cell")), cap, ctypes.byref(cnt), ctypes.byref(bad))
        if rc == ERR_UNSUPPORTED and bad.value != 2**64 - 1:
            err = GeohipUnsupportedError(f"ingest_points: {lib.geohip_last_error(self.h).decode(errors='replace')}")
            err.bad = bad.value
            raise err
        self._check(rc, "ingest_points")
        return {k: v[:cnt.value] for k, v in out.items()}

    def ingest_trajectory(self, spec: IngestSpec, text, grid: Grid | None = None, traj: TrajSpec | None = None,
                          with_ts=True, with_cell=False, with_oid=True, cap=None):
        """geohip_ingest_trajectory (TrajectoryStream: the Point's objID, x, y, timestamp, cell):
        dict(x, y[, ts][, cell][, oid]) trimmed to the record count; ``oid`` = the objID spans
        (ingest_oid_compact / oid_spans_to_strings read them)."""
        if isinstance(text, (bytes, bytearray)):
            text = np.frombuffer(text, dtype=np.uint8)
        dev = self._mem_for(text, dtype="uint8")
        nbytes = int(text.numel()) if dev else int(text.size)
        if cap is None:
            cap = nbytes // 2 + 1
        if dev:
            import torch
            mk = lambda dt: torch.empty(max(cap, 1), dtype=dt, device=text.device)  # noqa: E731
            i64, i32, f64 = torch.int64, torch.int32, torch.float64
        else:
            mk = lambda dt: np.empty(max(cap, 1), dtype=dt)  # noqa: E731
            i64, i32, f64 = np.int64, np.uint32, np.float64
        out = {"x": mk(f64), "y": mk(f64)}
        if with_ts:
            out["ts"] = mk(i64)
        if with_cell:
            out["cell"] = mk(i32)
        if with_oid:
            out["oid"] = mk(i64)
        cnt, bad = c_uint64(0), c_uint64(0)
        rc = lib.geohip_ingest_trajectory(self.h, ctypes.byref(grid) if grid is not None else None, ctypes.byref(spec),
                                          ctypes.byref(traj) if traj is not None else None, _ptr(text), nbytes,
                                          _ptr(out["x"]), _ptr(out["y"]), _ptr(out.get("ts")), _ptr(out.get("cell")),
                                          _ptr(out.get("oid")), cap, ctypes.byref(cnt), ctypes.byref(bad))
        if rc == ERR_UNSUPPORTED and bad.value != 2**64 - 1:
            err = GeohipUnsupportedError(f"ingest_trajectory: {lib.geohip_last_error(self.h).decode(errors='replace')}")
            err.bad = bad.value
            raise err
        self._check(rc, "ingest_trajectory")
        return {k: v[:cnt.value] for k, v in out.items()}

    def ingest_oid_compact(self, text, spans):
        """geohip_ingest_oid_compact (device tensors): (oid_text uint8, oid_off int64 [m + 1], bit 63 =
        null) -- the form format_points takes."""
        import torch
        self._dev(text, "text", "uint8")
        self._dev(spans, "spans", "int64")
        if self._mem != MEM_DEVICE:
            self.set_mem(MEM_DEVICE)
        m = spans.numel()
        off = torch.empty(m + 1, dtype=torch.int64, device=text.device)
        ln = c_uint64(0)
        rc = lib.geohip_ingest_oid_compact(self.h, text.data_ptr(), text.numel(), spans.data_ptr(), m, None, 0,
                                           off.data_ptr(), ctypes.byref(ln))
        if rc not in (OK, ERR_CAPACITY):
            self._check(rc, "ingest_oid_compact")
        out = torch.empty(max(ln.value, 1), dtype=torch.uint8, device=text.device)
        rc = lib.geohip_ingest_oid_compact(self.h, text.data_ptr(), text.numel(), spans.data_ptr(), m, out.data_ptr(),
                                           ln.value, off.data_ptr(), ctypes.byref(ln))
        self._check(rc, "ingest_oid_compact")
        return out[:ln.value], off

    def synth_uniform_async(self, x, y, base, seed, bbox):
        self._dev(x, "x")
        self._dev(y, "y")
        min_x, max_x, min_y, max_y = bbox
        rc = lib.geohip_synth_uniform_async(self.h, _ptr(x), _ptr(y), len(x), base, seed, min_x, max_x, min_y, max_y)
        self._check(rc, "synth_uniform_async")

    def debug_knn_pass_stats(self):
        """(entries gathered, of them spilled, kept at or below the k-th bin) of the last kNN pass."""
        out = np.zeros(3, dtype=np.uint32)
        self._check(lib.geohip_debug_knn_pass_stats(self.h, out.ctypes.data_as(c_void_p)), "debug_knn_pass_stats")
        return tuple(int(v) for v in out)

    def debug_knn_pass_trace(self, grid, x, y, qx, qy, r, k, ablation=0):
        """One traced kNN pass on device x/y: [nblocks, 8] timestamps (100 MHz, 0 = not reached)."""
        buf = np.zeros(16 * 1024, dtype=np.uint64)
        nb = c_uint32(0)
        self._dev(x, "x")
        self.set_mem(MEM_DEVICE)
        rc = lib.geohip_debug_knn_pass_trace(self.h, ctypes.byref(grid), _ptr(x), _ptr(y), x.numel(), qx, qy, r, k,
                                             ablation, buf.ctypes.data_as(c_void_p), len(buf), ctypes.byref(nb))
        self._check(rc, "debug_knn_pass_trace")
        return buf[:16 * nb.value].reshape(nb.value, 16)

    def selftest_fp64(self, a, b):
        """Device fp64 primitive bits (test hook): returns (sqrt|a|, a/b, hypot(a,b), a*b-b*b)."""
        import torch
        outs = [torch.empty_like(a) for _ in range(4)]
        self.set_mem(MEM_DEVICE)
        rc = lib.geohip_debug_selftest_fp64(self.h, _ptr(a), _ptr(b), len(a), *[_ptr(o) for o in outs])
        self._check(rc, "selftest_fp64")
        return outs
