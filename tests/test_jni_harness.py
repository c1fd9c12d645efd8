"""The JNI shim (jvm/native/geohip_jni.c) compiled and executed without a JVM.

No JDK exists in this image, so the shim is built (by __graft_entry__.build(), gcc -Wall -Werror)
against a test-only jni.h stand-in (tests/jni_stub/jni.h: the JNI types and the function-table
members the shim uses) together with a fake JNIEnv (tests/jni_stub/fake_jni.c: direct ByteBuffers,
int[] / double[] / Object[] arrays, pending exceptions).  The tests call the very
Java_GeoFlink_utils_GeoHip_* entry points a JVM would call for GeoHip's native methods
(jvm/src/GeoFlink/utils/GeoHip.java), so what is exercised is the shim's own marshalling:
two-phase sizing, status -> exception mapping, buffer validation, pairs_array, grid_of.

CPU: the build, and every argument check the shim makes before it reaches the library.  GPU: each
native method against the C oracle (cref), including the two-phase pair calls and the
GEOHIP_ERR_ARG -> IllegalArgumentException mapping where the reference calls System.exit(1)
(UniformGrid.java:272-276).  Reference surface: PointPointRangeQuery.java:32-36,
PointPointKNNQuery.java:29-33, PointPointJoinQuery.java:20-24, PointPolygonRangeQuery.java:26-30.
"""
import ctypes
import subprocess
from ctypes import POINTER, c_char_p, c_double, c_int32, c_int64, c_uint8, c_void_p
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
STUB = ROOT / "tests" / "jni_stub"
LIB = STUB / "libgeohip_jni_test.so"
P = "Java_GeoFlink_utils_GeoHip_"

IAE = "java/lang/IllegalArgumentException"


def build_cmd(out=LIB):
    return ["gcc", "-O1", "-Wall", "-Wextra", "-Wno-unused-parameter", "-Werror", "-shared", "-fPIC",
            f"-I{STUB}", f"-I{ROOT / 'include'}", str(ROOT / "jvm" / "native" / "geohip_jni.c"),
            str(STUB / "fake_jni.c"), f"-L{ROOT / 'spatialflink_amd'}", "-lgeohip",
            "-Wl,-rpath,$ORIGIN/../../spatialflink_amd", "-o", str(out)]


class Jni:
    """The shim's entry points over the fake JNIEnv."""

    def __init__(self):
        if not LIB.exists():
            pytest.skip("tests/jni_stub/libgeohip_jni_test.so not built (run __graft_entry__.build())")
        L = self.L = ctypes.CDLL(str(LIB))
        J = c_void_p  # jobject
        L.fake_env.restype = c_void_p
        L.fake_direct.restype = J
        L.fake_direct.argtypes = [c_void_p, c_int64]
        L.fake_ints.restype = J
        L.fake_ints.argtypes = [c_void_p, c_int32]
        L.fake_doubles.restype = J
        L.fake_doubles.argtypes = [c_void_p, c_int32]
        L.fake_len.restype = c_int32
        L.fake_len.argtypes = [J]
        L.fake_data.restype = c_void_p
        L.fake_data.argtypes = [J]
        L.fake_elem.restype = J
        L.fake_elem.argtypes = [J, c_int32]
        L.fake_exception_class.restype = c_char_p
        L.fake_exception_message.restype = c_char_p
        self.env = L.fake_env()
        E = [c_void_p, c_void_p]  # JNIEnv*, jclass
        sig = {
            "abiVersion": (c_int32, E),
            "create": (c_int64, E + [c_int32]),
            "destroy": (None, E + [c_int64]),
            "rangeOrder": (None, E + [c_int64, c_int32]),
            "rangePP": (J, E + [c_int64, J, J, J, c_int32, c_double, c_double, c_double, c_uint8]),
            "knnPP": (c_int32, E + [c_int64, J, J, J, c_int32, c_double, c_double, c_double, c_int32, J, J]),
            "knnRangePP": (J, E + [c_int64, J, J, J, c_int32, c_double, c_double, c_double, c_int32, c_uint8, J, J]),
            "joinPP": (J, E + [c_int64, J, J, J, J, c_int32, J, J, c_int32, c_double, c_uint8]),
            "rangePPoly": (J, E + [c_int64, J, J, J, c_int32, J, J, J, J, c_double, c_uint8]),
            "joinPPoly": (J, E + [c_int64, J, J, J, J, c_int32, J, J, J, J, c_double, c_uint8]),
            "knnPPoly": (c_int32, E + [c_int64, J, J, J, c_int32, J, J, J, c_double, c_int32, c_uint8, J, J]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, P + name)
            f.restype, f.argtypes = res, args
        self.keep = []

    def call(self, name, *args):
        """Call a native method; returns (result, (exception class, message) or None)."""
        self.L.fake_clear()
        r = getattr(self.L, P + name)(self.env, None, *args)
        cls = self.L.fake_exception_class().decode()
        return r, ((cls, self.L.fake_exception_message().decode()) if cls else None)

    # Java objects
    def direct(self, a):
        a = np.ascontiguousarray(a, np.float64)
        self.keep.append(a)
        return self.L.fake_direct(a.ctypes.data if len(a) else None, 8 * len(a))

    def heap_buffer(self, n):
        return self.L.fake_direct(None, 8 * n)

    def ints(self, a):
        a = np.ascontiguousarray(a, np.int32)
        return self.L.fake_ints(a.ctypes.data, len(a))

    def doubles(self, a):
        a = np.ascontiguousarray(a, np.float64)
        return self.L.fake_doubles(a.ctypes.data, len(a))

    def new_ints(self, n):
        return self.L.fake_ints(None, n)

    def new_doubles(self, n):
        return self.L.fake_doubles(None, n)

    def int_array(self, o):
        n = self.L.fake_len(o)
        return np.ctypeslib.as_array(ctypes.cast(self.L.fake_data(o), POINTER(c_int32)), (max(n, 0),)).copy() \
            if n > 0 else np.zeros(0, np.int32)

    def double_array(self, o):
        n = self.L.fake_len(o)
        return np.ctypeslib.as_array(ctypes.cast(self.L.fake_data(o), POINTER(c_double)), (n,)).copy() \
            if n > 0 else np.zeros(0)

    def elem(self, o, i):
        return self.L.fake_elem(o, i)

    def reset(self):
        self.L.fake_reset()
        self.keep.clear()


def _grid(n=100):
    from spatialflink_amd import synth
    bj = synth.BEIJING
    l = (bj[1] - bj[0]) / n
    return np.array([bj[0], bj[2], l, n], np.float64)


def test_shim_builds_warning_free_against_the_stub(tmp_path):
    r = subprocess.run(build_cmd(tmp_path / "libgeohip_jni_check.so"), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_argument_checks_before_the_library():
    """Checks the shim makes before any libgeohip call (ctx handle 0: reaching the library would
    fail with a different message): heap / short / null buffers, negative sizes, short kNN outputs."""
    j = Jni()
    g = j.doubles(_grid())
    x = j.direct(np.zeros(10))
    short = j.direct(np.zeros(5))
    for bx, by, n in [(j.heap_buffer(10), x, 10), (x, short, 10), (None, x, 10), (x, x, -1)]:
        r, exc = j.call("rangePP", 0, g, bx, by, n, 116.4, 39.9, 0.5, 0)
        assert r is None and exc and exc[0] == IAE, exc
        assert "direct ByteBuffers" in exc[1]
    r, exc = j.call("knnPP", 0, g, x, x, 10, 116.4, 39.9, 0.5, 8, j.new_ints(4), j.new_doubles(8))
    assert r == -1 and exc[0] == IAE and "hold k" in exc[1]
    r, exc = j.call("knnRangePP", 0, g, x, x, 10, 116.4, 39.9, 0.5, 8, 0, j.new_ints(8), None)
    assert r is None and exc[0] == IAE
    r, exc = j.call("joinPP", 0, g, g, x, x, 10, x, short, 10, 0.05, 0)
    assert r is None and exc[0] == IAE
    r, exc = j.call("knnPPoly", 0, g, j.heap_buffer(10), x, 10, j.ints([0, 4]), j.doubles(np.zeros(4)),
                    j.doubles(np.zeros(4)), 0.1, 3, 0, j.new_ints(3), j.new_doubles(3))
    assert r == -1 and exc[0] == IAE
    # polygon arrays that disagree: the shim's own check
    r, exc = j.call("rangePPoly", 0, g, x, x, 10, None, j.ints([0, 4]), j.doubles(np.zeros(4)),
                    j.doubles(np.zeros(3)), 0.1, 0)
    assert r is None and exc == (IAE, "polygon arrays")
    r, exc = j.call("abiVersion")
    from spatialflink_amd import _abi
    assert exc is None and r == _abi.lib.geohip_abi_version() == 2
    j.reset()


# ---- GPU: every native method against the oracle ----------------------------------------------

@pytest.fixture(scope="module")
def jni_ctx():
    j = Jni()
    h, exc = j.call("create", 1)
    assert exc is None and h
    yield j, h
    j.call("destroy", h)
    j.reset()


@pytest.mark.gpu
def test_point_point_natives(jni_ctx):
    import cref
    from spatialflink_amd import synth
    j, h = jni_ctx
    gv = _grid(100)
    g = j.doubles(gv)
    cg = cref.grid(gv[0], gv[1], gv[2], 100)
    hx, hy = synth.uniform(300_000, 71)
    x, y = j.direct(hx), j.direct(hy)
    qx, qy = synth.README_QUERY
    n = len(hx)
    want = sorted(cref.range_pp(cg, hx, hy, qx, qy, 0.3).tolist())
    r, exc = j.call("rangePP", h, g, x, y, n, qx, qy, 0.3, 0)
    assert exc is None
    assert j.int_array(r).tolist() == want  # the default: ascending
    _, exc = j.call("rangeOrder", h, 1)  # what the GeoHip constructor sets: the unordered set
    assert exc is None
    r, exc = j.call("rangePP", h, g, x, y, n, qx, qy, 0.3, 0)
    assert exc is None and sorted(j.int_array(r).tolist()) == want
    _, exc = j.call("rangeOrder", h, 5)
    assert exc[0] == IAE
    k = 50
    oi, od = j.new_ints(k), j.new_doubles(k)
    cnt, exc = j.call("knnPP", h, g, x, y, n, qx, qy, 0.3, k, oi, od)
    wi, wd = cref.knn_pp(cg, hx, hy, qx, qy, 0.3, k)
    assert exc is None and cnt == len(wi)
    assert j.int_array(oi)[:cnt].tolist() == wi.tolist()
    assert np.array_equal(j.double_array(od)[:cnt].view(np.uint64), wd.view(np.uint64))
    ki, kd = j.new_ints(k), j.new_doubles(k)
    res, exc = j.call("knnRangePP", h, g, x, y, n, qx, qy, 0.3, k, 0, ki, kd)
    assert exc is None
    assert j.int_array(j.elem(res, 0)).tolist() == [len(wi)]
    assert j.int_array(ki)[:len(wi)].tolist() == wi.tolist()
    assert sorted(j.int_array(j.elem(res, 1)).tolist()) == sorted(cref.range_pp(cg, hx, hy, qx, qy, 0.3).tolist())
    # k = 0 and r < 0 in the join: GEOHIP_ERR_ARG -> IllegalArgumentException (System.exit(1) in
    # UniformGrid.getNeighboringCells)
    cnt, exc = j.call("knnPP", h, g, x, y, n, qx, qy, 0.3, 0, oi, od)
    assert cnt == -1 and exc[0] == IAE
    hqx, hqy = synth.uniform(500, 72)
    r, exc = j.call("joinPP", h, g, g, x, y, n, j.direct(hqx), j.direct(hqy), len(hqx), -0.01, 0)
    assert r is None and exc[0] == IAE
    # the two-phase join (count-only, then the pairs)
    r, exc = j.call("joinPP", h, g, g, x, y, n, j.direct(hqx), j.direct(hqy), len(hqx), 0.02, 0)
    assert exc is None
    got = j.int_array(r).reshape(-1, 2)
    want = cref.join_pp(cg, cg, hx, hy, hqx, hqy, 0.02)
    assert len(got) == len(want) > 0
    from helpers import pairs_sorted
    assert np.array_equal(pairs_sorted(got), pairs_sorted(want))


@pytest.mark.gpu
def test_point_polygon_natives(jni_ctx):
    import cref
    from helpers import pairs_sorted
    from spatialflink_amd import synth
    j, h = jni_ctx
    gv = _grid(500)
    g = j.doubles(gv)
    cg = cref.grid(gv[0], gv[1], gv[2], 500)
    hx, hy = synth.uniform(400_000, 73)
    x, y = j.direct(hx), j.direct(hy)
    off, vx, vy = synth.star_polygons(40, 74, r_min=0.02, r_max=0.05)
    ro, jvx, jvy = j.ints(off.astype(np.int32)), j.doubles(vx), j.doubles(vy)
    r, exc = j.call("rangePPoly", h, g, x, y, len(hx), None, ro, jvx, jvy, 0.005, 0)
    assert exc is None
    got = j.int_array(r).reshape(-1, 2)
    want = cref.range_ppoly(cg, hx, hy, off, vx, vy, 0.005)
    assert len(got) == len(want) > 0 and np.array_equal(pairs_sorted(got), pairs_sorted(want))
    r, exc = j.call("joinPPoly", h, g, g, x, y, len(hx), None, ro, jvx, jvy, 0.005, 0)
    assert exc is None
    got = j.int_array(r).reshape(-1, 2)
    want = cref.join_ppoly(cg, cg, hx, hy, off, vx, vy, 0.005)
    assert len(got) == len(want) > 0 and np.array_equal(pairs_sorted(got), pairs_sorted(want))
    # one polygon (its single ring) for the kNN
    k = 40
    oi, od = j.new_ints(k), j.new_doubles(k)
    p0 = slice(int(off[0]), int(off[1]))
    cnt, exc = j.call("knnPPoly", h, g, x, y, len(hx), j.ints([0, off[1] - off[0]]), j.doubles(vx[p0]),
                      j.doubles(vy[p0]), 0.01, k, 0, oi, od)
    wi, wd = cref.knn_ppoly(cg, hx, hy, vx[p0], vy[p0], 0.01, k)
    assert exc is None and cnt == len(wi) > 0
    assert j.int_array(oi)[:cnt].tolist() == wi.tolist()
    assert np.array_equal(j.double_array(od)[:cnt].view(np.uint64), wd.view(np.uint64))
    # a polygon whose ring has <= 3 coords: the reference leaves it null -> GEOHIP_ERR_ARG -> IAE
    r, exc = j.call("rangePPoly", h, g, x, y, len(hx), None, j.ints([0, 3]), j.doubles(vx[:3]), j.doubles(vy[:3]),
                    0.005, 0)
    assert r is None and exc[0] == IAE
