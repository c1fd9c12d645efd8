"""Consistency of the JVM drop-in sources (jvm/): no JDK exists in this image, so they are
checked as text -- every native method of GeoFlink.utils.GeoHip has its JNI symbol in
jvm/native/geohip_jni.c, every libgeohip function the shim calls is declared in include/geohip.h
and exported by libgeohip.so, and the operator classes keep the reference operators' constructor
and run() signatures (PointPointRangeQuery.java:32-36, PointPointKNNQuery.java:29-33,
PointPointJoinQuery.java:20-24, PointPolygonRangeQuery.java:26-30).  With a JDK present the shim
is also compiled (gcc -fsyntax-only against its jni.h)."""
import os
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
JAVA = ROOT / "jvm" / "src" / "GeoFlink"
SHIM = ROOT / "jvm" / "native" / "geohip_jni.c"


def _natives():
    src = (JAVA / "utils" / "GeoHip.java").read_text()
    return re.findall(r"private static native \S+ (\w+)\(", src)


def test_every_native_method_has_its_jni_symbol():
    shim = SHIM.read_text()
    names = _natives()
    assert len(names) >= 10
    for n in names:
        assert f"Java_GeoFlink_utils_GeoHip_{n}(" in shim, n


def test_shim_calls_only_exported_abi_functions():
    shim = SHIM.read_text()
    header = (ROOT / "include" / "geohip.h").read_text()
    called = set(re.findall(r"\b(geohip_[a-z_0-9]+)\s*\(", shim))
    called.discard("geohip_jni")
    assert called
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    lib = ROOT / "spatialflink_amd" / "libgeohip.so"
    syms = subprocess.run([nm, "-D", "--defined-only", str(lib)], capture_output=True, text=True).stdout
    for f in sorted(called):
        assert re.search(rf"\b{f}\s*\(", header), f"{f} not declared in include/geohip.h"
        assert re.search(rf"\s{f}$", syms, re.M), f"{f} not exported by libgeohip.so"


@pytest.mark.parametrize("cls,sig", [
    ("GeoHipPointPointRangeQuery", r"public DataStream<Point> run\(DataStream<Point> pointStream, Point queryPoint, "
                                   r"double queryRadius\)"),
    ("GeoHipPointPointKNNQuery", r"run\(DataStream<Point> pointStream,\s+Point queryPoint, double queryRadius,\s+"
                                 r"Integer k\)"),
    ("GeoHipPointPointJoinQuery", r"public DataStream<Tuple2<Point, Point>> run\(DataStream<Point> ordinaryPointStream, "
                                  r"DataStream<Point> queryPointStream,\s+double queryRadius\)"),
    ("GeoHipPointPolygonRangeQuery", r"public DataStream<Point> run\(DataStream<Point> pointStream, Polygon queryPolygon, "
                                     r"double queryRadius\)"),
])
def test_operator_signatures(cls, sig):
    src = (JAVA / "spatialOperators" / "geohip" / f"{cls}.java").read_text()
    assert re.search(sig, src), cls
    assert re.search(rf"public {cls}\(QueryConfiguration conf, SpatialIndex index(1, SpatialIndex index2)?\)", src)


def test_shim_compiles_with_a_jdk():
    home = os.environ.get("JAVA_HOME")
    inc = Path(home) / "include" if home else None
    if not inc or not (inc / "jni.h").exists():
        pytest.skip("no JDK (jni.h) in this image")
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Werror", f"-I{inc}", f"-I{inc / 'linux'}",
                        f"-I{ROOT / 'include'}", str(SHIM)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
