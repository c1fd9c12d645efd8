"""Build libgeohip.so in-tree for gfx950 with hipcc (no JIT cache, no CMake).

``python -m spatialflink_amd.build`` or ``__graft_entry__.build()``.  Objects go to
``build/geohip/``; the shared library lands next to this file so it travels with the
repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = ROOT / "build" / "geohip"
LIB = PKG / "libgeohip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GEOHIP_ARCH", "gfx950")

# -ffp-contract=off: the reference evaluates fp64 in Java source order without FMA contraction.
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall",
          "-Wno-unused-function", f"-I{ROOT / 'include'}"]

SOURCES = {
    "plan.cpp": ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"],
    "abi.cpp": ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"],
    "ingest_abi.cpp": ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"],
    "pp_kernels.hip": ["-x", "hip", f"--offload-arch={ARCH}"],
    "cell_kernels.hip": ["-x", "hip", f"--offload-arch={ARCH}"],
    "ingest.hip": ["-x", "hip", f"--offload-arch={ARCH}"],
    "band.hip": ["-x", "hip", f"--offload-arch={ARCH}"],
    "format.hip": ["-x", "hip", f"--offload-arch={ARCH}"],
    "sort.hip": ["-x", "hip", f"--offload-arch={ARCH}"],
}


def _compile(src: str, extra: list[str]) -> Path:
    out = OBJ / (src + ".o")
    s = CSRC / src
    deps = [s] + list(CSRC.glob("*.h")) + [ROOT / "include" / "geohip.h"]
    if out.exists() and all(out.stat().st_mtime >= d.stat().st_mtime for d in deps):
        return out
    cmd = [HIPCC, *COMMON, *extra, "-c", str(s), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return out


def build(verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda kv: _compile(*kv), SOURCES.items()))
    newest = max(o.stat().st_mtime for o in objs)
    if not LIB.exists() or LIB.stat().st_mtime < newest:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(LIB)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
