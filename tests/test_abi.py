"""CPU: the C-ABI library loads and exports every symbol include/geohip.h declares;
contexts fail loudly (no silent CPU path) where no device exists."""
import re
import subprocess
from pathlib import Path

import pytest

from spatialflink_amd import _abi

ROOT = Path(__file__).resolve().parents[1]


def header_symbols():
    text = (ROOT / "include" / "geohip.h").read_text()
    return sorted(set(re.findall(r"\b(geohip_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", str(_abi.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (geohip_\w+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_abi.HEADER_SYMBOLS) == header_symbols()


def test_version():
    assert "gfx950" in _abi.version()


def test_no_device_fails_loudly():
    if _abi.device_count() > 0:
        pytest.skip("a device is present")
    with pytest.raises(_abi.GeohipDeviceError):
        _abi.Context(0)


def test_oracle_not_imported_by_product():
    for f in (ROOT / "spatialflink_amd").rglob("*.py"):
        src = f.read_text()
        assert "cref" not in src and "restate" not in src and "oracle" not in src.replace("oracle/", ""), f
