"""GPU: the point CSV/TSV output codec (geohip_format_points_csv, SURVEY.md 8(f) row 4;
Serialization.PointToCSVTSVOutputSchema, Serialization.java:98-152) byte for byte against the
CPU restatement oracle/jdk_double.py (JDK 8 FloatingDecimal Double.toString; parity unpinned:
no JVM runs here).  Doubles of every path -- the int, long and big-integer digit loops, the
integer fast path, subnormals, powers of ten, the JDK-4511638 anomalies, NaN / infinities /
signed zeros -- and records with objIDs, timestamps, schema gaps, shared positions, multi-byte
delimiters and an index subset."""
import math
import struct

import numpy as np
import pytest

import jdk_double as J
from spatialflink_amd import _abi

pytestmark = pytest.mark.gpu


def _doubles(rng, n):
    bits = rng.integers(0, 1 << 63, n, dtype=np.uint64) * 2 + rng.integers(0, 2, n, dtype=np.uint64)
    rand = bits.view(np.float64)
    coords = np.concatenate([rng.uniform(115.5, 117.6, n // 4), rng.uniform(39.6, 41.1, n // 4)])
    rounded = np.round(coords, rng.integers(0, 14))
    ints = rng.integers(-(1 << 62), 1 << 62, n // 8).astype(np.float64)
    small_ints = rng.integers(-100000, 100000, n // 8).astype(np.float64)
    pow10 = np.array([10.0 ** e for e in range(-320, 309)])
    special = np.array([0.0, -0.0, math.nan, math.inf, -math.inf, 5e-324, 2.2250738585072014e-308,
                        1.7976931348623157e308, 1e23, 2e23, 0.1, 1 / 3, 2.0 ** 53, 2.0 ** 63, 9007199254740993.0,
                        1e-7, 1e-3, 1e7, 123456789.0, 4.35, 0.5, -1.5])
    sub = (rng.integers(1, 1 << 52, n // 8, dtype=np.uint64)).view(np.float64)
    return np.concatenate([rand, coords, rounded, ints, small_ints, pow10, special, sub])


def test_double_to_string_all_paths(ctx):
    import torch
    rng = np.random.default_rng(3)
    v = _doubles(rng, 40000)
    x = torch.from_numpy(v).cuda()
    spec = _abi.make_csv_out_spec((5, 6, 0, 7), ",")  # x alone at position 0; "0" fields between
    text, off = ctx.format_points_csv(spec, x, x)
    got = bytes(text.cpu().numpy()).decode().split("\n")[:-1]
    assert len(got) == len(v)
    for d, g in zip(v.tolist(), got):
        want = J.format_point_csv(None, 0, d, d, (5, 6, 0, 7), ",")
        assert g == want, (repr(d), g, want)


def test_csv_records_fields_and_subsets(ctx):
    import torch
    rng = np.random.default_rng(4)
    n = 5000
    x = rng.uniform(115.5, 117.6, n)
    y = rng.uniform(39.6, 41.1, n)
    x[::97] = np.round(x[::97], 4)
    ts = rng.integers(0, 1 << 45, n).astype(np.int64)
    ts[::13] = -ts[::13]
    oids = [str(i * 7919) if i % 11 else "id-" + str(i) for i in range(n)]
    oid_bytes = "".join(oids).encode()
    oid_off = np.zeros(n + 1, np.int64)
    oid_off[1:] = np.cumsum([len(o) for o in oids])
    tx, ty, tts = (torch.from_numpy(a).cuda() for a in (x, y, ts))
    ttext = torch.from_numpy(np.frombuffer(oid_bytes, np.uint8).copy()).cuda()
    toff = torch.from_numpy(oid_off).cuda()
    idx = rng.permutation(n)[:1777].astype(np.int32)
    tidx = torch.from_numpy(idx).cuda()
    for attrs, delim in (((0, 1, 2, 3), ","), ((3, 0, 1, 2), "\t"), ((0, 2, 4, 6), ";"), ((0, 1, 2, 2), "|"),
                         ((1, 0, 3, 5), "<->")):
        spec = _abi.make_csv_out_spec(attrs, delim)
        for use_idx in (False, True):
            text, off = ctx.format_points_csv(spec, tx, ty, tts, ttext, toff, tidx if use_idx else None)
            pts = idx.tolist() if use_idx else list(range(n))
            want = "".join(J.format_point_csv(oids[p], int(ts[p]), float(x[p]), float(y[p]), attrs, delim) + "\n"
                           for p in pts)
            assert bytes(text.cpu().numpy()).decode() == want
            o = off.cpu().numpy()
            assert o[0] == 0 and o[-1] == len(want.encode())
    # no objID column: "null"; capacity too small reports the size
    spec = _abi.make_csv_out_spec((0, 1, 2, 3), ",")
    text, _ = ctx.format_points_csv(spec, tx[:3], ty[:3])
    assert bytes(text.cpu().numpy()).decode().split("\n")[0].startswith("null,0,")
    with pytest.raises(_abi.GeohipCapacityError):
        ctx.format_points_csv(spec, tx, ty, cap=100)
