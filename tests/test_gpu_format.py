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


def _oid_tensors(oids):
    import torch
    enc = [o.encode() for o in oids]
    off = np.zeros(len(enc) + 1, np.int64)
    off[1:] = np.cumsum([len(e) for e in enc])
    text = np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy()
    return torch.from_numpy(text).cuda(), torch.from_numpy(off).cuda()


_ODD_OIDS = ["", "plain", 'q"uote', "back\\slash", "</tag>", "a/b", "tab\there", "nl\nx", "\x01\x1f", "\x7f",
             "\u0080\u0085\u009f ", "  ⃿℀", "café", "\U0001F600 smile", "\b\f\r"]


@pytest.mark.parametrize("delim", [",", "\t", ";", "<->", "é", "\\\\t"])
def test_wkt_records(ctx, delim):
    """PointToWKTOutputSchema (Serialization.java:72-92) byte for byte vs the restatement."""
    import torch
    rng = np.random.default_rng(11)
    n = 3000
    x = _doubles(rng, 400)[:n]
    x = np.concatenate([x, rng.uniform(115.5, 117.6, n - len(x))])
    y = rng.permutation(x)
    ts = rng.integers(-(1 << 40), 1 << 44, n).astype(np.int64)  # 1935 .. 2527
    ts[::5] = 0
    oids = [_ODD_OIDS[i % len(_ODD_OIDS)] + str(i) for i in range(n)]
    toid, toff = _oid_tensors(oids)
    tx, ty, tts = (torch.from_numpy(a).cuda() for a in (x, y, ts))
    idx = rng.permutation(n)[:1001].astype(np.int32)
    sep = "\\t" if delim == "\\\\t" else delim
    for off_min in (0, 480, -300):
        spec = _abi.make_text_out_spec(_abi.FMT_WKT, delimiter=delim, date_format=_abi.DATE_YMD_HMS,
                                       utc_offset_min=off_min)
        for use_idx, with_oid in ((False, True), (True, True), (True, False)):
            text, off = ctx.format_points(spec, tx, ty, tts, toid if with_oid else None, toff if with_oid else None,
                                          torch.from_numpy(idx).cuda() if use_idx else None)
            pts = idx.tolist() if use_idx else range(n)
            want = "".join(J.format_point_wkt(oids[p] if with_oid else None, int(ts[p]), float(x[p]), float(y[p]), sep,
                                              off_min) + "\n" for p in pts)
            assert bytes(text.cpu().numpy()).decode() == want
            assert int(off[-1]) == len(want.encode())


def test_geojson_records(ctx):
    """PointToGeoJSONOutputSchema (Serialization.java:28-50) with org.json's HashMap key order,
    numberToString and quote, byte for byte vs the restatement."""
    import torch
    rng = np.random.default_rng(12)
    v = _doubles(rng, 4000)
    v = v[np.isfinite(v)]
    n = len(v)
    x, y = v, rng.permutation(v)
    ts = rng.integers(-(1 << 40), 1 << 44, n).astype(np.int64)
    ts[::3] = 0
    oids = [_ODD_OIDS[i % len(_ODD_OIDS)] + ("" if i % 7 else str(i)) for i in range(n)]
    toid, toff = _oid_tensors(oids)
    tx, ty, tts = (torch.from_numpy(a).cuda() for a in (x, y, ts))
    for off_min, with_oid, with_ts in ((0, True, True), (330, True, True), (0, False, True), (0, False, False)):
        spec = _abi.make_text_out_spec(_abi.FMT_GEOJSON, date_format=_abi.DATE_YMD_HMS, utc_offset_min=off_min)
        text, off = ctx.format_points(spec, tx, ty, tts if with_ts else None, toid if with_oid else None,
                                      toff if with_oid else None)
        got = bytes(text.cpu().numpy()).decode().split("\n")[:-1]
        assert len(got) == n
        for p in range(n):
            want = J.format_point_geojson(oids[p] if with_oid else None, int(ts[p]) if with_ts else 0, float(x[p]),
                                          float(y[p]), off_min)
            assert got[p] == want, (p, got[p], want)


def test_codec_errors_where_the_reference_throws(ctx):
    import torch
    x = torch.tensor([116.0, math.nan, 117.0], dtype=torch.float64, device="cuda")
    y = torch.tensor([40.0, 40.5, math.inf], dtype=torch.float64, device="cuda")
    gj = _abi.make_text_out_spec(_abi.FMT_GEOJSON)
    with pytest.raises(_abi.GeohipArgumentError):  # JSONObject.toString -> null -> NPE
        ctx.format_points(gj, x, y)
    text, _ = ctx.format_points(gj, x, y, idx=torch.tensor([0], dtype=torch.int32, device="cuda"))
    assert bytes(text.cpu().numpy()).decode() == '{"geometry":{"coordinates":[116,40],"type":"Point"},"type":"Feature"}\n'
    # a padded kNN list (sentinel -1 = 0xffffffff) names no point
    csv = _abi.make_csv_out_spec()
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.format_points_csv(csv, x, y, idx=torch.tensor([0, -1], dtype=torch.int32, device="cuda"))
    with pytest.raises(_abi.GeohipArgumentError):
        ctx.format_points(_abi.make_text_out_spec(_abi.FMT_WKT), x, y, idx=torch.tensor([3], dtype=torch.int32,
                                                                                         device="cuda"))
    # a nonzero timestamp without the caller's DateFormat, or outside the supported years
    ts = torch.tensor([0, 1, 0], dtype=torch.int64, device="cuda")
    with pytest.raises(_abi.GeohipUnsupportedError):
        ctx.format_points(_abi.make_text_out_spec(_abi.FMT_WKT), x, y, ts)
    far = torch.tensor([0, 1 << 60, 0], dtype=torch.int64, device="cuda")
    with pytest.raises(_abi.GeohipUnsupportedError):
        ctx.format_points(_abi.make_text_out_spec(_abi.FMT_WKT, date_format=_abi.DATE_YMD_HMS), x, y, far)
    # the CSV codec never formats dates: its timestamps are Long.toString
    text, _ = ctx.format_points(_abi.make_text_out_spec(_abi.FMT_CSV), x, y, far)
    assert bytes(text.cpu().numpy()).decode().split("\n")[1] == "null,%d,NaN,40.5" % (1 << 60)


@pytest.mark.parametrize("delim", ["é", "€", "\U0001F600", "a\U0001F600", "\\\\t"])
def test_csv_multibyte_delimiter_delete_char(ctx, delim):
    """deleteCharAt(length - 1) drops one UTF-16 unit of the last delimiter: the whole of a BMP
    character, the low half of a supplementary one (its high half is written as '?')."""
    import torch
    x = torch.tensor([116.5, 117.25], dtype=torch.float64, device="cuda")
    y = torch.tensor([40.0, 39.75], dtype=torch.float64, device="cuda")
    spec = _abi.make_csv_out_spec((0, 1, 2, 3), delim)
    text, _ = ctx.format_points_csv(spec, x, y)
    sep = "\\t" if delim == "\\\\t" else delim
    want = "".join(J.format_point_csv(None, 0, float(a), float(b), (0, 1, 2, 3), sep) + "\n"
                   for a, b in ((116.5, 40.0), (117.25, 39.75)))
    assert bytes(text.cpu().numpy()).decode() == want
