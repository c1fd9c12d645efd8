"""Ingest codec: CPU checks of the oracle and of the device parser.

The device record parser (spatialflink_amd/csrc/ingest_parse.h) is __host__ __device__ code;
``_abi.debug_ingest_record`` runs the same functions host-compiled, so these tests check its
decisions without a GPU.  The kernels that split a batch into records and run the parser per
lane are checked on the GPU by tests/test_gpu_ingest.py.

Known answers are derived by hand from the Java code (paths relative to
/root/reference/src/main/java/GeoFlink): CSVTSVToSpatial / CSVTSVToTSpatial
spatialStreams/Deserialization.java:248-254, 306-321 (quote removal, split on \\s*d\\s*,
Double.valueOf / Long.valueOf); GeoJSONToSpatial :132-146; WKTToSpatial :223-228, :1510-1514.
The reference holds no deserializer fixtures, so parity of the grammar corners is unpinned
beyond these hand-derived answers (Parity).
"""
from __future__ import annotations

import math
import random
import struct
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import cref  # noqa: E402  (oracle: the checker)
from spatialflink_amd import _abi  # noqa: E402

NAN = float("nan")
INF = float("inf")

# ATC-style CSVTSVToTSpatial schema: [oid, ts, x, y] -> csvTsvSchemaAttr = [0, 1, 2, 3]
CSV_T = ("csv", ",", 2, 3, 1)
CSV = ("csv", ",", 2, 3, -1)
TSV = ("csv", "\t", 0, 1, -1)
WKT = ("wkt", ",", 0, 1, -1)
GEO = ("geojson", ",", 0, 1, -1)
_FMT = {"csv": cref.CSV, "geojson": cref.GEOJSON, "wkt": cref.WKT}

# (spec, record, expected (x, y, ts) or None where the reference throws, device-may-reject)
# device-may-reject: valid Java input outside the device grammar (the batch call then returns
# GEOHIP_ERR_UNSUPPORTED and the caller hands the batch to the reference deserializer).
KNOWN = [
    (CSV_T, b"7,1611022449423,116.4148990000001,39.92037412345", (116.4148990000001, 39.92037412345, 1611022449423), False),
    (CSV_T, b'"7","1611022449423","116.5","39.75"', (116.5, 39.75, 1611022449423), False),
    (CSV_T, b"7 , 12 , 116.5 , 39.75", (116.5, 39.75, 12), False),
    (CSV_T, b"7,12,116.5", None, False),  # get(3): IndexOutOfBoundsException
    (CSV_T, b"7,12,116.5,abc", None, False),  # NumberFormatException
    (CSV_T, b"7,12,1e3,-2.5E-1", (1000.0, -0.25, 12), False),
    (CSV_T, b"7,12,+1.5d,2f", (1.5, 2.0, 12), False),  # Java type suffixes
    (CSV_T, b"7,12,NaN,-Infinity", (NAN, -INF, 12), False),
    (CSV_T, b"7,12,.5,5.", (0.5, 5.0, 12), False),
    (CSV_T, b"7,12,.,1", None, False),
    (CSV_T, b"7,12,1e,1", None, False),
    (CSV_T, b"7,12,nan,1", None, False),  # NaN is case-sensitive
    (CSV_T, b"7,12,1.5\x01,2", (1.5, 2.0, 12), False),  # Double.valueOf trims every char <= ' '
    (CSV_T, b"7,+12,1,2", (1.0, 2.0, 12), False),
    (CSV_T, b"7,12.0,1,2", None, False),  # Long.valueOf
    (CSV_T, b"7, 12\x01,1,2", None, False),  # Long.valueOf does not trim
    (CSV_T, b"7,9223372036854775808,1,2", None, False),  # Long overflow
    (CSV_T, b"7,-9223372036854775808,1,2", (1.0, 2.0, -9223372036854775808), False),
    (CSV_T, b"7,9223372036854775807,1,2", (1.0, 2.0, 9223372036854775807), False),
    (CSV_T, b"7,12,0x1.8p1,2", (3.0, 2.0, 12), False),  # hex significand
    (CSV_T, b"7,12,-0X.8P-1d,0x1p-1074", (-0.25, 5e-324, 12), False),
    (CSV_T, b"7,12,0x1p-1075,0x1.0000000000001p-1075", (0.0, 5e-324, 12), False),  # tie to even / just above
    (CSV_T, b"7,12,0x1.fffffffffffff8p1023,0x1p99999999999", (INF, INF, 12), False),  # rounds past MAX / int range
    (CSV_T, b"7,12,0x0.0p5,-0x1p-99999999999", (0.0, -0.0, 12), False),
    (CSV_T, b"7,12,0x1.00000000000008p0,0x1.00000000000018p0", (1.0, 1.0000000000000004, 12), False),  # ties
    (CSV_T, b"7,12,0x123456789abcdef0123p-70,2", (float.fromhex("0x123456789abcdef0123p-70"), 2.0, 12), False),
    (CSV_T, b"7,12,0xp1,2", None, False),
    (CSV_T, b"7,12,0x1.8p,2", None, False),
    (CSV_T, b"7,12,0x1.8,2", None, False),  # hex needs a binary exponent
    (CSV_T, b"7,12,1.5,2,extra", (1.5, 2.0, 12), False),
    (CSV_T, b",12,1,2", (1.0, 2.0, 12), False),  # leading "" field
    (CSV_T, b"7,12,0.1,0.30000000000000004", (0.1, 0.30000000000000004, 12), False),
    (CSV_T, b"7,12,9007199254740993,2", (9007199254740992.0, 2.0, 12), False),  # tie -> even
    (CSV_T, b"7,12,1.000000000000000000000001,2", (1.0, 2.0, 12), False),  # 25 digits, decided by truncation
    (CSV_T, b"7,12,2.2250738585072011e-308,4.9e-324", (2.225073858507201e-308, 5e-324, 12), False),
    (CSV_T, b"7,12,1e400,1e-400", (INF, 0.0, 12), False),
    (CSV_T, b"7,12,-0.0,0", (-0.0, 0.0, 12), False),
    (CSV_T, b"7,12,1e1000000,2", (INF, 2.0, 12), False),  # 7-digit exponent
    (CSV_T, b"7,12,1e-99999999999999,0e99999999999", (0.0, 0.0, 12), False),
    (CSV_T, b"7,12,-0.001e1000000002,2", (-INF, 2.0, 12), False),
    (CSV_T, b'7,12,1"5,2', (15.0, 2.0, 12), False),  # quotes deleted inside a token
    (CSV_T, b'7,1"2,-"1".5"e1,2', (-15.0, 2.0, 12), False),
    (CSV_T, b"7,12,1 5,2", None, False),
    (CSV, b"a,b,116.5,39.75", (116.5, 39.75, 0), False),
    (CSV, b"a,b,116.5,", None, False),  # trailing "" removed -> get(3) throws
    (CSV, b"a,b,116.5,\t", None, False),
    (TSV, b"116.5\t39.75", (116.5, 39.75, 0), False),
    (TSV, b"116.5 \t 39.75", (116.5, 39.75, 0), False),
    (TSV, b"116.5 39.75", None, False),  # no tab: one field
    (TSV, b" 116.5\t39.75 ", (116.5, 39.75, 0), False),
    (TSV, b'116.5"\t"39.75', (116.5, 39.75, 0), False),
    (WKT, b"POINT (116.5 39.75)", (116.5, 39.75, 0), False),
    (WKT, b"POINT(116.5 39.75)", (116.5, 39.75, 0), False),
    (WKT, b"id,POINT ( 116.5   39.75 ) trailing", (116.5, 39.75, 0), False),
    (WKT, b"POINT (116.5,39.75)", None, False),
    (WKT, b"POINT EMPTY", None, False),
    (WKT, b"MULTIPOINT ((1 2))", None, False),
    (WKT, b"POINT (1 2 3)", (1.0, 2.0, 0), False),
    (WKT, b"POINT (nan NaN 0x1p4)", (NAN, NAN, 0), False),  # WKTReader: NaN ignoring case
    (WKT, b"POINT (1 2 3 4)", None, False),
    (WKT, b"POINT (1 2 x)", None, False),
    (WKT, b"POINT (1.5d -2e1)", (1.5, -20.0, 0), False),
    (WKT, b"point (1 2)", None, False),
    (WKT, b"POINTZ (1 2)", None, False),
    (GEO, b'{"geometry":{"coordinates":[116.44412,39.93984],"type":"Point"},"properties":{"oID":"2560",'
          b'"timestamp":"2008-02-02 20:12:32"},"type":"Feature"}', (116.44412, 39.93984, 0), False),
    (GEO, b'{"type":"Point","coordinates":[1,2]}', (1.0, 2.0, 0), False),
    (GEO, b'{"type":"Point","coordinates":[ -0 , 2.5e-1 ]}', (0.0, 0.25, 0), False),  # IntNode 0
    (GEO, b'{"type":"Point","coordinates":[-0.0,1]}', (-0.0, 1.0, 0), False),
    (GEO, b'{"type":"Point","coordinates":[01,2]}', None, False),
    (GEO, b'{"type":"Point","coordinates":[+1,2]}', None, False),
    (GEO, b'{"type":"Point","coordinates":[1.,2]}', None, False),
    (GEO, b'{"type":"LineString","coordinates":[[1,2],[3,4]]}', (1.0, 2.0, 0), False),
    (GEO, b'{"type":"Point","coordinates":[1e400,2]}', None, False),
    (GEO, b'{"type":"Point","coordinates":[9223372036854775807,-9223372036854775808]}',
     (9.223372036854776e18, -9.223372036854776e18, 0), False),  # LongNode
    (GEO, b'{"type":"Point","coordinates":[9223372036854775808,1]}', None, False),  # BigIntegerNode
]


def _spec_oracle(s):
    return cref.ingest_spec(_FMT[s[0]], s[1], s[2], s[3], s[4])


def _spec_dev(s):
    return _abi.make_ingest_spec(_FMT[s[0]], s[1], s[2], s[3], s[4])


def _bits(v):
    return struct.pack("<d", v)


def _same(a, b):
    return _bits(a) == _bits(b) or (math.isnan(a) and math.isnan(b))


@pytest.mark.parametrize("spec,rec,want,may_reject", KNOWN)
def test_oracle_known_answers(spec, rec, want, may_reject):
    got = cref.ingest_record(_spec_oracle(spec), rec)
    if want is None:
        assert got is None
    else:
        assert got is not None and _same(got[0], want[0]) and _same(got[1], want[1]) and got[2] == want[2]


@pytest.mark.parametrize("spec,rec,want,may_reject", KNOWN)
def test_device_parser_known_answers(spec, rec, want, may_reject):
    got = _abi.debug_ingest_record(_spec_dev(spec), rec)
    if want is None:
        assert got is None
    elif got is None:
        assert may_reject, "device parser rejected a record it must decide"
    else:
        assert _same(got[0], want[0]) and _same(got[1], want[1]) and got[2] == want[2]


def _rand_decimal(rng: random.Random) -> str:
    nint = rng.choice([0, 1, 1, 2, 3, 5, 10, 17, 20])
    nfrac = rng.choice([0, 1, 2, 5, 10, 13, 16, 17, 19, 22])
    if nint + nfrac == 0:
        nint = 1
    ip = "".join(rng.choice("0123456789") for _ in range(nint))
    fp = "".join(rng.choice("0123456789") for _ in range(nfrac))
    s = ip + ("." + fp if nfrac or rng.random() < 0.1 else "")
    if rng.random() < 0.4:
        s += rng.choice("eE") + rng.choice(["", "+", "-"]) + str(rng.choice([0, 1, 5, 22, 23, 100, 290, 300, 307, 308,
                                                                                  309, 320, 324, 330, 340, 350]))
    if rng.random() < 0.3:
        s = rng.choice("+-") + s
    return s


def test_decimal_conversion_fuzz():
    """Random decimal tokens: device parser == oracle == Python float (all correctly rounded)."""
    rng = random.Random(20260116)
    spec_d, spec_o = _spec_dev(TSV), _spec_oracle(TSV)
    rejected = 0
    n = 20000
    for _ in range(n):
        a, b = _rand_decimal(rng), _rand_decimal(rng)
        rec = f"{a}\t{b}".encode()
        want = (float(a), float(b))
        o = cref.ingest_record(spec_o, rec)
        assert o is not None and _same(o[0], want[0]) and _same(o[1], want[1]), rec
        d = _abi.debug_ingest_record(spec_d, rec)
        if d is None:
            rejected += 1
            sig = [len(t.lstrip("+-").split("e")[0].split("E")[0].replace(".", "").lstrip("0")) for t in (a, b)]
            assert max(sig) > 19, f"rejected a token of <= 19 significant digits: {rec}"
            continue
        assert _same(d[0], want[0]) and _same(d[1], want[1]), rec
    assert rejected < n // 100


def test_decimal_halfway_cases():
    """Points at (and 1e-35 relative around) the midpoint of adjacent doubles, written with 17-41
    significant digits: where the device parser decides, it matches Python's correctly rounded float."""
    from decimal import Decimal, getcontext
    getcontext().prec = 80
    rng = np.random.default_rng(7)
    spec_d = _spec_dev(TSV)
    vals = rng.uniform(-1e3, 1e3, 300).tolist() + [1.0, 0.1, 116.41, 39.92, 5e-324, 1e300, 2.0 ** -1022]
    decided = 0
    for v in vals:
        mid = (Decimal(v) + Decimal(float(np.nextafter(v, np.inf)))) / 2
        for t in (mid, mid * (1 + Decimal(10) ** -35), mid * (1 - Decimal(10) ** -35)):
            for digits in (16, 17, 20, 40):
                s = format(t, f".{digits}e")
                d = _abi.debug_ingest_record(spec_d, f"{s}\t1".encode())
                if d is not None:
                    decided += 1
                    assert _same(d[0], float(s)), s
                else:
                    assert digits + 1 > 19, s
    assert decided > len(vals) * 6


def _noise(rng, chars=" \t\""):
    return "".join(rng.choice(chars) for _ in range(rng.choice([0, 0, 0, 1, 2])))


def test_csv_shape_fuzz():
    """Random spaces, tabs, quotes and control characters around fields: the device parser either
    agrees bit-exactly with the oracle or rejects; it never accepts what the reference rejects."""
    rng = random.Random(99)
    for delim in (",", ";", "\t", " "):
        spec = ("csv", delim, 2, 3, 1)
        sd, so = _spec_dev(spec), _spec_oracle(spec)
        accepted = 0
        for _ in range(4000):
            nf = rng.choice([3, 4, 4, 4, 5])
            fields = []
            for f in range(nf):
                v = rng.choice(["12", "-7", "+3", "1.5", "116.4148990000001", "x", "", "1e5", "0.30000000000000004",
                                "NaN", "2.5d", "1 2", "16\x01"]) if f else rng.choice(["a", "7", "", " q"])
                fields.append(_noise(rng) + v + _noise(rng))
            sep = [rng.choice([delim, " " + delim, delim + " ", '"' + delim + '"', delim + delim])
                   for _ in range(nf - 1)]
            rec = fields[0] + "".join(s + f for s, f in zip(sep, fields[1:]))
            rec = rec.encode()
            o = cref.ingest_record(so, rec)
            d = _abi.debug_ingest_record(sd, rec)
            if o is None:
                assert d is None, (delim, rec, d)
            elif d is not None:
                accepted += 1
                assert _same(d[0], o[0]) and _same(d[1], o[1]) and d[2] == o[2], (delim, rec, d, o)
        assert accepted > 200, delim


def test_oracle_batch_framing():
    spec = _spec_oracle(CSV)
    one = cref.ingest(spec, b"a,b,1,2")
    assert one["x"].tolist() == [1.0]
    two = cref.ingest(spec, b"a,b,1,2\na,b,3,4\n")  # a trailing '\n' ends the last record
    assert two["y"].tolist() == [2.0, 4.0]
    assert len(cref.ingest(spec, b"")["x"]) == 0
    with pytest.raises(cref.IngestRejected) as e:
        cref.ingest(spec, b"a,b,1,2\n\na,b,3,4")  # an empty line is a record: get(2) throws
    assert e.value.bad == 1


def test_oracle_cell_assignment():
    """Point(x, y, uGrid) -> HelperClass.assignGridCellID (HelperClass.java:104-116)."""
    g = cref.grid(115.5, 39.6, (117.6 - 115.5) / 100, 100)
    got = cref.ingest_record(_spec_oracle(WKT), b"POINT (116.414899 39.920374)", g)
    cx, cy = cref.cell(g, 116.414899, 39.920374)
    assert (cx, cy) == (43, 15)  # the README query cell
    assert got[3] == 43 * 100 + 15
    assert cref.ingest_record(_spec_oracle(WKT), b"POINT (117.6 39.7)", g)[3] == 0xFFFFFFFF  # cx == n
    assert cref.ingest_record(_spec_oracle(WKT), b"POINT (NaN 39.7)", g)[3] == 0 * 100 + 4  # (int)NaN == 0


def test_spec_validation():
    with pytest.raises(_abi.GeohipArgumentError):
        _abi.debug_ingest_record(_abi.make_ingest_spec(cref.CSV, "|", 0, 1), b"1|2")  # regex metacharacter
    with pytest.raises(_abi.GeohipArgumentError):
        _abi.debug_ingest_record(_abi.make_ingest_spec(cref.CSV, ",", -1, 1), b"1,2")


def test_hex_and_long_exponent_fuzz():
    """Random hex significands (Double.parseDouble's parseHexString grammar) and decimal tokens with
    long exponents: device parser == oracle (glibc strtod, correctly rounded) == Python."""
    rng = random.Random(424242)
    spec_d, spec_o = _spec_dev(TSV), _spec_oracle(TSV)
    for _ in range(20000):
        toks = []
        for _t in range(2):
            if rng.random() < 0.7:
                ih = "".join(rng.choice("0123456789abcdefABCDEF") for _ in range(rng.choice([0, 1, 2, 7, 14, 16, 20])))
                fh = "".join(rng.choice("0123456789abcdef") for _ in range(rng.choice([0, 1, 3, 13, 15, 20])))
                if not ih and not fh:
                    ih = "1"
                body = ih + ("." + fh if fh or rng.random() < 0.2 else "")
                ex = rng.choice([0, 1, -1, 52, -1022, -1074, -1075, -1080, 1023, 1024, -1100, 900, -990,
                                 rng.randint(-1200, 1200)])
                t = rng.choice(["", "-", "+"]) + rng.choice(["0x", "0X"]) + body + rng.choice("pP") + str(ex)
                t += rng.choice(["", "", "d", "F"])
                try:
                    want = float.fromhex(t.rstrip("dF"))
                except OverflowError:
                    want = -INF if t.startswith("-") else INF
            else:
                m = rng.choice(["1", "0", "0.0", "7.25", "123456789", "0.000001"])
                e = rng.choice([1000000, 99999999, 123456789012, -1000000, -99999999999])
                t = rng.choice(["", "-"]) + m + "e" + str(e)
                want = float(t)
            toks.append((t, want))
        rec = f"{toks[0][0]}\t{toks[1][0]}".encode()
        o = cref.ingest_record(spec_o, rec)
        d = _abi.debug_ingest_record(spec_d, rec)
        assert o is not None and d is not None, rec
        for k in range(2):
            assert _same(o[k], toks[k][1]) and _same(d[k], toks[k][1]), (rec, o, d)
