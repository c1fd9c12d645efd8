"""TrajectoryStream ingest (SURVEY.md 8(f) row 1 remainder): the Point's objID and GeoJSON timestamp.

CPU checks of the device parser (ingest_parse.h, run host-compiled through
``_abi.debug_ingest_traj_record``) against the independent C restatement
(oracle/ingest_oracle.c, ``cref.ingest_traj``), record by record: both reject, or both give the
same x / y bits, timestamp and objID bytes (null included).  Reference (paths relative to
/root/reference/src/main/java/GeoFlink):

  CSVTSVToTSpatial.map   spatialStreams/Deserialization.java:306-321
      strOId = split(str.replace("\\"", ""), "\\s*" + d + "\\s*").get(csvTsvSchemaAttr.get(0))
  GeoJSONToTSpatial.map  spatialStreams/Deserialization.java:149-208
      time = dateFormat.parse(properties[propertyTimeStamp].textValue()).getTime() (0 on ParseException)
      strOId = properties[propertyObjID].toString().replaceAll("\\"", "")  (null when absent)
  Point(objID, x, y, timeStampMillisec, uGrid)   spatialObjects/Point.java:91-100

The date known answers are derived by hand (UTC epoch arithmetic); the DateFormat is
conf/geoflink-conf.yml's "yyyy-MM-dd HH:mm:ss".  Parity unpinned beyond them (no JVM here).
"""
from __future__ import annotations

import random
import struct
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import cref  # noqa: E402  (oracle: the checker)
from spatialflink_amd import _abi  # noqa: E402


def _bits(v):
    return struct.unpack("<Q", struct.pack("<d", v))[0]


def _device(spec, traj, rec):
    r = _abi.debug_ingest_traj_record(spec, traj, rec)
    if r is None:
        return None
    x, y, ts, span = r
    return x, y, ts, _abi.oid_spans_to_strings(rec, [span])[0]


def _oracle(spec, traj, rec):
    try:
        o = cref.ingest_traj(spec, traj, rec)
    except cref.IngestRejected:
        return None
    oid = o["oid"][0]
    return float(o["x"][0]), float(o["y"][0]), int(o["ts"][0]), None if oid is None else oid.decode()


def _same(a, b):
    if a is None or b is None:
        return a is None and b is None
    return _bits(a[0]) == _bits(b[0]) and _bits(a[1]) == _bits(b[1]) and a[2] == b[2] and a[3] == b[3]


# ---- known answers (hand-derived from the Java lines) -------------------------------------
CSV_SPEC = dict(fmt=0, delim=",", fx=2, fy=3, fts=1, foid=0)
DAY = 86400000


@pytest.mark.parametrize("rec,oid", [
    (b"abc,1611,116.5,39.9", "abc"),
    (b'  ab"c" , 12,116.5,39.9', "  abc"),      # field 0 keeps its leading \s; quotes deleted
    (b'"7","12","116.5","39.75"', "7"),
    (b"id 7 ,1,2,3", "id 7"),                    # \s before the delimiter: part of the separator
    (b"a b\tc,1,2,3", "a b\tc"),
    (b",1,2,3", None),                           # "" objID: valid Java, handed back to the host
])
def test_csv_objid_known(rec, oid):
    sp_d = _abi.make_ingest_spec(0, ",", 2, 3, 1, 0)
    sp_o = cref.ingest_spec(0, ",", 2, 3, 1, 0)
    got, want = _device(sp_d, None, rec), _oracle(sp_o, None, rec)
    if oid is None:
        assert got is None and want is None
    else:
        assert got is not None and got[3] == oid and _same(got, want)


def test_csv_objid_last_field_keeps_trailing_blanks():
    sp_d = _abi.make_ingest_spec(0, ",", 2, 3, 1, 4)
    sp_o = cref.ingest_spec(0, ",", 2, 3, 1, 4)
    rec = b"a,1,2,3,  last one  "
    got = _device(sp_d, None, rec)
    assert got[3] == "last one  " and _same(got, _oracle(sp_o, None, rec))
    assert _device(sp_d, None, b"a,1,2,3,   ") is None and _oracle(sp_o, None, b"a,1,2,3,   ") is None


GJ = b'{"type":"Feature","geometry":{"type":"Point","coordinates":[116.5,39.9]}%s}'


@pytest.mark.parametrize("props,ts,oid", [
    (b',"properties":{"oID":"abc","timestamp":"2020-01-02 03:04:05"}', 1577934245000, "abc"),
    (b',"properties":{"oID":123,"timestamp":"1970-01-01 00:00:00"}', 0, "123"),
    (b',"properties":{"oID":-42,"timestamp":"1970-01-02 00:00:00"}', DAY, "-42"),
    (b',"properties":{"oID":true}', 0, "true"),
    (b',"properties":{"oID":null}', 0, "null"),                # NullNode.toString()
    (b'', 0, None),                                            # no properties: objID null
    (b',"properties":{}', 0, None),
    (b',"properties":"x"', 0, None),                           # get() on a text node: null
    (b',"properties":{"timestamp":"garbage"}', 0, None),       # ParseException caught: 0
    (b',"properties":{"timestamp":""}', 0, None),
    (b',"properties":{"timestamp":"  1970-01-01 00:00:10 tail"}', 10000, None),  # blanks, trailing text
    (b',"properties":{"timestamp":"1970-01-32 00:00:00"}', 31 * DAY, None),        # lenient day carry
    (b',"properties":{"timestamp":"1970-13-01 00:00:00"}', 365 * DAY, None),       # lenient month carry
    (b',"properties":{"timestamp":"1970-01-01 24:00:60"}', DAY + 60000, None),
    (b',"properties":{"oID":"a","timestamp":"2020-01-02 03:04:05"},"properties":{"oID":"b"}', 0, "b"),  # last wins
])
def test_geojson_properties_known(props, ts, oid):
    rec = GJ % props
    sp_d, tr_d = _abi.make_ingest_spec(1), _abi.make_traj_spec()
    sp_o, tr_o = cref.ingest_spec(1), cref.traj_spec()
    got, want = _device(sp_d, tr_d, rec), _oracle(sp_o, tr_o, rec)
    assert got is not None and got[2] == ts and got[3] == oid, got
    assert _same(got, want), (got, want)


@pytest.mark.parametrize("props,throws", [
    (b',"properties":{"timestamp":5}', True),                  # textValue() null -> NPE
    (b',"properties":{"timestamp":null}', True),
    (b',"properties":{"timestamp":"2020-1-2 03:04:05"}', False),  # lenient one-digit fields: host
    (b',"properties":{"timestamp":"2020-01-02 03:04:059"}', False),
    (b',"properties":{"oID":1.5}', False),                     # DoubleNode text: host
    (b',"properties":{"oID":-0}', False),
    (b',"properties":{"oID":"a\\"b"}', False),                 # escapes: host
    (b',"properties":{"oID":{"k":1}}', False),
])
def test_geojson_rejections(props, throws):
    rec = GJ % props
    assert _device(_abi.make_ingest_spec(1), _abi.make_traj_spec(), rec) is None
    assert _oracle(cref.ingest_spec(1), cref.traj_spec(), rec) is None


def test_date_offset_and_no_dateformat():
    rec = GJ % b',"properties":{"timestamp":"2020-01-02 03:04:05"}'
    got = _device(_abi.make_ingest_spec(1), _abi.make_traj_spec(utc_offset_min=480), rec)  # UTC+8 (Beijing)
    assert got[2] == 1577934245000 - 8 * 3600000
    assert _same(got, _oracle(cref.ingest_spec(1), cref.traj_spec(utc_offset_min=480), rec))
    none = _device(_abi.make_ingest_spec(1), _abi.make_traj_spec(date_format=0), GJ % b',"properties":{"timestamp":5}')
    assert none is not None and none[2] == 0  # dateFormat == null: the node is never read


# ---- fuzz: device parser == oracle, record by record ---------------------------------------
def _rand_oid(rng):
    k = rng.randrange(10)
    if k == 0:
        return ""
    if k == 1:
        return " " * rng.randrange(1, 3) + "id" + str(rng.randrange(1000))
    if k == 2:
        return "id" + str(rng.randrange(1000)) + " " * rng.randrange(1, 3)
    if k == 3:
        return '"' + str(rng.randrange(10 ** 6)) + '"'
    if k == 4:
        return "a" + '"' + "b c"
    if k == 5:
        return "x\x01y"
    if k == 6:
        return "\t" + str(rng.randrange(99))
    return "".join(rng.choice("abcdefXYZ0123456789-_.") for _ in range(rng.randrange(1, 24)))


def test_csv_objid_fuzz():
    rng = random.Random(7)
    checked = accepted = 0
    for trial in range(4000):
        delim = rng.choice([",", ";", ":", "\t"])
        nf = rng.randrange(4, 7)
        order = list(range(nf))
        rng.shuffle(order)
        foid, fts, fx, fy = order[:4]
        fields = []
        for f in range(nf):
            if f == fx:
                v = f"{rng.uniform(115, 118):.{rng.randrange(1, 15)}f}"
            elif f == fy:
                v = repr(rng.uniform(39, 42))
            elif f == fts:
                v = str(rng.randrange(-10 ** 12, 10 ** 13))
            elif f == foid:
                v = _rand_oid(rng)
            else:
                v = _rand_oid(rng)
            if rng.random() < 0.2:
                v = " " * rng.randrange(3) + v + " " * rng.randrange(3)
            fields.append(v)
        sep = delim if rng.random() < 0.7 else (" " + delim + " ")
        rec = sep.join(fields).encode()
        sp_d = _abi.make_ingest_spec(0, delim, fx, fy, fts, foid)
        sp_o = cref.ingest_spec(0, delim, fx, fy, fts, foid)
        got, want = _device(sp_d, None, rec), _oracle(sp_o, None, rec)
        assert _same(got, want), (rec, got, want)
        checked += 1
        accepted += got is not None
    assert accepted > checked // 3


def _rand_value(rng, depth=0):
    k = rng.randrange(7 if depth < 2 else 5)
    if k == 0:
        return str(rng.randrange(-1000, 1000))
    if k == 1:
        return '"' + "".join(rng.choice("abc xyz09") for _ in range(rng.randrange(8))) + '"'
    if k == 2:
        return rng.choice(["true", "false", "null"])
    if k == 3:
        return repr(rng.uniform(-10, 10))
    if k == 4:
        return '"a\\"b"'
    if k == 5:
        return "[" + ",".join(_rand_value(rng, depth + 1) for _ in range(rng.randrange(3))) + "]"
    return "{" + ",".join(f'"k{i}":{_rand_value(rng, depth + 1)}' for i in range(rng.randrange(3))) + "}"


def _rand_date(rng):
    k = rng.randrange(8)
    y, mo, d, h, mi, s = (rng.randrange(1583, 10000), rng.randrange(100), rng.randrange(100), rng.randrange(100),
                          rng.randrange(100), rng.randrange(100))
    if k < 4:
        return f'"{y:04d}-{mo:02d}-{d:02d} {h:02d}:{mi:02d}:{s:02d}"'
    if k == 4:
        return f'"{rng.choice(["", " ", "x", "abc", "+1", "-5", "N/A"])}"'
    if k == 5:
        return f'"{y}-{mo}-{d} {h}:{mi}:{s}"'
    if k == 6:
        return f'"{y:04d}-{mo:02d}-{d:02d} {h:02d}:{mi:02d}:{s:02d}{rng.choice(["", "Z", ".5", " tail", "9"])}"'
    return _rand_value(rng)


def test_geojson_traj_fuzz():
    rng = random.Random(11)
    accepted = 0
    for trial in range(3000):
        members = [f'"type":"Feature"',
                   f'"geometry":{{"type":"Point","coordinates":[{rng.uniform(115, 118)!r},{rng.uniform(39, 42)!r}]}}']
        if rng.random() < 0.85:
            props = []
            if rng.random() < 0.8:
                v = _rand_value(rng) if rng.random() < 0.4 else rng.choice(['"v1"', "17", '""'])
                props.append('"oID":' + v)
            if rng.random() < 0.8:
                props.append(f'"timestamp":{_rand_date(rng)}')
            for i in range(rng.randrange(3)):
                props.append(f'"p{i}":{_rand_value(rng)}')
            rng.shuffle(props)
            members.append('"properties":{' + ",".join(props) + "}")
        if rng.random() < 0.2:
            members.append(f'"id":{_rand_value(rng)}')
        rng.shuffle(members)
        ws = rng.choice(["", " "])
        rec = ("{" + ws + ("," + ws).join(members) + ws + "}").encode()
        off = rng.choice([0, 0, 480, -300])
        sp_d, tr_d = _abi.make_ingest_spec(1), _abi.make_traj_spec(utc_offset_min=off)
        sp_o, tr_o = cref.ingest_spec(1), cref.traj_spec(utc_offset_min=off)
        got, want = _device(sp_d, tr_d, rec), _oracle(sp_o, tr_o, rec)
        assert _same(got, want), (rec, got, want)
        accepted += got is not None
    assert accepted > 1000


def test_wkt_trajectory_has_no_objid():
    rec = b"POINT (116.5 39.9)"
    got = _device(_abi.make_ingest_spec(2), None, rec)
    assert got == (116.5, 39.9, 0, None) and _same(got, _oracle(cref.ingest_spec(2), None, rec))
