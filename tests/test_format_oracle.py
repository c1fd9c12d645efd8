"""CPU: the JDK 8 Double.toString restatement (oracle/jdk_double.py) and the CSV/TSV record
layout of Serialization.PointToCSVTSVOutputSchema (Serialization.java:98-152).

Parity unpinned (no JVM here): Java's documented outputs for well-known values -- including the
JDK 8 FloatingDecimal anomalies JDK-4511638 reports (1.0E23 -> 9.999999999999999E22,
2.0E23 -> 1.9999999999999998E23) -- and the round-trip property (Double.parseDouble of the
string gives the double back) over random bit patterns."""
import math
import random
import struct

import jdk_double as J

KNOWN = [(1.0, "1.0"), (0.1, "0.1"), (100.0, "100.0"), (1e7, "1.0E7"), (1234567.0, "1234567.0"), (0.001, "0.001"),
         (1e-4, "1.0E-4"), (116.414899, "116.414899"), (39.920374, "39.920374"),
         (1.7976931348623157e308, "1.7976931348623157E308"), (5e-324, "4.9E-324"), (1e23, "9.999999999999999E22"),
         (2e23, "1.9999999999999998E23"), (2.0 ** 53, "9.007199254740992E15"), (1 / 3, "0.3333333333333333"),
         (100 / 3, "33.333333333333336"), (-0.0, "-0.0"), (0.0, "0.0"), (math.nan, "NaN"), (math.inf, "Infinity"),
         (-math.inf, "-Infinity"), (123456789.0, "1.23456789E8"), (1e-7, "1.0E-7"), (-2.5, "-2.5"),
         (12345678.9, "1.23456789E7"), (0.00012345, "1.2345E-4"), (1e21, "1.0E21"), (1e22, "1.0E22")]


def test_known_values():
    for v, s in KNOWN:
        assert J.java_double_to_string(v) == s, (v, J.java_double_to_string(v), s)


def test_round_trip_random_bits():
    rng = random.Random(5)
    for _ in range(20000):
        d = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0]
        if d != d or math.isinf(d):
            continue
        s = J.java_double_to_string(d)
        assert float(s) == d, (repr(d), s)


def test_csv_record_layout():
    assert J.format_point_csv("17", 1611022449423, 116.5, 40.25, (0, 1, 2, 3), ",") == "17,1611022449423,116.5,40.25"
    # a gap (position 2 holds no field -> "0") and the final character deleted
    assert J.format_point_csv("a", 5, 1.0, 2.0, (0, 1, 3, 4), "\t") == "a\t5\t0\t1.0\t2.0"
    # a shared position: the later field (y) wins
    assert J.format_point_csv(None, 0, 1.0, 2.0, (0, 1, 2, 2), ";") == "null;0;2.0"
    # a two-character delimiter keeps its first character at the end
    assert J.format_point_csv("x", 1, 3.0, 4.0, (0, 1, 2, 3), "||") == "x||1||3.0||4.0|"


def test_csv_delete_char_is_one_utf16_unit():
    # a BMP delimiter character goes whole; a supplementary one leaves its high surrogate ('?')
    assert J.format_point_csv("x", 1, 3.0, 4.0, (0, 1, 2, 3), "é") == "xé1é3.0é4.0"
    assert J.format_point_csv("x", 1, 3.0, 4.0, (0, 1, 2, 3), "\U0001F600") == "x\U0001F6001\U0001F6003.0\U0001F6004.0?"


def test_java8_hashmap_order_of_the_schema_keys():
    # String.hashCode by hand: "type" = 't'*31^3 + 'y'*31^2 + 'p'*31 + 'e' = 3575610 = 0x368f3a;
    # (h ^ h >>> 16) & 15 = (0x368f3a ^ 0x36) & 15 = 0xc = 12
    assert J.java_string_hash("type") == 3575610
    assert J.java8_hashmap_order(["geometry", "properties", "type"]) == ["geometry", "type", "properties"]
    assert J.java8_hashmap_order(["coordinates", "type"]) == ["coordinates", "type"]
    assert J.java8_hashmap_order(["oID", "timestamp"]) == ["oID", "timestamp"]


def test_json_number_and_quote():
    assert J.json_number_to_string(116.0) == "116"
    assert J.json_number_to_string(116.5) == "116.5"
    assert J.json_number_to_string(-0.0) == "-0"
    assert J.json_number_to_string(1e-5) == "1.0E-5"  # an exponent: nothing shaved
    assert J.json_number_to_string(100.0) == "100"
    assert J.json_quote("") == '""'
    assert J.json_quote('a"b\\c</d/e') == '"a\\"b\\\\c<\\/d/e"'
    assert J.json_quote("\x01\t\u0085  ") == '"\\u0001\\t\\u0085\\u2028 "'


def test_wkt_and_geojson_layout():
    # 2021-01-19 02:14:09.423 UTC
    ts = 1611022449423
    assert J.java_date_ymd_hms(ts) == "2021-01-19 02:14:09"
    assert J.java_date_ymd_hms(ts, 480) == "2021-01-19 10:14:09"
    assert J.java_date_ymd_hms(-1) == "1969-12-31 23:59:59"
    assert J.format_point_wkt("17", ts, 116.5, 40.25, ",") == '"17, POINT(116.5 40.25), 2021-01-19 02:14:09",'
    assert J.format_point_wkt(None, 0, 116.5, 40.0, "\t") == '"POINT(116.5 40.0)"\t'
    assert (J.format_point_geojson("17", ts, 116.5, 40.0) ==
            '{"geometry":{"coordinates":[116.5,40],"type":"Point"},"type":"Feature",'
            '"properties":{"oID":"17","timestamp":"2021-01-19 02:14:09"}}')
    assert J.format_point_geojson(None, 0, 1.0, 2.0) == '{"geometry":{"coordinates":[1,2],"type":"Point"},"type":"Feature"}'
