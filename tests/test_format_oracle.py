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
