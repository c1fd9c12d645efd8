"""CPU oracle (test infrastructure only) of the point CSV/TSV output codec, SURVEY.md 8(f) row 4:
Serialization.PointToCSVTSVOutputSchema.serialize (spatialStreams/Serialization.java:98-152)
and the JDK 8 Double.toString it relies on (StringBuffer.append(double) ->
sun.misc.FloatingDecimal.BinaryToASCIIBuffer: getBinaryToASCIIConverter, dtoa,
estimateDecExp, developLongDigits, roundup, getChars).

PARITY UNPINNED: this is a restatement of the published JDK 8 FloatingDecimal algorithm; no JVM
runs here and the reference ships no serializer fixtures, so the strings are checked against
this restatement (and Java's documented outputs for a handful of well-known values in
tests/test_format_oracle.py), not against the reference itself.  The quirks are kept: the
int / long stopping tests are strict (b + m > tens) with Java's wrapping int / long arithmetic,
the big-integer test is not (10 S <= B + M), and a carry in roundup keeps the digit count.
"""
from __future__ import annotations

import math

import struct

EXP_SHIFT = 52
FRACT_HOB = 1 << 52
EXP_BIAS = 1023
SIGNIF_MASK = (1 << 52) - 1
MAX_SMALL_BIN_EXP = 62
MIN_SMALL_BIN_EXP = -21
N_5_BITS = [0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31, 33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61]
LONG_5_POW_LEN = 27
INSIGNIFICANT_DIGITS = [0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7, 8, 8, 8,
                        9, 9, 9, 9, 10, 10, 10, 11, 11, 11, 12, 12, 12, 12, 13, 13, 13, 14, 14, 14, 15, 15, 15, 15,
                        16, 16, 16, 17, 17, 17, 18, 18, 18, 19]


def _i32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def _i64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= 1 << 63 else v


def _bits(d: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", d))[0]


def _from_bits(b: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", b & ((1 << 64) - 1)))[0]


def _ntz64(v: int) -> int:
    return (v & -v).bit_length() - 1


def estimate_dec_exp(fract_bits: int, bin_exp: int) -> int:
    """FloatingDecimal.estimateDecExp: floor of a fp64 estimate of log10 (Java evaluation order)."""
    d2 = _from_bits((EXP_BIAS << 52) | (fract_bits & SIGNIF_MASK))
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + float(bin_exp) * 0.301029995663981
    db = _bits(d)
    exponent = ((db >> 52) & 0x7FF) - EXP_BIAS
    neg = (db >> 63) != 0
    if 0 <= exponent < 52:
        mask = SIGNIF_MASK >> exponent
        r = ((db & SIGNIF_MASK) | FRACT_HOB) >> (EXP_SHIFT - exponent)
        r = _i32(r)
        return (-r if (mask & db) == 0 else -r - 1) if neg else r
    if exponent < 0:
        return 0 if (db & ~(1 << 63)) == 0 else (-1 if neg else 0)
    return int(d)


class _Buf:
    def __init__(self):
        self.digits: list[str] = []
        self.dec_exponent = 0

    def roundup(self):
        i = len(self.digits) - 1
        q = self.digits[i]
        if q == "9":
            while q == "9" and i > 0:
                self.digits[i] = "0"
                i -= 1
                q = self.digits[i]
            if q == "9":  # carry out: high-order 1, the rest already 0, one more decimal exponent
                self.dec_exponent += 1
                self.digits[0] = "1"
                return
        self.digits[i] = chr(ord(q) + 1)

    def develop_long_digits(self, dec_exponent: int, lvalue: int, insignificant: int):
        if insignificant != 0:
            pow10 = 10 ** insignificant
            residue = lvalue % pow10
            lvalue //= pow10
            dec_exponent += insignificant
            if residue >= (pow10 >> 1):
                lvalue += 1
        ds = []
        c = lvalue % 10
        lvalue //= 10
        while c == 0:
            dec_exponent += 1
            c = lvalue % 10
            lvalue //= 10
        while lvalue != 0:
            ds.append(chr(c + 48))
            dec_exponent += 1
            c = lvalue % 10
            lvalue //= 10
        ds.append(chr(c + 48))
        self.digits = ds[::-1]
        self.dec_exponent = dec_exponent + 1

    def dtoa(self, bin_exp: int, fract_bits: int, n_sig: int):
        tail_zeros = _ntz64(fract_bits)
        n_fract_bits = EXP_SHIFT + 1 - tail_zeros
        n_tiny_bits = max(0, n_fract_bits - bin_exp - 1)
        if MIN_SMALL_BIN_EXP <= bin_exp <= MAX_SMALL_BIN_EXP:
            if n_tiny_bits < LONG_5_POW_LEN and (n_fract_bits + N_5_BITS[n_tiny_bits]) < 64 and n_tiny_bits == 0:
                ins = 0
                if bin_exp > n_sig:
                    p2 = bin_exp - n_sig - 1
                    ins = INSIGNIFICANT_DIGITS[p2] if 1 < p2 < len(INSIGNIFICANT_DIGITS) else 0
                fb = fract_bits << (bin_exp - EXP_SHIFT) if bin_exp >= EXP_SHIFT else fract_bits >> (EXP_SHIFT - bin_exp)
                self.develop_long_digits(0, fb, ins)
                return
        dec_exp = estimate_dec_exp(fract_bits, bin_exp)
        B5 = max(0, -dec_exp)
        B2 = B5 + n_tiny_bits + bin_exp
        S5 = max(0, dec_exp)
        S2 = S5 + n_tiny_bits
        M5 = B5
        M2 = B2 - n_sig
        fract_bits >>= tail_zeros
        B2 -= n_fract_bits - 1
        common2 = min(B2, S2)
        B2 -= common2
        S2 -= common2
        M2 -= common2
        if n_fract_bits == 1:
            M2 -= 1
        if M2 < 0:
            B2 -= M2
            S2 -= M2
            M2 = 0
        Bbits = n_fract_bits + B2 + (N_5_BITS[B5] if B5 < len(N_5_BITS) else B5 * 3)
        tenSbits = S2 + 1 + (N_5_BITS[S5 + 1] if S5 + 1 < len(N_5_BITS) else (S5 + 1) * 3)
        digits: list[str] = []
        if Bbits < 64 and tenSbits < 64:
            wrap = _i32 if (Bbits < 32 and tenSbits < 32) else _i64
            b = wrap((fract_bits * 5 ** B5) << B2)
            s = wrap((5 ** S5) << S2)
            m = wrap((5 ** M5) << M2)
            tens = wrap(s * 10)
            q = b // s
            b = wrap(10 * (b % s))
            m = wrap(m * 10)
            low = b < m
            high = wrap(b + m) > tens
            if q == 0 and not high:
                dec_exp -= 1
            else:
                digits.append(chr(48 + q))
            if dec_exp < -3 or dec_exp >= 8:
                high = low = False
            while not low and not high:
                q = b // s
                b = wrap(10 * (b % s))
                m = wrap(m * 10)
                if m > 0:
                    low = b < m
                    high = wrap(b + m) > tens
                else:  # m overflowed
                    low = high = True
                digits.append(chr(48 + q))
            low_digit_difference = wrap(wrap(b << 1) - tens)
        else:
            # exact big-integer arithmetic (FDBigInteger's normalisation shift scales every term
            # alike and leaves the comparisons unchanged); M starts scaled by 10 as
            # valueOfPow52(M5 + 1, M2 + 1) does, quoRemIteration leaves 10 (B mod S)
            S = (5 ** S5) << S2
            B = (fract_bits * 5 ** B5) << B2
            M = (5 ** (M5 + 1)) << (M2 + 1)
            tenS = (5 ** (S5 + 1)) << (S2 + 1)
            q, B = B // S, 10 * (B % S)
            low = B < M
            high = tenS <= B + M
            if q == 0 and not high:
                dec_exp -= 1
            else:
                digits.append(chr(48 + q))
            if dec_exp < -3 or dec_exp >= 8:
                high = low = False
            while not low and not high:
                q, B = B // S, 10 * (B % S)
                M *= 10
                low = B < M
                high = tenS <= B + M
                digits.append(chr(48 + q))
            low_digit_difference = ((B << 1) > tenS) - ((B << 1) < tenS) if (high and low) else 0
        self.digits = digits
        self.dec_exponent = dec_exp + 1
        if high:
            if low:
                if low_digit_difference == 0:
                    if (ord(self.digits[-1]) & 1) != 0:
                        self.roundup()
                elif low_digit_difference > 0:
                    self.roundup()
            else:
                self.roundup()

    def chars(self, negative: bool) -> str:
        out = "-" if negative else ""
        de, nd, ds = self.dec_exponent, len(self.digits), self.digits
        if 0 < de < 8:
            cl = min(nd, de)
            out += "".join(ds[:cl])
            if cl < de:
                out += "0" * (de - cl) + ".0"
            else:
                out += "." + ("".join(ds[cl:]) if cl < nd else "0")
        elif -3 < de <= 0:
            out += "0." + "0" * (-de) + "".join(ds)
        else:
            out += ds[0] + "." + ("".join(ds[1:]) if nd > 1 else "0") + "E"
            if de <= 0:
                out += "-"
                e = -de + 1
            else:
                e = de - 1
            out += str(e)
        return out


def java_double_to_string(d: float) -> str:
    """Double.toString(d) of JDK 8 (FloatingDecimal.toJavaFormatString)."""
    bits = _bits(d)
    neg = (bits >> 63) != 0
    fract = bits & SIGNIF_MASK
    bin_exp = (bits >> 52) & 0x7FF
    if bin_exp == 0x7FF:
        return ("-Infinity" if neg else "Infinity") if fract == 0 else "NaN"
    if bin_exp == 0:
        if fract == 0:
            return "-0.0" if neg else "0.0"
        lz = 64 - fract.bit_length()
        shift = lz - (63 - EXP_SHIFT)
        fract <<= shift
        bin_exp = 1 - shift
        n_sig = 64 - lz
    else:
        fract |= FRACT_HOB
        n_sig = EXP_SHIFT + 1
    bin_exp -= EXP_BIAS
    b = _Buf()
    b.dtoa(bin_exp, fract, n_sig)
    return b.chars(neg)


def format_point_csv(oid, ts: int, x: float, y: float, attrs, delim: str) -> str:
    """PointToCSVTSVOutputSchema.serialize (Serialization.java:106-152): positionMap from
    csvTsvSchemaAttr (objID, timeStampMillisec, x, y; a later field wins a shared position),
    fields 0..max in order, "0" where no field sits, each followed by the delimiter, the final
    character deleted.  oid None -> "null" (StringBuffer.append of a null String)."""
    pos = {}
    for name, p in zip(("objID", "ts", "x", "y"), attrs):
        pos[p] = name
    parts = []
    for i in range(max(pos) + 1):
        f = pos.get(i)
        if f == "objID":
            parts.append("null" if oid is None else oid)
        elif f == "ts":
            parts.append(str(int(ts)))
        elif f == "x":
            parts.append(java_double_to_string(x))
        elif f == "y":
            parts.append(java_double_to_string(y))
        else:
            parts.append("0")
        parts.append(delim)
    s = "".join(parts)
    # StringBuffer.deleteCharAt(length - 1) removes one UTF-16 unit: a supplementary last
    # character leaves its high surrogate, which String.getBytes(UTF_8) writes as '?'
    return s[:-1] + ("?" if ord(s[-1]) > 0xFFFF else "")


# ---------------------------------------------------------------- WKT / GeoJSON schemas ----
def java_date_ymd_hms(ms: int, utc_offset_min: int = 0) -> str:
    """SimpleDateFormat("yyyy-MM-dd HH:mm:ss").format(new Date(ms)) in a fixed-offset zone
    (the proleptic Gregorian calendar of datetime equals GregorianCalendar from 1583 on)."""
    import datetime
    t = datetime.datetime(1970, 1, 1) + datetime.timedelta(milliseconds=ms + utc_offset_min * 60000)
    if not 1583 <= t.year <= 9999:
        raise ValueError("outside the supported years")
    return t.strftime("%Y-%m-%d %H:%M:%S")


def format_point_wkt(oid, ts: int, x: float, y: float, delim: str, utc_offset_min: int = 0) -> str:
    """PointToWKTOutputSchema.serialize (Serialization.java:72-92)."""
    buf = ['"']
    if oid is not None:
        buf += [oid, delim + " "]
    buf += ["POINT(", java_double_to_string(x), " ", java_double_to_string(y), ")"]
    if ts != 0:
        buf += [delim + " ", java_date_ymd_hms(ts, utc_offset_min)]
    buf += ['"', delim]
    return "".join(buf)


def java_string_hash(s: str) -> int:
    """String.hashCode over the UTF-16 units."""
    h = 0
    for u in _utf16_units(s):
        h = (31 * h + u) & 0xFFFFFFFF
    return h


def _utf16_units(s: str):
    b = s.encode("utf-16-be")
    return [int.from_bytes(b[i:i + 2], "big") for i in range(0, len(b), 2)]


def java8_hashmap_order(keys):
    """Iteration order of a java.util.HashMap (Java 8) after putting `keys` in order into a
    default-constructed map: table of 16 buckets (no resize below 13 entries), bucket index
    (h ^ (h >>> 16)) & 15, insertion order inside a bucket."""
    assert len(keys) <= 12
    buckets = {}
    for k in keys:
        h = java_string_hash(k)
        buckets.setdefault((h ^ (h >> 16)) & 15, []).append(k)
    return [k for b in sorted(buckets) for k in buckets[b]]


def json_number_to_string(d: float) -> str:
    """org.json JSONObject.numberToString(Double) (20200518): non-finite throws; Double.toString
    with trailing zeros and then a trailing '.' shaved when it has a '.' and no exponent."""
    if math.isnan(d) or math.isinf(d):
        raise ValueError("JSON does not allow non-finite numbers.")
    s = java_double_to_string(d)
    if s.find(".") > 0 and "e" not in s and "E" not in s:
        s = s.rstrip("0")
        if s.endswith("."):
            s = s[:-1]
    return s


def json_quote(s: str) -> str:
    """org.json JSONObject.quote over the UTF-16 units of s."""
    if not s:
        return '""'
    out = ['"']
    prev = 0
    # code points; a supplementary one is a surrogate pair in Java, never in an escaped range
    for ch in s:
        c = ord(ch)
        if ch in ('\\', '"'):
            out.append("\\" + ch)
        elif ch == "/":
            out.append("\\/" if prev == ord("<") else "/")
        elif ch == "\b":
            out.append("\\b")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\f":
            out.append("\\f")
        elif ch == "\r":
            out.append("\\r")
        elif c < 0x20 or 0x80 <= c < 0xA0 or 0x2000 <= c < 0x2100:
            out.append("\\u%04x" % c)
        else:
            out.append(ch)
        prev = c if c <= 0xFFFF else 0xDC00  # the low surrogate precedes the next unit
    out.append('"')
    return "".join(out)


def _json_write(v) -> str:
    if isinstance(v, dict):
        return "{" + ",".join(json_quote(k) + ":" + _json_write(v[k]) for k in java8_hashmap_order(list(v))) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_json_write(e) for e in v) + "]"
    if isinstance(v, float):
        return json_number_to_string(v)
    return json_quote(v)


def format_point_geojson(oid, ts: int, x: float, y: float, utc_offset_min: int = 0) -> str:
    """PointToGeoJSONOutputSchema.serialize (Serialization.java:28-50) with org.json 20200518:
    keys put in source order into HashMap-backed JSONObjects, written in HashMap order."""
    geometry = {"coordinates": [float(x), float(y)], "type": "Point"}
    props = {}
    if oid is not None:  # put("oID", null) removes the key
        props["oID"] = oid
    if ts != 0:
        props["timestamp"] = java_date_ymd_hms(ts, utc_offset_min)
    obj = {"geometry": geometry}
    if props:
        obj["properties"] = props
    obj["type"] = "Feature"
    return _json_write(obj)
