// ingest_parse.h -- record parsers of the ingest codec, written once as
// __host__ __device__ code: the gfx950 kernels run them per record, and the CPU test suite runs the
// very same functions through geohip_debug_ingest_fast (no GPU needed to check their decisions).
//
// Reference (paths relative to /root/reference/src/main/java/GeoFlink):
//   CSVTSVToSpatial.map   spatialStreams/Deserialization.java:248-254
//       str.replace("\"", "").split("\\s*" + delimiter + "\\s*"); Double.valueOf(fields[attr[2|3]])
//   CSVTSVToTSpatial.map  spatialStreams/Deserialization.java:306-321   + Long.valueOf(fields[attr[1]])
//   GeoJSONToSpatial.map  spatialStreams/Deserialization.java:132-146   JTS GeoJsonReader, getCoordinate()
//   WKTToSpatial.map      spatialStreams/Deserialization.java:223-228, 1510-1514
//       str.indexOf("POINT"), JTS WKTReader.read(substring), getCoordinate()
//
// The device parser accepts exactly what it can decide bit-exactly -- decimal tokens (any digit
// count when the 19-digit truncation decides the rounding, exponents of any length), hex
// significands (FloatingDecimal.parseHexString), NaN/Infinity, Java type suffixes, quotes inside
// CSV tokens, 19-digit longs, a third WKT ordinate and the common record shapes -- and converts
// decimals with the Eisel-Lemire algorithm (correctly rounded, ties to even: the value
// Double.parseDouble returns).  Everything else returns kFallback and the batch call reports
// GEOHIP_ERR_UNSUPPORTED with the first such record: malformed text (where the reference throws
// NumberFormatException / IndexOutOfBounds / ParseException) and forms whose Java behaviour is
// not restated here (tokens of 100000+ characters, a zero hex significand with an exponent past
// int range, Z / M tags).  The library has no CPU parsing path; the caller
// hands such a batch back to the reference's own Java deserializer, which parses it or throws.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ingest_pow5.h"

namespace geohip {
namespace ingest {

constexpr int kOk = 0;
constexpr int kFallback = 1;

enum Format { kCsv = 0, kGeoJson = 1, kWkt = 2 };

// The objID of a record as a span of the batch text: (offset << kOidLenBits) | length, the bytes
// the reference's String holds once the quotes in them are deleted (CSV) -- or kOidNull for a
// null objID.  Offsets below 2^40 (batches are < 1 TiB), lengths below kMaxTokenLen.
constexpr int kOidLenBits = 24;
constexpr uint64_t kOidNull = (1ull << kOidLenBits) - 1;
constexpr int kPropKeyMax = 60;

struct Spec {
    int32_t format;
    int32_t delim;  // CSV/TSV delimiter byte
    int32_t fx, fy;  // csvTsvSchemaAttr[2], [3]
    int32_t fts;     // csvTsvSchemaAttr[1] (Long.valueOf timestamp), < 0: not parsed
    int32_t foid;    // csvTsvSchemaAttr[0] (the objID span), < 0: not produced
    // GeoJSONToTSpatial (traj != 0): properties[kts] parsed by the DateFormat (date_fmt: 0 none,
    // 1 "yyyy-MM-dd HH:mm:ss" in a zone of fixed offset utc_off_min), properties[koid] the objID
    int32_t traj, date_fmt, utc_off_min;
    int32_t kts_len, koid_len;
    char kts[kPropKeyMax], koid[kPropKeyMax];
};

struct Parsed {
    double x, y;
    int64_t ts;
    uint64_t oid;  // span (kOidNull: null); only when the spec asks for it
};

#if defined(__HIP_DEVICE_COMPILE__)
__device__ const uint64_t kPow5[] = {GEOHIP_POW5_INIT};
#else
static const uint64_t kPow5[] = {GEOHIP_POW5_INIT};
#endif

__host__ __device__ inline void mul_64x64(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
#if defined(__HIP_DEVICE_COMPILE__)
    lo = a * b;
    hi = __umul64hi(a, b);
#else
    const unsigned __int128 p = (unsigned __int128)a * b;
    lo = (uint64_t)p;
    hi = (uint64_t)(p >> 64);
#endif
}

// Binary64 bits nearest to w * 10^q (ties to even) for an exact significand 0 <= w < 10^19
// (Eisel-Lemire; Mushtak & Lemire 2023 prove the 128-bit product always decides for such w).
__host__ __device__ inline uint64_t decimal_to_bits(uint64_t w, int32_t q) {
    if (w == 0 || q < GEOHIP_POW5_MIN_Q) return 0;
    if (q > GEOHIP_POW5_MAX_Q) return 0x7ffull << 52;
    const int lz = __builtin_clzll(w);
    w <<= lz;
    const int idx = 2 * (q - GEOHIP_POW5_MIN_Q);
    uint64_t hi, lo;
    mul_64x64(w, kPow5[idx], hi, lo);
    if ((hi & 0x1ff) == 0x1ff) {  // the truncated 5^q may matter below bit 55: add its low word
        uint64_t h2, l2;
        mul_64x64(w, kPow5[idx + 1], h2, l2);
        lo += h2;
        if (h2 > lo) hi++;
    }
    const int upper = (int)(hi >> 63);
    const int shift = upper + 9;  // 64 - 52 - 3
    uint64_t m = hi >> shift;     // 53 mantissa bits + 1 rounding bit
    int32_t p2 = (int32_t)((((152170 + 65536) * q) >> 16) + 63) + upper - lz + 1023;
    if (p2 <= 0) {  // subnormal or underflow to zero
        if (-p2 + 1 >= 64) return 0;
        m >>= -p2 + 1;
        m += m & 1;
        m >>= 1;
        return m | ((uint64_t)(m < (1ull << 52) ? 0 : 1) << 52);
    }
    if (lo <= 1 && q >= -4 && q <= 23 && (m & 3) == 1 && (m << shift) == hi) m &= ~1ull;  // exact tie: even
    m += m & 1;
    m >>= 1;
    if (m >= (2ull << 52)) {
        m = 1ull << 52;
        p2++;
    }
    m &= ~(1ull << 52);
    if (p2 >= 0x7ff) return 0x7ffull << 52;
    return m | ((uint64_t)p2 << 52);
}

__host__ __device__ inline bool is_digit(uint8_t c) { return (unsigned)(c - '0') < 10u; }
// java.util.regex \s
__host__ __device__ inline bool is_jspace(uint8_t c) {
    return c == ' ' || c == '\t' || c == '\n' || c == 0x0b || c == '\f' || c == '\r';
}

// A token this long could carry enough leading zeros to cancel a 10^6+ exponent, where
// FloatingDecimal's exponent clamp (expLimit) is not restated: such tokens go to the host.
constexpr uint64_t kMaxTokenLen = 100000;

// Hex significand (FloatingDecimal.parseHexString): 0[xX](hex+[.]|hex*.hex+)[pP][+-]?digits
// [fFdD]? after the sign, at p; the exact binary value correctly rounded (ties to even) to
// binary64, subnormals included; an exponent past int range is +-Infinity / 0 (a zero
// significand with one -> kFallback).
template <class R>
__host__ __device__ inline int parse_hex(const R& rd, uint64_t p, uint64_t e, bool neg, double* out) {
    p += 2;  // "0x"
    uint64_t m = 0;      // leading 60 significant bits
    int64_t e2 = 0;      // value = (m + below) * 2^e2
    bool sticky = false; // a nonzero bit below m
    int nh = 0;
    auto hv = [](uint8_t c) -> int {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    };
    uint8_t c = p < e ? rd(p) : 0;
    for (int v; p < e && (v = hv(c)) >= 0; c = ++p < e ? rd(p) : 0, nh++) {
        if ((m >> 56) == 0) m = m * 16 + (uint64_t)v;
        else {
            sticky |= v != 0;
            e2 += 4;
        }
    }
    if (p < e && c == '.') {
        c = ++p < e ? rd(p) : 0;
        for (int v; p < e && (v = hv(c)) >= 0; c = ++p < e ? rd(p) : 0, nh++) {
            if ((m >> 56) == 0) {
                m = m * 16 + (uint64_t)v;
                e2 -= 4;
            } else {
                sticky |= v != 0;
            }
        }
    }
    if (nh == 0 || p >= e || (c != 'p' && c != 'P')) return kFallback;
    c = ++p < e ? rd(p) : 0;
    bool eneg = false;
    if (p < e && (c == '+' || c == '-')) {
        eneg = c == '-';
        c = ++p < e ? rd(p) : 0;
    }
    int64_t ev = 0;
    int ne = 0;
    bool big = false;  // past int range (Integer.parseInt of the exponent fails)
    while (p < e && is_digit(c)) {
        if (ev > 214748364 || (ev == 214748364 && c - '0' > 7)) big = true;
        if (!big) ev = ev * 10 + (c - '0');
        ne++;
        c = ++p < e ? rd(p) : 0;
    }
    if (ne == 0) return kFallback;
    if (p < e && (c == 'f' || c == 'F' || c == 'd' || c == 'D')) p++;
    if (p != e) return kFallback;
    const uint64_t sign = neg ? 1ull << 63 : 0ull;
    if (m == 0) {
        if (big) return kFallback;
        *out = __builtin_bit_cast(double, sign);
        return kOk;
    }
    uint64_t bits;
    if (big) {
        bits = eneg ? 0ull : 0x7ffull << 52;
    } else {
        const int lz = __builtin_clzll(m);
        m <<= lz;  // value = 1.f * 2^ex
        const int64_t ex = e2 + (eneg ? -ev : ev) + 63 - lz;
        if (ex > 1023) {
            bits = 0x7ffull << 52;
        } else {
            const int sh = ex >= -1022 ? 11 : (int)(11 + (-1022 - ex) < 70 ? 11 + (-1022 - ex) : 70);
            uint64_t mant = 0;
            bool up = false;
            if (sh < 64) {
                mant = m >> sh;
                const uint64_t rem = m & ((1ull << sh) - 1), half = 1ull << (sh - 1);
                up = rem > half || (rem == half && (sticky || (mant & 1)));
            } else if (sh == 64) {
                up = m > (1ull << 63) || (m == (1ull << 63) && sticky);
            }
            mant += up ? 1 : 0;
            if (ex >= -1022) {
                int64_t be = ex + 1023;
                if (mant >> 53) {
                    mant >>= 1;
                    be++;
                }
                bits = be >= 0x7ff ? 0x7ffull << 52 : ((uint64_t)be << 52) | (mant & ((1ull << 52) - 1));
            } else {
                bits = mant;  // subnormal (a carry to 2^52 is the smallest normal)
            }
        }
    }
    *out = __builtin_bit_cast(double, bits | sign);
    return kOk;
}

// Decimal token [s, e) -> double (correctly rounded, ties to even).
// json: RFC 8259 number grammar as Jackson reads it (no '+', no leading zeros, digits on both
//   sides of '.'); an integer token is an IntNode/LongNode, so "-0" is +0.0, and an integer
//   outside long range (BigIntegerNode, which JTS's reader rejects) goes to kFallback.
// else: FloatingDecimal.readJavaFormatString's grammar on an already trimmed token: [+-]?
//   then "NaN" | "Infinity" | hex (parse_hex) | digits[.digits][(e|E)[+-]?digits][fFdD].
// Exponents of any length: beyond 10^8 the value is 0 or +-Infinity for a nonzero significand.
// More than 19 significant digits: the token is truncated to 19 and converted at w and w + 1;
// equal results decide it (the true value lies between them), unequal -> kFallback.
template <class R>
__host__ __device__ inline int parse_decimal(const R& rd, uint64_t s, uint64_t e, bool json, double* out) {
    if (s >= e || e - s >= kMaxTokenLen) return kFallback;
    uint64_t p = s;
    uint8_t c = rd(p);
    bool neg = false;
    if (c == '-' || (!json && c == '+')) {
        neg = c == '-';
        if (++p >= e) return kFallback;
        c = rd(p);
    }
    if (!json && c == '0' && p + 1 < e && (rd(p + 1) == 'x' || rd(p + 1) == 'X')) return parse_hex(rd, p, e, neg, out);
    if (!json && (c == 'N' || c == 'I')) {
        const char* word = c == 'N' ? "NaN" : "Infinity";
        const uint64_t len = c == 'N' ? 3 : 8;
        if (e - p != len) return kFallback;
        for (uint64_t i = 1; i < len; i++)
            if (rd(p + i) != (uint8_t)word[i]) return kFallback;
        const uint64_t bits = c == 'N' ? 0x7ff8000000000000ull : ((0x7ffull << 52) | (neg ? 1ull << 63 : 0ull));
        *out = __builtin_bit_cast(double, bits);
        return kOk;
    }
    const uint64_t int0 = p;
    uint64_t w = 0;
    int nd = 0;      // significant digits held in w
    int32_t q = 0;   // value = (w + tail) * 10^q
    int ni = 0, nf = 0;
    bool trunc = false;  // a non-zero digit was dropped past the 19th
    while (p < e && is_digit(c)) {
        if (nd || c != '0') {
            if (nd < 19) {
                w = w * 10 + (uint64_t)(c - '0');
                nd++;
            } else {
                q++;
                trunc |= c != '0';
            }
        }
        ni++;
        if (++p < e) c = rd(p);
    }
    if (json && (ni == 0 || (ni > 1 && rd(int0) == '0'))) return kFallback;
    bool frac = false, expo = false;
    if (p < e && c == '.') {
        frac = true;
        if (++p < e) c = rd(p);
        while (p < e && is_digit(c)) {
            if (nd < 19) {
                if (nd || c != '0') {
                    w = w * 10 + (uint64_t)(c - '0');
                    nd++;
                }
                q--;
            } else {
                trunc |= c != '0';
            }
            nf++;
            if (++p < e) c = rd(p);
        }
        if (json && nf == 0) return kFallback;
    }
    if (ni + nf == 0) return kFallback;
    if (p < e && (c == 'e' || c == 'E')) {
        expo = true;
        if (++p >= e) return kFallback;
        c = rd(p);
        bool eneg = false;
        if (c == '+' || c == '-') {
            eneg = c == '-';
            if (++p >= e) return kFallback;
            c = rd(p);
        }
        int32_t ev = 0;
        int ne = 0;
        while (p < e && is_digit(c)) {
            if (ev < 100000000) ev = ev * 10 + (c - '0');  // beyond: 0 or Infinity either way
            ne++;
            if (++p < e) c = rd(p);
        }
        if (ne == 0) return kFallback;
        q += eneg ? -ev : ev;
    }
    if (p < e && !json && (c == 'f' || c == 'F' || c == 'd' || c == 'D')) p++;  // type suffix
    if (p != e) return kFallback;  // hex, stray characters
    if (json && !frac && !expo) {
        // IntNode / LongNode (then Long.valueOf of its text): within long range only
        if (nd > 19 || (nd == 19 && w > (neg ? 9223372036854775808ull : 9223372036854775807ull))) return kFallback;
        if (w == 0) neg = false;  // IntNode 0
    }
    uint64_t bits = decimal_to_bits(w, q);
    if (trunc && decimal_to_bits(w + 1, q) != bits) return kFallback;
    // JSON overflow: DoubleNode(Infinity) re-serialises as "Infinity", which JTS's JSON reader rejects
    if (json && (bits & (0x7ffull << 52)) == (0x7ffull << 52)) return kFallback;
    bits |= neg ? 1ull << 63 : 0ull;
    *out = __builtin_bit_cast(double, bits);
    return kOk;
}

// Long.valueOf: [+-]?digits, no trim, within [-2^63, 2^63 - 1] (else NumberFormatException)
template <class R>
__host__ __device__ inline int parse_long(const R& rd, uint64_t s, uint64_t e, int64_t* out) {
    if (s >= e) return kFallback;
    uint64_t p = s;
    const uint8_t c0 = rd(p);
    const bool neg = c0 == '-';
    if (c0 == '+' || c0 == '-') p++;
    if (p >= e) return kFallback;
    uint64_t v = 0;
    const uint64_t lim = neg ? 9223372036854775808ull : 9223372036854775807ull;
    for (; p < e; p++) {
        const uint8_t c = rd(p);
        if (!is_digit(c)) return kFallback;
        const uint64_t d = (uint64_t)(c - '0');
        if (v > (lim - d) / 10) return kFallback;  // beyond the long range
        v = v * 10 + d;
    }
    *out = neg ? (int64_t)(0ull - v) : (int64_t)v;
    return kOk;
}

// A token with the quotes inside it deleted (str.replace("\"", "") before the split), copied
// into a local buffer; tokens longer than kQuoteBuf -> kFallback.
constexpr int kQuoteBuf = 96;
struct BufReader {
    const uint8_t* b;
    __host__ __device__ uint8_t operator()(uint64_t p) const { return b[p]; }
};
template <class R>
__host__ __device__ inline bool unquote(const R& rd, uint64_t t0, uint64_t t1, uint8_t* buf, uint64_t* len) {
    uint64_t n = 0;
    for (uint64_t p = t0; p < t1; p++) {
        const uint8_t c = rd(p);
        if (c == '"') continue;
        if (n >= (uint64_t)kQuoteBuf) return false;
        buf[n++] = c;
    }
    *len = n;
    return true;
}

// A CSV field's number: quotes inside the token are deleted first (the reference deletes every
// quote before the split)
template <class R>
__host__ __device__ inline bool has_quote(const R& rd, uint64_t t0, uint64_t t1) {
    for (uint64_t p = t0; p < t1; p++)
        if (rd(p) == '"') return true;
    return false;
}
template <class R>
__host__ __device__ inline int field_decimal(const R& rd, uint64_t t0, uint64_t t1, double* v) {
    if (!has_quote(rd, t0, t1)) return parse_decimal(rd, t0, t1, false, v);
    uint8_t buf[kQuoteBuf];
    uint64_t n = 0;
    if (!unquote(rd, t0, t1, buf, &n)) return kFallback;
    return parse_decimal(BufReader{buf}, 0, n, false, v);
}
template <class R>
__host__ __device__ inline int field_long(const R& rd, uint64_t t0, uint64_t t1, int64_t* v) {
    if (!has_quote(rd, t0, t1)) return parse_long(rd, t0, t1, v);
    uint8_t buf[kQuoteBuf];
    uint64_t n = 0;
    if (!unquote(rd, t0, t1, buf, &n)) return kFallback;
    return parse_long(BufReader{buf}, 0, n, v);
}

// CSVTSVToSpatial / CSVTSVToTSpatial.  Quotes are deleted before the split, so they never end a
// field; a separator is the delimiter with the \s runs around it (non-space delimiters) or a
// maximal run of \s / quotes that contains the delimiter (whitespace delimiters).  A field's
// number token is its text without surrounding chars <= ' ' or quotes (Double.valueOf trims).
// Long.valueOf does not trim: the timestamp field is rejected if \s survives the split around it
// (before field 0, after the last field) or if it holds any other control character.
//
// The objID (CSVTSVToTSpatial's strArrayList.get(csvTsvSchemaAttr.get(0)), Deserialization.java:
// 313-314) is the field's raw bytes between its separators: the \s / quote runs the split consumes
// around the delimiter are outside it, the leading \s of field 0 and the trailing \s of the last
// field stay (no separator match there), and the quotes inside it are deleted when the span is
// read (geohip_ingest_oid_compact).  An empty or control-character objID goes to the host.
template <class R>
__host__ __device__ inline int parse_csv(const R& rd, uint64_t p, const Spec& sp, Parsed* o) {
    int need = sp.fx > sp.fy ? sp.fx : sp.fy;
    if (sp.fts > need) need = sp.fts;
    if (sp.foid > need) need = sp.foid;
    const uint64_t rec0 = p;
    const uint8_t d = (uint8_t)sp.delim;
    const bool wsd = is_jspace(d);
    for (int f = 0;; f++) {
        uint64_t t0 = ~0ull, t1 = 0;
        bool lead = false, trail = false, ctrl = false, sep = false;
        for (;;) {
            const uint8_t c = rd(p);
            if (c == '\n') break;
            if (!wsd) {
                if (c == d) {
                    p++;
                    sep = true;
                    break;
                }
            } else if (is_jspace(c) || c == '"') {
                uint64_t r = p;
                bool hasd = false, hasws = false;
                for (;;) {
                    const uint8_t c2 = rd(r);
                    if (c2 == '\n' || !(is_jspace(c2) || c2 == '"')) break;
                    hasd |= c2 == d;
                    hasws |= c2 != '"';
                    r++;
                }
                p = r;
                if (hasd) {
                    sep = true;
                    break;
                }
                if (hasws) (t0 == ~0ull ? lead : trail) = true;
                continue;
            }
            if (c > ' ' && c != '"') {
                if (t0 == ~0ull) t0 = p;
                t1 = p + 1;
                trail = false;  // blanks between token characters stay inside [t0, t1)
            } else if (c != '"') {
                if (!is_jspace(c)) ctrl = true;
                (t0 == ~0ull ? lead : trail) = true;
            }
            p++;
        }
        if (f == sp.fx || f == sp.fy) {
            double v;
            if (t0 == ~0ull || field_decimal(rd, t0, t1, &v) != kOk) return kFallback;
            if (f == sp.fx) o->x = v;
            if (f == sp.fy) o->y = v;
        }
        if (f == sp.fts && (ctrl || (f == 0 && lead) || (!sep && trail) || t0 == ~0ull ||
                            field_long(rd, t0, t1, &o->ts) != kOk))
            return kFallback;
        if (f == sp.foid) {
            if (ctrl || t0 == ~0ull) return kFallback;
            const uint64_t a = f == 0 ? rec0 : t0, b = sep ? t1 : p;  // p: the record's '\n'
            if (b - a >= kMaxTokenLen) return kFallback;
            o->oid = (a << kOidLenBits) | (b - a);
        }
        if (f == need) return kOk;
        if (!sep) return kFallback;  // fewer fields than the schema names: the reference throws
    }
}

__host__ __device__ inline bool json_space(uint8_t c) { return c == ' ' || c == '\t' || c == '\r'; }
__host__ __device__ inline bool json_numch(uint8_t c) {
    return is_digit(c) || c == '-' || c == '+' || c == '.' || c == 'e' || c == 'E';
}

// GeoJSONToSpatial: the first coordinate of the first "coordinates" member (a Point's [x, y(, z)];
// for other geometries JTS getCoordinate() is also the first position of the nested arrays).
template <class R>
__host__ __device__ inline int parse_geojson(const R& rd, uint64_t p, Parsed* o) {
    const char key[] = "\"coordinates\"";
    for (;; p++) {
        const uint8_t c = rd(p);
        if (c == '\n') return kFallback;
        if (c != '"') continue;
        int k = 1;
        while (k < 13 && rd(p + k) == (uint8_t)key[k]) k++;
        if (k == 13) break;
    }
    p += 13;
    while (json_space(rd(p))) p++;
    if (rd(p) != ':') return kFallback;
    p++;
    while (json_space(rd(p))) p++;
    if (rd(p) != '[') return kFallback;
    do {
        p++;
        while (json_space(rd(p))) p++;
    } while (rd(p) == '[');
    uint64_t t = p;
    while (json_numch(rd(t))) t++;
    if (parse_decimal(rd, p, t, true, &o->x) != kOk) return kFallback;
    p = t;
    while (json_space(rd(p))) p++;
    if (rd(p) != ',') return kFallback;
    p++;
    while (json_space(rd(p))) p++;
    t = p;
    while (json_numch(rd(t))) t++;
    if (parse_decimal(rd, p, t, true, &o->y) != kOk) return kFallback;
    p = t;
    while (json_space(rd(p))) p++;
    const uint8_t c = rd(p);
    return (c == ']' || c == ',') ? kOk : kFallback;
}

// ---- GeoJSONToTSpatial (Deserialization.java:149-208): properties[propertyTimeStamp] through the
// DateFormat, properties[propertyObjID] as nodeOId.toString().replaceAll("\"", "").
// The record is the Kafka value object; Jackson's ObjectNode keeps the LAST member of a repeated
// key, so a later "properties" (or a later key inside it) replaces an earlier one.

// one JSON string at p ('"'): the end (past the closing quote) and whether it holds a backslash
template <class R>
__host__ __device__ inline bool json_string_end(const R& rd, uint64_t p, uint64_t* end, bool* esc) {
    *esc = false;
    for (p++;; p++) {
        const uint8_t c = rd(p);
        if (c == '\n') return false;
        if (c == '"') break;
        if (c == '\\') {
            *esc = true;
            if (rd(++p) == '\n') return false;
        }
    }
    *end = p + 1;
    return true;
}
// any JSON value at p: its end (nested containers by a depth count, strings skipped whole)
template <class R>
__host__ __device__ inline bool json_skip_value(const R& rd, uint64_t p, uint64_t* end) {
    const uint64_t p0 = p;
    int depth = 0;
    for (;;) {
        const uint8_t c = rd(p);
        if (c == '\n') return false;
        if (c == '"') {
            bool esc;
            if (!json_string_end(rd, p, &p, &esc)) return false;
        } else if (c == '{' || c == '[') {
            depth++;
            p++;
        } else if (c == '}' || c == ']') {
            if (depth == 0) break;  // the enclosing container's end
            depth--;
            p++;
        } else if (c == ',' && depth == 0) {
            break;
        } else {
            p++;
        }
        if (depth == 0 && (rd(p) == ',' || rd(p) == '}' || rd(p) == ']' || json_space(rd(p)))) break;
    }
    *end = p;
    return p != p0;  // an empty value is not JSON
}
template <class R>
__host__ __device__ inline uint64_t json_ws(const R& rd, uint64_t p) {
    while (json_space(rd(p))) p++;
    return p;
}
template <class R>
__host__ __device__ inline bool key_is(const R& rd, uint64_t a, uint64_t b, const char* k, int klen) {
    if (b - a != (uint64_t)klen) return false;
    for (int i = 0; i < klen; i++)
        if (rd(a + (uint64_t)i) != (uint8_t)k[i]) return false;
    return true;
}

// SimpleDateFormat("yyyy-MM-dd HH:mm:ss").parse (lenient, zone of fixed offset off_min) of the
// string s[a, b) (no escapes), as DateFormat.parse(String) then Date.getTime():
//   * 'yyyy-MM-dd HH:mm:ss' with exactly those digit counts (after ' ' / '\t', which subParse
//     skips), year 1583..9999 (Gregorian throughout), any 2-digit month / day / hour / minute /
//     second (the lenient calendar carries them over linearly), followed by the end or by an
//     ASCII character that cannot continue the seconds number -> the epoch milliseconds;
//   * nothing parseable at all (empty, or a first character that starts no number: ASCII, not a
//     digit, '-' or '+') -> ParseException, caught by the reference: 0;
//   * anything else (other digit counts, signs, non-ASCII, the other fields' leniencies) -> the
//     host.
__host__ __device__ inline int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
    y -= m <= 2 ? 1 : 0;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
template <class R>
__host__ __device__ inline int parse_date_ymd_hms(const R& rd, uint64_t a, uint64_t b, int32_t off_min, int64_t* ms) {
    while (a < b && (rd(a) == ' ' || rd(a) == '\t')) a++;
    if (a == b) {
        *ms = 0;
        return kOk;
    }
    const uint8_t c0 = rd(a);
    // ('N' could begin a NaN symbol DecimalFormat accepts: the host decides)
    if (c0 < 0x80 && !is_digit(c0) && c0 != '-' && c0 != '+' && c0 != 'N') {
        *ms = 0;
        return kOk;
    }
    const char pat[] = "dddd-dd-dd dd:dd:dd";
    if (b - a < 19) return kFallback;
    int64_t v[6] = {0, 0, 0, 0, 0, 0};
    int k = 0;
    for (int i = 0; i < 19; i++) {
        const uint8_t c = rd(a + (uint64_t)i);
        if (pat[i] == 'd') {
            if (!is_digit(c)) return kFallback;
            v[k] = v[k] * 10 + (c - '0');
        } else {
            if (c != (uint8_t)pat[i]) return kFallback;
            k++;
        }
    }
    if (b - a > 19) {
        const uint8_t c = rd(a + 19);
        if (c >= 0x80 || is_digit(c) || c == 'E' || c == 'e' || c == '.' || c == ',') return kFallback;
    }
    if (v[0] < 1583) return kFallback;
    // month carried into the year (month 0 = December of the year before), day 0 = the last day
    // of the month before, hours / minutes / seconds past their range carried forward
    const int64_t m0 = v[1] - 1;
    const int64_t y = v[0] + (m0 >= 0 ? m0 / 12 : -1);
    const int64_t m = (m0 % 12 + 12) % 12 + 1;
    const int64_t days = days_from_civil(y, m, 1) + v[2] - 1;
    const int64_t secs = ((days * 24 + v[3]) * 60 + v[4]) * 60 + v[5] - (int64_t)off_min * 60;
    *ms = secs * 1000;
    return kOk;
}

template <class R>
__host__ __device__ inline int parse_geojson_traj(const R& rd, uint64_t p, const Spec& sp, Parsed* o) {
    if (parse_geojson(rd, p, o) != kOk) return kFallback;
    o->ts = 0;
    o->oid = kOidNull;
    p = json_ws(rd, p);
    if (rd(p) != '{') return kFallback;
    p = json_ws(rd, p + 1);
    uint64_t ts_a = 0, ts_b = 0, oid_a = 0, oid_b = 0;  // value spans of the last "properties"
    bool ts_found = false, oid_found = false;
    for (;;) {
        if (rd(p) != '"') return kFallback;
        uint64_t ke;
        bool esc;
        if (!json_string_end(rd, p, &ke, &esc) || esc) return kFallback;  // escaped keys: the host
        const bool props = key_is(rd, p + 1, ke - 1, "properties", 10);
        p = json_ws(rd, ke);
        if (rd(p) != ':') return kFallback;
        p = json_ws(rd, p + 1);
        uint64_t ve;
        if (props) {
            ts_found = oid_found = false;  // this "properties" replaces any earlier one
            if (rd(p) == '{') {
                uint64_t q = json_ws(rd, p + 1);
                if (rd(q) != '}') {
                    for (;;) {
                        if (rd(q) != '"') return kFallback;
                        uint64_t k2;
                        if (!json_string_end(rd, q, &k2, &esc) || esc) return kFallback;
                        const bool is_ts = key_is(rd, q + 1, k2 - 1, sp.kts, sp.kts_len);
                        const bool is_oid = key_is(rd, q + 1, k2 - 1, sp.koid, sp.koid_len);
                        q = json_ws(rd, k2);
                        if (rd(q) != ':') return kFallback;
                        q = json_ws(rd, q + 1);
                        uint64_t e2;
                        if (!json_skip_value(rd, q, &e2)) return kFallback;
                        if (is_ts) {
                            ts_found = true;
                            ts_a = q;
                            ts_b = e2;
                        }
                        if (is_oid) {
                            oid_found = true;
                            oid_a = q;
                            oid_b = e2;
                        }
                        q = json_ws(rd, e2);
                        if (rd(q) == ',') {
                            q = json_ws(rd, q + 1);
                            continue;
                        }
                        if (rd(q) != '}') return kFallback;
                        break;
                    }
                }
                ve = q + 1;
            } else if (!json_skip_value(rd, p, &ve)) {
                return kFallback;
            }
        } else if (!json_skip_value(rd, p, &ve)) {
            return kFallback;
        }
        p = json_ws(rd, ve);
        if (rd(p) == ',') {
            p = json_ws(rd, p + 1);
            continue;
        }
        if (rd(p) != '}') return kFallback;
        break;
    }
    if (rd(json_ws(rd, p + 1)) != '\n') return kFallback;  // trailing text after the value
    if (ts_found && sp.date_fmt != 0) {
        // nodeTime.textValue(): a string's text, null (-> NullPointerException) for other nodes
        if (rd(ts_a) != '"') return kFallback;
        uint64_t e;
        bool esc;
        if (!json_string_end(rd, ts_a, &e, &esc) || esc || e != ts_b) return kFallback;
        if (parse_date_ymd_hms(rd, ts_a + 1, ts_b - 1, sp.utc_off_min, &o->ts) != kOk) return kFallback;
    }
    if (oid_found) {
        // toString() then every '"' deleted: a string's characters (no escapes, printable ASCII
        // here), an integer's digits, true / false / null as written; others -> the host
        const uint8_t c = rd(oid_a);
        uint64_t a = oid_a, b = oid_b;
        if (c == '"') {
            a++;
            b--;
            for (uint64_t t = a; t < b; t++) {
                const uint8_t ch = rd(t);
                if (ch < 0x20 || ch >= 0x7f || ch == '\\') return kFallback;
            }
        } else if (c == '-' || is_digit(c)) {
            uint64_t t = a + (c == '-' ? 1 : 0);
            if (t >= b || (rd(t) == '0' && (b - t > 1 || c == '-'))) return kFallback;  // "-0", leading zeros
            for (; t < b; t++)
                if (!is_digit(rd(t))) return kFallback;  // fractions, exponents: DoubleNode text differs
        } else if (!(key_is(rd, a, b, "true", 4) || key_is(rd, a, b, "false", 5) || key_is(rd, a, b, "null", 4))) {
            return kFallback;
        }
        if (b - a >= kMaxTokenLen) return kFallback;
        o->oid = (a << kOidLenBits) | (b - a);
    }
    return kOk;
}

// JTS WKTReader tokenizer word characters (a-z A-Z 0-9 - + . and 160-255)
__host__ __device__ inline bool wkt_word(uint8_t c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || is_digit(c) || c == '-' || c == '+' || c == '.' ||
           c >= 160;
}
template <class R>
__host__ __device__ inline uint64_t wkt_skip(const R& rd, uint64_t p) {
    for (;;) {
        const uint8_t c = rd(p);
        if (c > ' ' || c == '\n') return p;
        p++;
    }
}

// WKTReader.getNextNumber: a word equal to "NaN" ignoring case is NaN, else Double.parseDouble
template <class R>
__host__ __device__ inline int wkt_number(const R& rd, uint64_t s, uint64_t e, double* v) {
    if (e - s == 3 && (rd(s) | 32) == 'n' && (rd(s + 1) | 32) == 'a' && (rd(s + 2) | 32) == 'n') {
        *v = __builtin_bit_cast(double, 0x7ff8000000000000ull);
        return kOk;
    }
    return parse_decimal(rd, s, e, false, v);
}

// WKTToSpatial: "POINT" (first occurrence) then "(" x y [z] ")" (getPreciseCoordinate reads a
// third ordinate when a word follows; getCoordinate() keeps x and y).  POINT EMPTY and Z / M
// tags go to the host.
template <class R>
__host__ __device__ inline int parse_wkt(const R& rd, uint64_t p, Parsed* o) {
    for (;; p++) {
        const uint8_t c = rd(p);
        if (c == '\n') return kFallback;
        if (c == 'P' && rd(p + 1) == 'O' && rd(p + 2) == 'I' && rd(p + 3) == 'N' && rd(p + 4) == 'T') break;
    }
    p += 5;
    if (wkt_word(rd(p))) return kFallback;
    p = wkt_skip(rd, p);
    if (rd(p) != '(') return kFallback;
    p = wkt_skip(rd, p + 1);
    uint64_t t = p;
    while (wkt_word(rd(t))) t++;
    if (p == t || wkt_number(rd, p, t, &o->x) != kOk) return kFallback;
    p = wkt_skip(rd, t);
    if (p == t) return kFallback;  // the next token is not separated by blanks: ',' or ')' -> error
    t = p;
    while (wkt_word(rd(t))) t++;
    if (p == t || wkt_number(rd, p, t, &o->y) != kOk) return kFallback;
    p = wkt_skip(rd, t);
    if (wkt_word(rd(p))) {  // a third ordinate (z): read, validated, dropped
        if (p == t) return kFallback;
        t = p;
        while (wkt_word(rd(t))) t++;
        double z;
        if (wkt_number(rd, p, t, &z) != kOk) return kFallback;
        p = wkt_skip(rd, t);
    }
    return rd(p) == ')' ? kOk : kFallback;
}

template <class R>
__host__ __device__ inline int parse_record(const R& rd, uint64_t start, const Spec& sp, Parsed* o) {
    o->oid = kOidNull;
    if (sp.format == kCsv) return parse_csv(rd, start, sp, o);
    if (sp.format == kGeoJson) return sp.traj ? parse_geojson_traj(rd, start, sp, o) : parse_geojson(rd, start, o);
    return parse_wkt(rd, start, o);  // WKTToTSpatial: objID null, timestamp 0 as WKTToSpatial
}

// HelperClass.assignGridCellID axis index: (int)Math.floor((v - min) / cellLength)
__host__ __device__ inline int32_t java_cell(double v, double mn, double l) {
    const double f = __builtin_floor((v - mn) / l);
    if (f != f) return 0;
    if (f >= 2147483647.0) return 2147483647;
    if (f <= -2147483648.0) return (int32_t)0x80000000u;
    return (int32_t)f;
}

}  // namespace ingest
}  // namespace geohip
