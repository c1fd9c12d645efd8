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
// count when the 19-digit truncation decides the rounding), NaN/Infinity, Java type suffixes
// and the common record shapes -- and converts them with the Eisel-Lemire algorithm (correctly
// rounded, ties to even: the value Double.parseDouble returns).  Everything else returns
// kFallback and the batch call reports GEOHIP_ERR_UNSUPPORTED with the first such record:
// malformed text (where the reference throws NumberFormatException / IndexOutOfBounds) and the
// rare valid forms outside the device grammar (hex significands, 6+ digit exponents, quotes
// inside a token, ...).  The library has no CPU parsing path; the caller hands
// such a batch back to the reference's own Java deserializer, which parses it or throws.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ingest_pow5.h"

namespace geohip {
namespace ingest {

constexpr int kOk = 0;
constexpr int kFallback = 1;

enum Format { kCsv = 0, kGeoJson = 1, kWkt = 2 };

struct Spec {
    int32_t format;
    int32_t delim;  // CSV/TSV delimiter byte
    int32_t fx, fy;  // csvTsvSchemaAttr[2], [3]
    int32_t fts;     // csvTsvSchemaAttr[1] (Long.valueOf timestamp), < 0: not parsed
};

struct Parsed {
    double x, y;
    int64_t ts;
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

// Decimal token [s, e) -> double (correctly rounded, ties to even).
// json: RFC 8259 number grammar as Jackson reads it (no '+', no leading zeros, digits on both
//   sides of '.'); an integer token is an IntNode/LongNode, so "-0" is +0.0 and integers of
//   more than 18 digits (LongNode overflow, BigIntegerNode) go to kFallback.
// else: FloatingDecimal.readJavaFormatString's grammar on an already trimmed token: [+-]?
//   then "NaN" | "Infinity" | digits[.digits][(e|E)[+-]?digits][fFdD].  Hex significands and
//   exponents of 6+ digits -> kFallback.
// More than 19 significant digits: the token is truncated to 19 and converted at w and w + 1;
// equal results decide it (the true value lies between them), unequal -> kFallback.
template <class R>
__host__ __device__ inline int parse_decimal(const R& rd, uint64_t s, uint64_t e, bool json, double* out) {
    if (s >= e) return kFallback;
    uint64_t p = s;
    uint8_t c = rd(p);
    bool neg = false;
    if (c == '-' || (!json && c == '+')) {
        neg = c == '-';
        if (++p >= e) return kFallback;
        c = rd(p);
    }
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
            if (ne == 6) return kFallback;  // |exponent| >= 10^6: Java saturates; not decided here
            ev = ev * 10 + (c - '0');
            ne++;
            if (++p < e) c = rd(p);
        }
        if (ne == 0) return kFallback;
        q += eneg ? -ev : ev;
    }
    if (p < e && !json && (c == 'f' || c == 'F' || c == 'd' || c == 'D')) p++;  // type suffix
    if (p != e) return kFallback;  // hex, stray characters
    if (json && !frac && !expo) {
        if (nd > 18) return kFallback;
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

// Long.valueOf: [+-]?digits, no trim; 18 digits at most here (longer -> host range check)
template <class R>
__host__ __device__ inline int parse_long(const R& rd, uint64_t s, uint64_t e, int64_t* out) {
    if (s >= e) return kFallback;
    uint64_t p = s;
    const uint8_t c0 = rd(p);
    const bool neg = c0 == '-';
    if (c0 == '+' || c0 == '-') p++;
    if (p >= e || e - p > 18) return kFallback;
    int64_t v = 0;
    for (; p < e; p++) {
        const uint8_t c = rd(p);
        if (!is_digit(c)) return kFallback;
        v = v * 10 + (c - '0');
    }
    *out = neg ? -v : v;
    return kOk;
}

// CSVTSVToSpatial / CSVTSVToTSpatial.  Quotes are deleted before the split, so they never end a
// field; a separator is the delimiter with the \s runs around it (non-space delimiters) or a
// maximal run of \s / quotes that contains the delimiter (whitespace delimiters).  A field's
// number token is its text without surrounding chars <= ' ' or quotes (Double.valueOf trims).
// Long.valueOf does not trim: the timestamp field is rejected if \s survives the split around it
// (before field 0, after the last field) or if it holds any other control character.
template <class R>
__host__ __device__ inline int parse_csv(const R& rd, uint64_t p, const Spec& sp, Parsed* o) {
    int need = sp.fx > sp.fy ? sp.fx : sp.fy;
    if (sp.fts > need) need = sp.fts;
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
            if (t0 == ~0ull || parse_decimal(rd, t0, t1, false, &v) != kOk) return kFallback;
            if (f == sp.fx) o->x = v;
            if (f == sp.fy) o->y = v;
        }
        if (f == sp.fts && (ctrl || (f == 0 && lead) || (!sep && trail) || t0 == ~0ull ||
                            parse_long(rd, t0, t1, &o->ts) != kOk))
            return kFallback;
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

// WKTToSpatial: "POINT" (first occurrence) then "(" x y ")"; POINT EMPTY, Z / M tags, a third
// ordinate and NaN words go to the host.
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
    if (parse_decimal(rd, p, t, false, &o->x) != kOk) return kFallback;
    p = wkt_skip(rd, t);
    if (p == t) return kFallback;  // the next token is not separated by blanks: ',' or ')' -> error
    t = p;
    while (wkt_word(rd(t))) t++;
    if (parse_decimal(rd, p, t, false, &o->y) != kOk) return kFallback;
    p = wkt_skip(rd, t);
    return rd(p) == ')' ? kOk : kFallback;
}

template <class R>
__host__ __device__ inline int parse_record(const R& rd, uint64_t start, const Spec& sp, Parsed* o) {
    if (sp.format == kCsv) return parse_csv(rd, start, sp, o);
    if (sp.format == kGeoJson) return parse_geojson(rd, start, o);
    return parse_wkt(rd, start, o);
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
