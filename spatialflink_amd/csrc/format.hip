// format.hip -- point CSV/TSV output codec.
//
// The device form of Serialization.PointToCSVTSVOutputSchema.serialize
// (spatialStreams/Serialization.java:98-152) for a batch of result points: every record is
// written into one text buffer ('\n' after each record, record offsets on the side), the
// doubles through a restatement of JDK 8's Double.toString (sun.misc.FloatingDecimal
// .BinaryToASCIIBuffer: dtoa with estimateDecExp, developLongDigits, roundup, getChars).
// Parity unpinned: the restatement is checked against the Python restatement in
// oracle/jdk_double.py, not against a JVM (none runs here).
//
//   fmt_len    one thread per record: its byte length (every field formatted once)
//   scan       record offsets (3 small kernels)
//   fmt_write  one thread per record: the same formatting, bytes stored at its offset
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>

#include "geohip.h"
#include "join.h"

namespace geohip {
namespace {

constexpr int kFmtTB = 256;
constexpr int kBigLimbs = 40;  // 1280 bits: every B, S, M, 10 S of a double fits

// ---------------------------------------------------------------- small big integers -------
struct Big {
    uint32_t w[kBigLimbs];
    int n;  // used limbs
};
__device__ void big_set_u64(Big& a, uint64_t v) {
    a.w[0] = (uint32_t)v;
    a.w[1] = (uint32_t)(v >> 32);
    a.n = a.w[1] ? 2 : (a.w[0] ? 1 : 0);
}
__device__ void big_mul_small(Big& a, uint32_t m) {
    uint64_t c = 0;
    for (int i = 0; i < a.n; i++) {
        const uint64_t t = (uint64_t)a.w[i] * m + c;
        a.w[i] = (uint32_t)t;
        c = t >> 32;
    }
    if (c && a.n < kBigLimbs) a.w[a.n++] = (uint32_t)c;
}
__device__ void big_shl(Big& a, int s) {
    if (a.n == 0 || s == 0) return;
    const int ws = s / 32, bs = s % 32;
    int nn = a.n + ws + 1;
    if (nn > kBigLimbs) nn = kBigLimbs;
    for (int i = nn - 1; i >= 0; i--) {
        const int j = i - ws;
        uint32_t v = 0;
        if (j >= 0 && j < a.n) v = a.w[j] << bs;
        if (bs && j - 1 >= 0 && j - 1 < a.n) v |= a.w[j - 1] >> (32 - bs);
        a.w[i] = v;
    }
    a.n = nn;
    while (a.n > 0 && a.w[a.n - 1] == 0) a.n--;
}
__device__ void big_pow52(Big& a, uint64_t f, int p5, int p2) {  // f * 5^p5 * 2^p2
    big_set_u64(a, f);
    while (p5 >= 13) {
        big_mul_small(a, 1220703125u);  // 5^13
        p5 -= 13;
    }
    uint32_t r = 1;
    for (int i = 0; i < p5; i++) r *= 5u;
    big_mul_small(a, r);
    big_shl(a, p2);
}
__device__ int big_cmp(const Big& a, const Big& b) {
    if (a.n != b.n) return a.n > b.n ? 1 : -1;
    for (int i = a.n - 1; i >= 0; i--)
        if (a.w[i] != b.w[i]) return a.w[i] > b.w[i] ? 1 : -1;
    return 0;
}
__device__ void big_sub(Big& a, const Big& b) {  // a -= b, a >= b
    int64_t br = 0;
    for (int i = 0; i < a.n; i++) {
        int64_t t = (int64_t)a.w[i] - (i < b.n ? (int64_t)b.w[i] : 0) - br;
        br = t < 0;
        a.w[i] = (uint32_t)(t + (br << 32));
    }
    while (a.n > 0 && a.w[a.n - 1] == 0) a.n--;
}
__device__ void big_add(Big& r, const Big& a, const Big& b) {
    const int n = a.n > b.n ? a.n : b.n;
    uint64_t c = 0;
    for (int i = 0; i < n; i++) {
        const uint64_t t = (uint64_t)(i < a.n ? a.w[i] : 0) + (i < b.n ? b.w[i] : 0) + c;
        r.w[i] = (uint32_t)t;
        c = t >> 32;
    }
    r.n = n;
    if (c && r.n < kBigLimbs) r.w[r.n++] = (uint32_t)c;
}
// FDBigInteger.quoRemIteration: q = this / S, this = 10 * (this % S)
__device__ int big_quorem10(Big& b, const Big& s) {
    int q = 0;
    while (big_cmp(b, s) >= 0) {
        big_sub(b, s);
        q++;
    }
    big_mul_small(b, 10);
    return q;
}

// ---------------------------------------------------------------- JDK 8 Double.toString ------
__constant__ int kN5Bits[27] = {0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31, 33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61};
__constant__ int kInsignificant[64] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6,
                                       6, 6, 7, 7, 7, 8, 8, 8, 9, 9, 9, 9, 10, 10, 10, 11, 11, 11, 12, 12,
                                       12, 12, 13, 13, 13, 14, 14, 14, 15, 15, 15, 15, 16, 16, 16, 17, 17, 17,
                                       18, 18, 18, 19};

__device__ __forceinline__ uint64_t pow5_u64(int e) {
    uint64_t r = 1;
    for (int i = 0; i < e; i++) r *= 5u;
    return r;
}

// FloatingDecimal.estimateDecExp (fp64 in Java order: this file builds with -ffp-contract=off)
__device__ int estimate_dec_exp(uint64_t fract_bits, int bin_exp) {
    const double d2 = __longlong_as_double((long long)((1023ull << 52) | (fract_bits & ((1ull << 52) - 1))));
    const double d = (d2 - 1.5) * 0.289529654 + 0.176091259 + (double)bin_exp * 0.301029995663981;
    const uint64_t db = (uint64_t)__double_as_longlong(d);
    const int exponent = (int)((db >> 52) & 0x7ff) - 1023;
    const bool neg = (db >> 63) != 0;
    if (exponent >= 0 && exponent < 52) {
        const uint64_t mask = ((1ull << 52) - 1) >> exponent;
        const int r = (int)(((db & ((1ull << 52) - 1)) | (1ull << 52)) >> (52 - exponent));
        return neg ? (((mask & db) == 0) ? -r : -r - 1) : r;
    }
    if (exponent < 0) return ((db & ~(1ull << 63)) == 0) ? 0 : (neg ? -1 : 0);
    return (int)d;
}

struct Digits {
    char d[24];
    int n;
    int dec_exponent;
};

__device__ void fd_roundup(Digits& g) {
    int i = g.n - 1;
    char q = g.d[i];
    if (q == '9') {
        while (q == '9' && i > 0) {
            g.d[i] = '0';
            q = g.d[--i];
        }
        if (q == '9') {  // carry out: high-order 1, the rest already 0, one more decimal exponent
            g.dec_exponent += 1;
            g.d[0] = '1';
            return;
        }
    }
    g.d[i] = (char)(q + 1);
}

__device__ void fd_long_digits(Digits& g, int dec_exponent, uint64_t lvalue, int insignificant) {
    if (insignificant != 0) {
        uint64_t pow10 = 1;
        for (int i = 0; i < insignificant; i++) pow10 *= 10u;
        const uint64_t residue = lvalue % pow10;
        lvalue /= pow10;
        dec_exponent += insignificant;
        if (residue >= (pow10 >> 1)) lvalue++;
    }
    char tmp[24];
    int k = 0;
    int c = (int)(lvalue % 10);
    lvalue /= 10;
    while (c == 0) {
        dec_exponent++;
        c = (int)(lvalue % 10);
        lvalue /= 10;
    }
    while (lvalue != 0) {
        tmp[k++] = (char)('0' + c);
        dec_exponent++;
        c = (int)(lvalue % 10);
        lvalue /= 10;
    }
    tmp[k++] = (char)('0' + c);
    for (int i = 0; i < k; i++) g.d[i] = tmp[k - 1 - i];
    g.n = k;
    g.dec_exponent = dec_exponent + 1;
}

// BinaryToASCIIBuffer.dtoa (isCompatibleFormat = true): the int / long paths with Java's
// wrapping arithmetic and strict stopping tests, the big-integer path with its non-strict one.
template <typename T, typename U>
__device__ void fd_small(Digits& g, uint64_t fract_bits, int B5, int B2, int S5, int S2, int M5, int M2, int& dec_exp,
                         bool& low, bool& high, long long& ldd) {
    auto wrap = [](U v) { return (T)v; };
    T b = wrap((U)((U)fract_bits * (U)pow5_u64(B5)) << B2);
    const T s = wrap((U)pow5_u64(S5) << S2);
    T m = wrap((U)pow5_u64(M5) << M2);
    const T tens = wrap((U)s * 10u);
    int q = (int)(b / s);
    b = wrap((U)10u * (U)(b % s));
    m = wrap((U)m * 10u);
    low = b < m;
    high = wrap((U)b + (U)m) > tens;
    if (q == 0 && !high) dec_exp--;
    else g.d[g.n++] = (char)('0' + q);
    if (dec_exp < -3 || dec_exp >= 8) high = low = false;
    while (!low && !high && g.n < 23) {
        q = (int)(b / s);
        b = wrap((U)10u * (U)(b % s));
        m = wrap((U)m * 10u);
        if (m > 0) {
            low = b < m;
            high = wrap((U)b + (U)m) > tens;
        } else {  // m overflowed
            low = true;
            high = true;
        }
        g.d[g.n++] = (char)('0' + q);
    }
    ldd = (long long)wrap((U)wrap((U)b << 1) - (U)tens);
}

__device__ void fd_dtoa(Digits& g, int bin_exp, uint64_t fract_bits, int n_sig) {
    const int tail_zeros = __builtin_ctzll(fract_bits);
    const int n_fract_bits = 53 - tail_zeros;
    int n_tiny_bits = n_fract_bits - bin_exp - 1;
    if (n_tiny_bits < 0) n_tiny_bits = 0;
    g.n = 0;
    if (bin_exp <= 62 && bin_exp >= -21 && n_tiny_bits < 27 && n_fract_bits + kN5Bits[n_tiny_bits] < 64 &&
        n_tiny_bits == 0) {
        int ins = 0;
        if (bin_exp > n_sig) {
            const int p2 = bin_exp - n_sig - 1;
            ins = (p2 > 1 && p2 < 64) ? kInsignificant[p2] : 0;
        }
        const uint64_t fb = bin_exp >= 52 ? fract_bits << (bin_exp - 52) : fract_bits >> (52 - bin_exp);
        fd_long_digits(g, 0, fb, ins);
        return;
    }
    int dec_exp = estimate_dec_exp(fract_bits, bin_exp);
    int B5 = dec_exp < 0 ? -dec_exp : 0;
    int B2 = B5 + n_tiny_bits + bin_exp;
    const int S5 = dec_exp > 0 ? dec_exp : 0;
    int S2 = S5 + n_tiny_bits;
    const int M5 = B5;
    int M2 = B2 - n_sig;
    fract_bits >>= tail_zeros;
    B2 -= n_fract_bits - 1;
    const int common2 = B2 < S2 ? B2 : S2;
    B2 -= common2;
    S2 -= common2;
    M2 -= common2;
    if (n_fract_bits == 1) M2 -= 1;
    if (M2 < 0) {
        B2 -= M2;
        S2 -= M2;
        M2 = 0;
    }
    const int Bbits = n_fract_bits + B2 + (B5 < 27 ? kN5Bits[B5] : B5 * 3);
    const int tenSbits = S2 + 1 + ((S5 + 1) < 27 ? kN5Bits[S5 + 1] : (S5 + 1) * 3);
    bool low, high;
    long long ldd = 0;
    if (Bbits < 64 && tenSbits < 64) {
        if (Bbits < 32 && tenSbits < 32) fd_small<int32_t, uint32_t>(g, fract_bits, B5, B2, S5, S2, M5, M2, dec_exp, low, high, ldd);
        else fd_small<int64_t, uint64_t>(g, fract_bits, B5, B2, S5, S2, M5, M2, dec_exp, low, high, ldd);
    } else {
        Big S, B, M, T, tenS;
        big_pow52(S, 1, S5, S2);
        big_pow52(B, fract_bits, B5, B2);
        big_pow52(M, 1, M5 + 1, M2 + 1);
        big_pow52(tenS, 1, S5 + 1, S2 + 1);
        int q = big_quorem10(B, S);
        low = big_cmp(B, M) < 0;
        big_add(T, B, M);
        high = big_cmp(tenS, T) <= 0;
        if (q == 0 && !high) dec_exp--;
        else g.d[g.n++] = (char)('0' + q);
        if (dec_exp < -3 || dec_exp >= 8) high = low = false;
        while (!low && !high && g.n < 23) {
            q = big_quorem10(B, S);
            big_mul_small(M, 10);
            low = big_cmp(B, M) < 0;
            big_add(T, B, M);
            high = big_cmp(tenS, T) <= 0;
            g.d[g.n++] = (char)('0' + q);
        }
        if (high && low) {
            big_shl(B, 1);
            ldd = big_cmp(B, tenS);
        }
    }
    g.dec_exponent = dec_exp + 1;
    if (high) {
        if (low) {
            if (ldd == 0) {
                if ((g.d[g.n - 1] & 1) != 0) fd_roundup(g);
            } else if (ldd > 0) {
                fd_roundup(g);
            }
        } else {
            fd_roundup(g);
        }
    }
}

// Double.toString(v) into out (<= 26 bytes); returns the length
__device__ int java_double_to_string(double v, char* out) {
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    const bool neg = (bits >> 63) != 0;
    uint64_t fract = bits & ((1ull << 52) - 1);
    int bin_exp = (int)((bits >> 52) & 0x7ff);
    int i = 0;
    if (bin_exp == 0x7ff) {
        const char* s = fract ? "NaN" : (neg ? "-Infinity" : "Infinity");
        while (s[i]) {
            out[i] = s[i];
            i++;
        }
        return i;
    }
    int n_sig;
    if (bin_exp == 0) {
        if (fract == 0) {
            const char* s = neg ? "-0.0" : "0.0";
            while (s[i]) {
                out[i] = s[i];
                i++;
            }
            return i;
        }
        const int lz = __builtin_clzll(fract);
        const int shift = lz - (63 - 52);
        fract <<= shift;
        bin_exp = 1 - shift;
        n_sig = 64 - lz;
    } else {
        fract |= 1ull << 52;
        n_sig = 53;
    }
    bin_exp -= 1023;
    Digits g;
    fd_dtoa(g, bin_exp, fract, n_sig);
    // getChars
    if (neg) out[i++] = '-';
    const int de = g.dec_exponent, nd = g.n;
    if (de > 0 && de < 8) {
        const int cl = nd < de ? nd : de;
        for (int t = 0; t < cl; t++) out[i++] = g.d[t];
        if (cl < de) {
            for (int t = 0; t < de - cl; t++) out[i++] = '0';
            out[i++] = '.';
            out[i++] = '0';
        } else {
            out[i++] = '.';
            if (cl < nd) {
                for (int t = cl; t < nd; t++) out[i++] = g.d[t];
            } else {
                out[i++] = '0';
            }
        }
    } else if (de <= 0 && de > -3) {
        out[i++] = '0';
        out[i++] = '.';
        for (int t = 0; t < -de; t++) out[i++] = '0';
        for (int t = 0; t < nd; t++) out[i++] = g.d[t];
    } else {
        out[i++] = g.d[0];
        out[i++] = '.';
        if (nd > 1) {
            for (int t = 1; t < nd; t++) out[i++] = g.d[t];
        } else {
            out[i++] = '0';
        }
        out[i++] = 'E';
        int e;
        if (de <= 0) {
            out[i++] = '-';
            e = -de + 1;
        } else {
            e = de - 1;
        }
        if (e <= 9) {
            out[i++] = (char)('0' + e);
        } else if (e <= 99) {
            out[i++] = (char)('0' + e / 10);
            out[i++] = (char)('0' + e % 10);
        } else {
            out[i++] = (char)('0' + e / 100);
            e %= 100;
            out[i++] = (char)('0' + e / 10);
            out[i++] = (char)('0' + e % 10);
        }
    }
    return i;
}

// Long.toString
__device__ int java_long_to_string(long long v, char* out) {
    char tmp[24];
    int k = 0, i = 0;
    unsigned long long a = v < 0 ? 0ull - (unsigned long long)v : (unsigned long long)v;
    do {
        tmp[k++] = (char)('0' + (int)(a % 10));
        a /= 10;
    } while (a);
    if (v < 0) out[i++] = '-';
    while (k) out[i++] = tmp[--k];
    return i;
}

constexpr int kMaxPos = 64;
// record flags raised by the formatting kernels (the host turns them into status codes)
constexpr unsigned kFlagIdx = 1u;       // idx[j] >= n: no such point (GEOHIP_ERR_ARG)
constexpr unsigned kFlagNonFinite = 2u; // GeoJSON of a NaN / infinite coordinate: the reference's
                                        // JSONObject.toString returns null (GEOHIP_ERR_ARG)
constexpr unsigned kFlagDate = 4u;      // a nonzero timestamp the date formatter cannot render
                                        // (no formatter named, or outside years 1583..9999)
struct FmtArgs {
    const double* x;
    const double* y;
    uint64_t n;                   // points: idx[j] < n
    const long long* ts;          // nullable: 0
    const unsigned char* oid;     // nullable: objID == null
    const unsigned long long* oid_off;
    const unsigned* idx;          // nullable: record j = point j
    uint64_t m;
    int format;                   // GEOHIP_FMT_CSV / _GEOJSON / _WKT
    int8_t field[kMaxPos];        // CSV: per position 0 objID, 1 ts, 2 x, 3 y, -1 "0"
    int npos;
    char delim[8];                // the SEPARATION string (UTF-8)
    int dlen;
    int csv_tail;                 // CSV: bytes of the last delimiter kept by deleteCharAt
    int csv_tail_q;               //      1: a '?' follows them (a lone high surrogate, UTF-8 encoded)
    int date;                     // GEOHIP_DATE_*
    long long off_ms;             // the formatter's fixed zone offset
    unsigned* flags;
};

// byte sink: WRITE = false only counts
template <bool WRITE>
struct Sink {
    unsigned char* dst;
    uint64_t len;
    __device__ void put(char c) {
        if (WRITE) dst[len] = (unsigned char)c;
        len++;
    }
    __device__ void put(const char* s, int n) {
        for (int t = 0; t < n; t++) put(s[t]);
    }
    __device__ void lit(const char* s) {
        while (*s) put(*s++);
    }
};

// SimpleDateFormat("yyyy-MM-dd HH:mm:ss") of a Date in a fixed-offset zone (proleptic Gregorian
// civil date, exact from the 1582-10-15 cutover on; callers keep to years 1583..9999)
__device__ bool format_ymd_hms(long long ms, long long off_ms, char* out) {
    const long long t = ms + off_ms;
    long long sec = t / 1000;
    if (t % 1000 < 0) sec--;
    long long days = sec / 86400;
    long long sod = sec - days * 86400;
    if (sod < 0) {
        sod += 86400;
        days--;
    }
    // civil_from_days (H. Hinnant)
    const long long z = days + 719468;
    const long long era = (z >= 0 ? z : z - 146096) / 146097;
    const long long doe = z - era * 146097;
    const long long yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    long long yr = yoe + era * 400;
    const long long doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const long long mp = (5 * doy + 2) / 153;
    const long long d = doy - (153 * mp + 2) / 5 + 1;
    const long long mo = mp < 10 ? mp + 3 : mp - 9;
    if (mo <= 2) yr++;
    if (yr < 1583 || yr > 9999) return false;
    const long long hh = sod / 3600, mi = (sod / 60) % 60, ss = sod % 60;
    const long long v[6] = {yr, mo, d, hh, mi, ss};
    const char sep[6] = {'-', '-', ' ', ':', ':', 0};
    int i = 0;
    for (int f = 0; f < 6; f++) {
        if (f == 0) {
            out[i++] = (char)('0' + yr / 1000);
            out[i++] = (char)('0' + (yr / 100) % 10);
        }
        out[i++] = (char)('0' + (v[f] / 10) % 10);
        out[i++] = (char)('0' + v[f] % 10);
        if (sep[f]) out[i++] = sep[f];
    }
    return true;  // 19 characters
}

// org.json JSONObject.numberToString(Double): Double.toString, trailing zeros (and then the
// point) shaved when there is a '.' and no exponent
__device__ int json_number(double v, char* out) {
    int n = java_double_to_string(v, out);
    bool dot = false, ex = false;
    for (int t = 0; t < n; t++) {
        dot = dot || out[t] == '.';
        ex = ex || out[t] == 'E' || out[t] == 'e';
    }
    if (dot && !ex) {
        while (out[n - 1] == '0') n--;
        if (out[n - 1] == '.') n--;
    }
    return n;
}

// org.json JSONObject.quote of a String given as UTF-8 bytes (decoded to the UTF-16 units it
// compares): \\ \" and </ escaped, \b \t \n \f \r, \\u00XX below ' ', in [U+0080, U+00A0) and
// \\u20XX in [U+2000, U+2100), lowercase hex; every other byte as is
template <bool WRITE>
__device__ void json_quote(Sink<WRITE>& s, const unsigned char* b, uint64_t n) {
    s.put('"');
    unsigned prev = 0;
    const char* hx = "0123456789abcdef";
    for (uint64_t t = 0; t < n;) {
        const unsigned c0 = b[t];
        unsigned cp = c0;
        int len = 1;
        if (c0 >= 0xC0 && c0 < 0xE0 && t + 1 < n) {
            cp = ((c0 & 0x1Fu) << 6) | (b[t + 1] & 0x3Fu);
            len = 2;
        } else if (c0 >= 0xE0 && c0 < 0xF0 && t + 2 < n) {
            cp = ((c0 & 0x0Fu) << 12) | ((b[t + 1] & 0x3Fu) << 6) | (b[t + 2] & 0x3Fu);
            len = 3;
        } else if (c0 >= 0xF0 && t + 3 < n) {
            cp = 0x10000u;  // a surrogate pair in Java: never escaped
            len = 4;
        }
        if (cp == '\\' || cp == '"') {
            s.put('\\');
            s.put((char)cp);
        } else if (cp == '/') {
            if (prev == '<') s.put('\\');
            s.put('/');
        } else if (cp == '\b') {
            s.lit("\\b");
        } else if (cp == '\t') {
            s.lit("\\t");
        } else if (cp == '\n') {
            s.lit("\\n");
        } else if (cp == '\f') {
            s.lit("\\f");
        } else if (cp == '\r') {
            s.lit("\\r");
        } else if (cp < 0x20 || (cp >= 0x80 && cp < 0xA0) || (cp >= 0x2000 && cp < 0x2100)) {
            s.lit("\\u");
            s.put(hx[(cp >> 12) & 15]);
            s.put(hx[(cp >> 8) & 15]);
            s.put(hx[(cp >> 4) & 15]);
            s.put(hx[cp & 15]);
        } else {
            for (int q = 0; q < len; q++) s.put((char)b[t + q]);
        }
        prev = cp;
        t += (uint64_t)len;
    }
    s.put('"');
}

// the record of point p; returns its length (0 and a flag where the reference would throw)
template <bool WRITE>
__device__ uint64_t fmt_record(const FmtArgs& a, uint64_t p, unsigned char* dst) {
    Sink<WRITE> s{dst, 0};
    char buf[32];
    const long long ts = a.ts ? a.ts[p] : 0ll;
    // bit 63 of oid_off[p]: this point's objID is null (offsets are the low 63 bits)
    constexpr unsigned long long kOffMask = ~(1ull << 63);
    const bool has_oid = a.oid != nullptr && !(a.oid_off[p] >> 63);
    const uint64_t ob = has_oid ? (a.oid_off[p] & kOffMask) : 0, oe = has_oid ? (a.oid_off[p + 1] & kOffMask) : 0;
    char date[20];
    if (a.format != GEOHIP_FMT_CSV && ts != 0) {
        if (a.date != GEOHIP_DATE_YMD_HMS || !format_ymd_hms(ts, a.off_ms, date)) {
            if (!WRITE) atomicOr(a.flags, kFlagDate);
            return 0;
        }
    }
    if (a.format == GEOHIP_FMT_WKT) {
        // PointToWKTOutputSchema.serialize (Serialization.java:72-92)
        s.put('"');
        if (has_oid) {
            for (uint64_t t = ob; t < oe; t++) s.put((char)a.oid[t]);
            s.put(a.delim, a.dlen);
            s.put(' ');
        }
        s.lit("POINT(");
        s.put(buf, java_double_to_string(a.x[p], buf));
        s.put(' ');
        s.put(buf, java_double_to_string(a.y[p], buf));
        s.put(')');
        if (ts != 0) {
            s.put(a.delim, a.dlen);
            s.put(' ');
            s.put(date, 19);
        }
        s.put('"');
        s.put(a.delim, a.dlen);
    } else if (a.format == GEOHIP_FMT_GEOJSON) {
        // PointToGeoJSONOutputSchema.serialize (Serialization.java:28-50): org.json HashMap
        // iteration order of the fixed keys (Java 8, 16 buckets, (h ^ h >>> 16) & 15):
        // geometry 10, type 12, properties 14; coordinates 8, type 12; oID 11, timestamp 15
        const double px = a.x[p], py = a.y[p];
        if (!__builtin_isfinite(px) || !__builtin_isfinite(py)) {
            if (!WRITE) atomicOr(a.flags, kFlagNonFinite);
            return 0;
        }
        s.lit("{\"geometry\":{\"coordinates\":[");
        s.put(buf, json_number(px, buf));
        s.put(',');
        s.put(buf, json_number(py, buf));
        s.lit("],\"type\":\"Point\"},\"type\":\"Feature\"");
        if (has_oid || ts != 0) {
            s.lit(",\"properties\":{");
            if (has_oid) {
                s.lit("\"oID\":");
                json_quote(s, a.oid + ob, oe - ob);
            }
            if (ts != 0) {
                if (has_oid) s.put(',');
                s.lit("\"timestamp\":\"");
                s.put(date, 19);
                s.put('"');
            }
            s.put('}');
        }
        s.put('}');
    } else {
        // PointToCSVTSVOutputSchema.serialize (Serialization.java:125-150)
        for (int pos = 0; pos < a.npos; pos++) {
            const int f = a.field[pos];
            if (f == 0) {
                if (has_oid) {
                    for (uint64_t t = ob; t < oe; t++) s.put((char)a.oid[t]);
                } else {
                    s.lit("null");
                }
            } else if (f == 1) {
                s.put(buf, java_long_to_string(ts, buf));
            } else if (f == 2) {
                s.put(buf, java_double_to_string(a.x[p], buf));
            } else if (f == 3) {
                s.put(buf, java_double_to_string(a.y[p], buf));
            } else {
                s.put('0');
            }
            // the delimiter after every field; deleteCharAt(length - 1) drops the record's last
            // UTF-16 unit: the last delimiter's last character (a '?' stays for the high half
            // of a supplementary one)
            if (pos + 1 < a.npos) {
                s.put(a.delim, a.dlen);
            } else {
                s.put(a.delim, a.csv_tail);
                if (a.csv_tail_q) s.put('?');
            }
        }
    }
    s.put('\n');
    return s.len;
}

__device__ __forceinline__ bool fmt_point(const FmtArgs& a, uint64_t j, uint64_t* p) {
    *p = a.idx ? a.idx[j] : j;
    return *p < a.n;
}

__global__ __launch_bounds__(kFmtTB) void fmt_len(FmtArgs a, unsigned long long* __restrict__ len) {
    const uint64_t j = (uint64_t)blockIdx.x * kFmtTB + threadIdx.x;
    if (j >= a.m) return;
    uint64_t p;
    if (!fmt_point(a, j, &p)) {  // e.g. a padded kNN list's sentinel: no such point
        atomicOr(a.flags, kFlagIdx);
        len[j] = 0;
        return;
    }
    len[j] = fmt_record<false>(a, p, nullptr);
}

// exclusive scan of len[0..m) into off[0..m] (off[m] = total): per-block sums, one block over
// them, per-block rescan
__global__ __launch_bounds__(kFmtTB) void fmt_scan_blocks(const unsigned long long* __restrict__ len, uint64_t m,
                                                          unsigned long long* __restrict__ bsum) {
    __shared__ unsigned long long sh[kFmtTB];
    const uint64_t j = (uint64_t)blockIdx.x * kFmtTB + threadIdx.x;
    sh[threadIdx.x] = j < m ? len[j] : 0ull;
    __syncthreads();
    for (int s = kFmtTB / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = sh[0];
}
__global__ __launch_bounds__(1) void fmt_scan_top(unsigned long long* __restrict__ bsum, uint64_t nb,
                                                  unsigned long long* __restrict__ total) {
    unsigned long long run = 0;
    for (uint64_t b = 0; b < nb; b++) {
        const unsigned long long v = bsum[b];
        bsum[b] = run;
        run += v;
    }
    *total = run;
}
__global__ __launch_bounds__(kFmtTB) void fmt_scan_apply(const unsigned long long* __restrict__ len, uint64_t m,
                                                         const unsigned long long* __restrict__ bsum,
                                                         const unsigned long long* __restrict__ total,
                                                         unsigned long long* __restrict__ off) {
    __shared__ unsigned long long sh[kFmtTB];
    const uint64_t j = (uint64_t)blockIdx.x * kFmtTB + threadIdx.x;
    sh[threadIdx.x] = j < m ? len[j] : 0ull;
    __syncthreads();
    for (int s = 1; s < kFmtTB; s <<= 1) {  // inclusive Hillis-Steele
        const unsigned long long v = (int)threadIdx.x >= s ? sh[threadIdx.x - s] : 0ull;
        __syncthreads();
        sh[threadIdx.x] += v;
        __syncthreads();
    }
    if (j < m) off[j] = bsum[blockIdx.x] + sh[threadIdx.x] - len[j];
    if (j == 0) off[m] = *total;
}

__global__ __launch_bounds__(kFmtTB) void fmt_write(FmtArgs a, const unsigned long long* __restrict__ off,
                                                    unsigned char* __restrict__ out, uint64_t cap) {
    const uint64_t j = (uint64_t)blockIdx.x * kFmtTB + threadIdx.x;
    if (j >= a.m) return;
    if (off[j + 1] > cap || off[j + 1] == off[j]) return;  // the whole record must fit; flagged ones are empty
    uint64_t p;
    if (!fmt_point(a, j, &p)) return;
    (void)fmt_record<true>(a, p, out + off[j]);
}

// bytes of the last UTF-8 sequence of s[0, n) (0: malformed)
int utf8_last_len(const char* s, int n) {
    int b = n - 1;
    while (b > 0 && ((unsigned char)s[b] & 0xC0u) == 0x80u) b--;
    const unsigned c = (unsigned char)s[b];
    const int want = c < 0x80 ? 1 : (c >= 0xC0 && c < 0xE0) ? 2 : (c >= 0xE0 && c < 0xF0) ? 3 : (c >= 0xF0 && c < 0xF8) ? 4 : 0;
    return want == n - b ? want : 0;
}

}  // namespace

int format_points_impl(geohip_ctx* ctx, const geohip_text_out_spec* spec, const double* x, const double* y, uint64_t n,
                       const int64_t* ts, const uint8_t* oid_text, const uint64_t* oid_off, const uint32_t* idx,
                       uint64_t m, uint8_t* out, uint64_t cap, uint64_t* out_len, uint64_t* rec_off) {
    if (!spec || !out_len) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null spec / out_len");
    *out_len = 0;
    if (ctx_mem(ctx) != GEOHIP_MEM_DEVICE) return ctx_fail(ctx, GEOHIP_ERR_ARG, "format_points needs GEOHIP_MEM_DEVICE");
    if (spec->format != GEOHIP_FMT_CSV && spec->format != GEOHIP_FMT_GEOJSON && spec->format != GEOHIP_FMT_WKT)
        return ctx_fail(ctx, GEOHIP_ERR_ARG, "unknown output format");
    if (spec->format != GEOHIP_FMT_GEOJSON && (spec->delim_len < 1 || spec->delim_len > 8))
        return ctx_fail(ctx, GEOHIP_ERR_ARG, "delimiter length must be 1..8");
    if (spec->date_format != GEOHIP_DATE_NONE && spec->date_format != GEOHIP_DATE_YMD_HMS)
        return ctx_fail(ctx, GEOHIP_ERR_ARG, "unknown date format");
    if (spec->utc_offset_min < -24 * 60 || spec->utc_offset_min > 24 * 60)
        return ctx_fail(ctx, GEOHIP_ERR_ARG, "utc offset outside +-24 h");
    if (m && (!x || !y)) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null x / y");
    if ((oid_text == nullptr) != (oid_off == nullptr)) return ctx_fail(ctx, GEOHIP_ERR_ARG, "oid_text and oid_off go together");
    if (cap && !out) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out");
    if (!idx && m > n) return ctx_fail(ctx, GEOHIP_ERR_ARG, "m > n without idx");
    FmtArgs a;
    memset(&a, 0, sizeof a);
    a.format = spec->format;
    if (spec->format == GEOHIP_FMT_CSV) {
        // positionMap (Serialization.java:117-120): later fields win a shared position
        const int32_t attrs[4] = {spec->attr_oid, spec->attr_ts, spec->attr_x, spec->attr_y};
        int maxp = -1;
        for (int k = 0; k < 4; k++) {
            if (attrs[k] < 0 || attrs[k] >= kMaxPos) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "schema positions must be 0..63");
            maxp = attrs[k] > maxp ? attrs[k] : maxp;
        }
        for (int p = 0; p < kMaxPos; p++) a.field[p] = -1;
        for (int k = 0; k < 4; k++) a.field[attrs[k]] = (int8_t)k;
        a.npos = maxp + 1;
        const int last = utf8_last_len(spec->delim, spec->delim_len);
        if (!last) return ctx_fail(ctx, GEOHIP_ERR_ARG, "delimiter is not UTF-8");
        a.csv_tail = spec->delim_len - last;
        a.csv_tail_q = last == 4 ? 1 : 0;
    }
    if (spec->format != GEOHIP_FMT_GEOJSON) {
        memcpy(a.delim, spec->delim, 8);
        a.dlen = spec->delim_len;
    }
    a.date = spec->date_format;
    a.off_ms = (long long)spec->utc_offset_min * 60000ll;
    a.x = x;
    a.y = y;
    a.n = n;
    a.ts = reinterpret_cast<const long long*>(ts);
    a.oid = oid_text;
    a.oid_off = reinterpret_cast<const unsigned long long*>(oid_off);
    a.idx = idx;
    a.m = m;
    hipStream_t st = ctx_stream(ctx);
    const uint64_t nb = (m + kFmtTB - 1) / kFmtTB;
    void *pl = nullptr, *po = nullptr, *pb = nullptr;
    int rc = ctx_ensure(ctx, 0, 8 * (m + 1), &pl);
    if (!rc) rc = ctx_ensure(ctx, 1, 8 * (m + 2), &po);
    if (!rc) rc = ctx_ensure(ctx, 2, 8 * (nb + 4), &pb);
    if (rc) return rc;
    unsigned long long* len = reinterpret_cast<unsigned long long*>(pl);
    unsigned long long* off = rec_off ? reinterpret_cast<unsigned long long*>(rec_off) : reinterpret_cast<unsigned long long*>(po);
    unsigned long long* bsum = reinterpret_cast<unsigned long long*>(pb);
    unsigned long long* total = bsum + nb + 1;  // total, then the flags word
    a.flags = reinterpret_cast<unsigned*>(total + 1);
    if (hipMemsetAsync(total, 0, 16, st) != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    if (m) {
        fmt_len<<<(unsigned)nb, kFmtTB, 0, st>>>(a, len);
        fmt_scan_blocks<<<(unsigned)nb, kFmtTB, 0, st>>>(len, m, bsum);
        fmt_scan_top<<<1, 1, 0, st>>>(bsum, nb, total);
        fmt_scan_apply<<<(unsigned)nb, kFmtTB, 0, st>>>(len, m, bsum, total, off);
        if (cap) fmt_write<<<(unsigned)nb, kFmtTB, 0, st>>>(a, off, out, cap);
    } else if (hipMemsetAsync(off, 0, 8, st) != hipSuccess) {
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("format launch: ") + hipGetErrorString(e));
    uint64_t* pin = ctx_pinned(ctx);
    if (hipMemcpyAsync(pin, total, 16, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "length readback failed");
    const unsigned flags = (unsigned)(pin[1] & 0xffffffffu);
    *out_len = pin[0];
    if (flags & kFlagIdx) return ctx_fail(ctx, GEOHIP_ERR_ARG, "idx entry >= n (no such point; e.g. a kNN sentinel)");
    if (flags & kFlagNonFinite)
        return ctx_fail(ctx, GEOHIP_ERR_ARG, "GeoJSON of a non-finite coordinate (JSONObject.toString throws)");
    if (flags & kFlagDate)
        return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "a nonzero timestamp needs GEOHIP_DATE_YMD_HMS and years 1583..9999");
    if (pin[0] > cap) return ctx_fail(ctx, GEOHIP_ERR_CAPACITY, "output capacity too small; *out_len = required");
    return GEOHIP_OK;
}

int format_csv_impl(geohip_ctx* ctx, const geohip_csv_out_spec* spec, const double* x, const double* y, uint64_t n,
                    const int64_t* ts, const uint8_t* oid_text, const uint64_t* oid_off, const uint32_t* idx,
                    uint64_t m, uint8_t* out, uint64_t cap, uint64_t* out_len, uint64_t* rec_off) {
    if (!spec || !out_len) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null spec / out_len");
    geohip_text_out_spec t;
    memset(&t, 0, sizeof t);
    t.format = GEOHIP_FMT_CSV;
    t.attr_oid = spec->attr_oid;
    t.attr_ts = spec->attr_ts;
    t.attr_x = spec->attr_x;
    t.attr_y = spec->attr_y;
    t.delim_len = spec->delim_len;
    memcpy(t.delim, spec->delim, 8);
    return format_points_impl(ctx, &t, x, y, n, ts, oid_text, oid_off, idx, m, out, cap, out_len, rec_off);
}

}  // namespace geohip
