// ingest.hip -- gfx950 kernels of the ingest codec: a batch of
// '\n'-separated CSV/TSV, GeoJSON or WKT point records -> SoA x[], y[] (+ timestamp, + cell).
//
// Replaces the per-record map functions of Deserialization.PointStream / TrajectoryStream
// (/root/reference/src/main/java/GeoFlink/spatialStreams/Deserialization.java:47-62, 64-80;
// CSVTSVToSpatial :248-254, CSVTSVToTSpatial :306-321, GeoJSONToSpatial :132-146,
// WKTToSpatial :223-228) and the cell assignment of the Point constructor
// (spatialObjects/Point.java:60-66 -> utils/HelperClass.java:104-116).
//
// One launch per batch (ingest_fused), HBM-streaming: every block takes the next 16 KB chunk by
// an arrival ticket, stages it (+ a 512-byte tail for the record straddling its end) in LDS with
// 16-byte loads, lists the record starts it owns in order (SWAR '\n' test + block scan),
// publishes its record count and finds its first record's index by a decoupled look-back over
// the earlier chunks' published counts (the record index of a record is its position in the
// batch, as in the arrival-ordered stream), then parses one record per lane with the
// ingest_parse.h functions (Eisel-Lemire fp64) and writes x/y/ts/cell coalesced by record index.
// The text is read once (+3 % for the tails); the count pass and scan launch of the earlier
// three-launch form, which read the text twice, are gone.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "ingest.h"
#include "join.h"

namespace geohip {
namespace {

constexpr int kThreads = 512;
constexpr unsigned kGeneralBlocks = 256;               // ingest_general's grid (strides over its list)
constexpr uint32_t kBytesPerThread = kIngestChunk / kThreads;  // 16-byte loads per thread: kLoads
constexpr int kLoads = (int)(kBytesPerThread / 16);
static_assert(kBytesPerThread % 16 == 0 && kLoads >= 2 && kLoads <= 4, "chunk layout");
static_assert(kIngestChunk + kIngestTail < 65536, "record starts are u16 offsets into the staged chunk");

// bit 7 of each byte set iff that byte of w is '\n' (exact: no borrow between bytes)
__device__ __forceinline__ uint32_t nl_bits(uint32_t w) {
    const uint32_t t = w ^ 0x0a0a0a0au;
    return ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t | 0x7f7f7f7fu);
}

// 16 bytes at text[p..p+16) (bytes at or past nbytes read as 0)
__device__ __forceinline__ uint4 load16(const uint8_t* text, uint64_t p, uint64_t nbytes) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    if (p + 16 <= nbytes) {  // plain loads: the next chunk's block reads this chunk's staged tail
                             // again from L2 (nontemporal loads: 426 against 405 us, same box)
        const v4u v = *reinterpret_cast<const v4u*>(text + p);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    uint32_t w[4] = {0, 0, 0, 0};
    for (int i = 0; i < 16; i++)
        if (p + i < nbytes) w[i >> 2] |= (uint32_t)text[p + i] << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// '\n' mask of the kBytesPerThread bytes starting at p (bit i = byte p + i); only positions < lim count
__device__ __forceinline__ uint64_t nl_mask(const uint4 (&v)[kLoads], uint64_t p, uint64_t lim) {
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < kLoads; j++) {
        const uint32_t wv[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t z = nl_bits(wv[k]);
            // gather bits 7, 15, 23, 31 into bits 4k .. 4k+3 of this load's 16
            const uint32_t g = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
            m |= (uint64_t)g << (16 * j + 4 * k);
        }
    }
    if (p + kBytesPerThread > lim) m &= p >= lim ? 0ull : ((1ull << (uint32_t)(lim - p)) - 1ull);
    return m;
}

// block-wide exclusive scan of one value per thread; returns the exclusive prefix, *total = sum
__device__ __forceinline__ unsigned block_excl_scan(unsigned v, unsigned* s_wave, unsigned* total) {
    const unsigned incl = wave_incl_scan(v);
    const int lane = lane_id(), wid = threadIdx.x / kWave;
    if (lane == kWave - 1) s_wave[wid] = incl;
    __syncthreads();
    unsigned base = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < kThreads / kWave; w++) {
        const unsigned s = s_wave[w];
        base += w < wid ? s : 0u;
        sum += s;
    }
    *total = sum;
    return base + incl - v;
}

// byte reader for the parsers: the staged LDS window first, global memory past it, and '\n'
// past the end of the batch (every parser stops at '\n')
struct LdsReader {
    const uint8_t* lds;
    uint64_t base;
    uint32_t len;
    const uint8_t* g;
    uint64_t n;
    __device__ __forceinline__ uint8_t operator()(uint64_t p) const {
        const uint64_t o = p - base;
        if (o < len) return lds[o];
        return p < n ? g[p] : (uint8_t)'\n';
    }
};

// CSV fast path over the staged bytes (LDS offsets, no bounds fallback to global memory): the
// common record shape -- no blanks, control characters or quotes up to the last field the schema
// names, numeric fields '-'? digits ('.' digits)? with at most 19 significant digits, the
// timestamp '-'? digits (<= 18).  On that subset ingest::parse_csv splits the same fields and
// computes the same (w, q) decimal (so the same Eisel-Lemire bits) and Long; anything else --
// or a record running past the staged bytes -- returns kFallback and takes the general parser.
// One pass, 32-bit offsets and few branches per byte: the general parser is SALU-bound on
// divergent per-byte control flow.
// The objID field (foid, not one of the number fields) is its bytes up to the delimiter: no
// blanks or quotes, so the span is the field as staged; empty -> kFallback.  c0: the chunk's text
// offset (spans are batch offsets).
__device__ __forceinline__ int fast_csv(const uint8_t* __restrict__ s, uint32_t p, uint32_t lim,
                                        const ingest::Spec& sp, ingest::Parsed* o, uint64_t c0) {
    const uint8_t d = (uint8_t)sp.delim;
    int need = sp.fx > sp.fy ? sp.fx : sp.fy;
    if (sp.fts > need) need = sp.fts;
    if (sp.foid > need) need = sp.foid;
    for (int f = 0; f <= need; f++) {
        const bool isx = f == sp.fx, isy = f == sp.fy, ist = f == sp.fts;
        if (isx || isy || ist) {
            if (p >= lim || ((isx || isy) && ist) || f == sp.foid) return ingest::kFallback;
            const bool neg = s[p] == '-';
            p += neg ? 1u : 0u;
            uint64_t w = 0;
            int32_t q = 0;
            int nd = 0, ni = 0, nf = 0;
            bool dot = false, bad = false;
            uint8_t c = 0;
            for (; p < lim; p++) {
                c = s[p];
                const unsigned dg = (unsigned)c - '0';
                if (dg < 10u) {
                    const bool take = nd != 0 || dg != 0;
                    bad |= take && nd == 19;
                    w = take && nd < 19 ? w * 10u + dg : w;
                    nd += take && nd < 19 ? 1 : 0;
                    q -= dot ? 1 : 0;
                    nf += dot ? 1 : 0;
                    ni += dot ? 0 : 1;
                } else if (c == '.' && !dot && !ist) {
                    dot = true;
                } else {
                    break;
                }
            }
            if (p >= lim || bad || ni == 0 || (dot && nf == 0)) return ingest::kFallback;
            if (ist) {
                if (ni > 18) return ingest::kFallback;
                // Long.valueOf of the (<= 18 digit) run: w holds it exactly (leading zeros skipped)
                o->ts = neg ? -(int64_t)w : (int64_t)w;
            } else {
                const uint64_t bits = ingest::decimal_to_bits(w, q) | (neg ? 1ull << 63 : 0ull);
                const double v = __builtin_bit_cast(double, bits);
                if (isx) o->x = v;
                if (isy) o->y = v;
            }
        } else {
            const uint32_t fs = p;
            for (; p < lim; p++) {
                const uint8_t c = s[p];
                if (c == d || c <= ' ' || c == '"') break;
            }
            if (p >= lim) return ingest::kFallback;
            if (f == sp.foid) {
                if (p == fs) return ingest::kFallback;
                o->oid = ((c0 + fs) << ingest::kOidLenBits) | (uint64_t)(p - fs);
            }
        }
        const uint8_t c = s[p];
        if (c == d && f < need) {
            p++;
            continue;
        }
        if (f == need && (c == d || c == '\n')) return ingest::kOk;
        return ingest::kFallback;
    }
    return ingest::kFallback;
}

// ---- SWAR form of fast_csv: a field is read as one 24-byte window (three u64 words from the
// staged LDS bytes), its digits / delimiter found from per-byte masks and its value converted
// eight digits at a time, instead of a per-lane loop with a dependent LDS read and a branch per
// byte.  It accepts a subset of fast_csv's records (fields within their 24-byte windows, at most
// 19 digits per number counting leading zeros, the record starting 112 bytes or more before the
// staged end) and gives the same (w, q) decimal -- so the same Eisel-Lemire bits -- and the same
// Long; anything else returns kSwarNo and fast_csv (then the general parser) decides as before.
constexpr int kSwarNo = 2;
constexpr uint32_t kSwarRecordSpan = 112;  // staged bytes a record start needs ahead of it (72 + 32 + 8)
constexpr uint32_t kSwarFieldSpan = 72;    // the last field start within a record's span

struct Win24 {
    uint64_t v[3];
    __device__ __forceinline__ uint32_t byte(uint32_t k) const {
        const uint64_t w = k < 8 ? v[0] : (k < 16 ? v[1] : v[2]);
        return (uint32_t)(w >> ((k & 7u) * 8u)) & 0xffu;
    }
    // 8 bytes starting at window offset off (0 <= off <= 16; bytes past the window read as 0)
    __device__ __forceinline__ uint64_t get8(uint32_t off) const {
        const uint64_t lo = off < 8 ? v[0] : (off < 16 ? v[1] : v[2]);
        const uint64_t hi = off < 8 ? v[1] : (off < 16 ? v[2] : 0ull);
        const uint32_t sh = (off & 7u) * 8u;
        return (lo >> sh) | ((hi << 1) << (63u - sh));
    }
};

__device__ __forceinline__ Win24 lds_win24(const uint8_t* __restrict__ s, uint32_t p) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(s + (p & ~7u));
    const uint64_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
    const uint32_t sh = (p & 7u) * 8u;
    Win24 r;
    r.v[0] = (w0 >> sh) | ((w1 << 1) << (63u - sh));
    r.v[1] = (w1 >> sh) | ((w2 << 1) << (63u - sh));
    r.v[2] = (w2 >> sh) | ((w3 << 1) << (63u - sh));
    return r;
}

// bit 7 of every byte -> one bit per byte (byte i -> bit i); per 32-bit half, one 32-bit multiply
// gathers the four bits (shifted copies land on distinct positions, so no carries)
__device__ __forceinline__ uint32_t byte_bits4(uint32_t m) {
    return ((((m >> 7) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu;
}
__device__ __forceinline__ uint32_t byte_bits(uint64_t m) {
    return byte_bits4((uint32_t)m) | (byte_bits4((uint32_t)(m >> 32)) << 4);
}
// per-byte masks, exact for every byte (no carry or borrow crosses a byte)
__device__ __forceinline__ uint64_t nondigit_m(uint64_t v) {
    const uint64_t x = v ^ 0x3030303030303030ull;
    return (((x & 0x7f7f7f7f7f7f7f7full) + 0x7676767676767676ull) | x) & 0x8080808080808080ull;
}
__device__ __forceinline__ uint64_t eq_m(uint64_t v, uint32_t c) {  // byte == c
    const uint64_t x = v ^ (0x0101010101010101ull * c);
    return ~((((x & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | x)) & 0x8080808080808080ull;
}
__device__ __forceinline__ uint64_t le20_m(uint64_t v) {  // byte <= 0x20
    return ~((((v & 0x7f7f7f7f7f7f7f7full) + 0x5f5f5f5f5f5f5f5full) | v)) & 0x8080808080808080ull;
}
__device__ __forceinline__ uint32_t mask24(uint64_t a, uint64_t b, uint64_t c) {
    return byte_bits(a) | (byte_bits(b) << 8) | (byte_bits(c) << 16);
}
// value of four digit values b0..b3 (bytes of v, b0 most significant): two byte dot products
// and a 24-bit multiply-add, all full rate (the 64-bit SWAR multiplies they replace are built
// of quarter-rate 32-bit multiplies)
__device__ __forceinline__ uint32_t digits4(uint32_t v) {
    const uint32_t hi = __builtin_amdgcn_udot4(v, 0x0000010au, 0u, false);  // b0 * 10 + b1
    return __builtin_amdgcn_udot4(v, 0x010a0000u, __umul24(hi, 100u), false);  // .. * 100 + b2 * 10 + b3
}
// value of m <= 8 ASCII digits starting at window offset off
__device__ __forceinline__ uint64_t digits8(const Win24& W, uint32_t off, uint32_t m) {
    uint64_t x = W.get8(off) - 0x3030303030303030ull;  // digit bytes are the low m: no borrow into them
    x = m ? (x << (8u * (8u - m))) : 0ull;  // the m digits in bytes 8 - m .. 7 (weights 10^(7 - byte))
    return __umul24(digits4((uint32_t)x), 10000u) + digits4((uint32_t)(x >> 32));
}
__device__ __forceinline__ uint64_t digits_n(const Win24& W, uint32_t off, uint32_t n) {  // n <= 19
    constexpr uint64_t p8 = 100000000ull;
    if (n <= 8) return digits8(W, off, n);
    if (n <= 16) return (uint64_t)(uint32_t)digits8(W, off, n - 8) * (uint32_t)p8 + digits8(W, off + n - 8, 8);
    return (digits8(W, off, n - 16) * p8 + digits8(W, off + n - 16, 8)) * p8 + digits8(W, off + n - 8, 8);
}
__device__ const uint64_t kPow10u[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull,
                                         10000000ull, 100000000ull, 1000000000ull, 10000000000ull,
                                         100000000000ull, 1000000000000ull, 10000000000000ull,
                                         100000000000000ull, 1000000000000000ull, 10000000000000000ull,
                                         100000000000000000ull, 1000000000000000000ull,
                                         10000000000000000000ull};

__device__ __forceinline__ int swar_csv(const uint8_t* __restrict__ s, uint32_t p, uint32_t lim,
                                        const ingest::Spec& sp, ingest::Parsed* o, uint64_t c0) {
    if (p + kSwarRecordSpan > lim) return kSwarNo;
    const uint32_t p0 = p;
    const uint32_t d = (uint32_t)(uint8_t)sp.delim;
    int need = sp.fx > sp.fy ? sp.fx : sp.fy;
    if (sp.fts > need) need = sp.fts;
    if (sp.foid > need) need = sp.foid;
    for (int f = 0; f <= need; f++) {
        if (p - p0 > kSwarFieldSpan) return kSwarNo;
        const Win24 W = lds_win24(s, p);
        const bool isx = f == sp.fx, isy = f == sp.fy, ist = f == sp.fts;
        uint32_t term;
        if (isx || isy || ist) {
            if (((isx || isy) && ist) || f == sp.foid) return kSwarNo;
            const uint32_t st = W.byte(0) == '-' ? 1u : 0u;
            const uint32_t nd = mask24(nondigit_m(W.v[0]), nondigit_m(W.v[1]), nondigit_m(W.v[2]));
            const uint32_t m1 = nd >> st;
            if (!m1) return kSwarNo;
            const uint32_t e1 = st + (uint32_t)__builtin_ctz(m1);
            const uint32_t ni = e1 - st;
            uint32_t nf = 0;
            term = e1;
            if (!ist && W.byte(e1) == '.') {
                const uint32_t m2 = e1 + 1 < 24 ? nd >> (e1 + 1) : 0u;
                if (!m2) return kSwarNo;
                term = e1 + 1 + (uint32_t)__builtin_ctz(m2);
                nf = term - e1 - 1;
                if (nf == 0) return kSwarNo;
            }
            if (ni == 0 || ni + nf > 19 || (ist && ni > 18)) return kSwarNo;
            const uint64_t iv = digits_n(W, st, ni);
            if (ist) {
                o->ts = st ? -(int64_t)iv : (int64_t)iv;
            } else {
                const uint64_t w = nf ? iv * kPow10u[nf] + digits_n(W, e1 + 1, nf) : iv;
                const uint64_t bits = ingest::decimal_to_bits(w, -(int32_t)nf) | (st ? 1ull << 63 : 0ull);
                const double v = __builtin_bit_cast(double, bits);
                if (isx) o->x = v;
                if (isy) o->y = v;
            }
        } else {
            const uint32_t stop = mask24(eq_m(W.v[0], d) | le20_m(W.v[0]) | eq_m(W.v[0], '"'),
                                         eq_m(W.v[1], d) | le20_m(W.v[1]) | eq_m(W.v[1], '"'),
                                         eq_m(W.v[2], d) | le20_m(W.v[2]) | eq_m(W.v[2], '"'));
            if (!stop) return kSwarNo;
            term = (uint32_t)__builtin_ctz(stop);
            if (f == sp.foid) {
                if (term == 0) return kSwarNo;
                o->oid = ((c0 + p) << ingest::kOidLenBits) | term;
            }
        }
        const uint32_t c = W.byte(term);
        if (c == d && f < need) {
            p += term + 1;
            continue;
        }
        if (f == need && (c == d || c == '\n')) return ingest::kOk;
        return kSwarNo;
    }
    return kSwarNo;
}

// Stage chunk vb (+ the tail) in LDS and list the record starts it owns, in order: byte 0 of the
// batch, then q + 1 for each '\n' at q.  Returns the chunk's record count (block-uniform).
// The record-start list holds CAP entries (the hot kernel: 4096, so its LDS is 25 KB; a chunk
// with more records -- shorter than 4 bytes on average, i.e. blank lines the reference rejects --
// goes to ingest_general, whose list holds every possible start).
constexpr unsigned kFastStarts = 4096;
template <unsigned CAP>
struct ChunkLds {
    uint4 text4[(kIngestChunk + kIngestTail) / 16];
    uint16_t start[CAP + 1];
    unsigned wave[kThreads / kWave];
};
template <unsigned CAP>
__device__ __forceinline__ unsigned stage_chunk(const uint8_t* __restrict__ text, uint64_t nbytes, unsigned vb,
                                                ChunkLds<CAP>& L) {
    const uint64_t c0 = (uint64_t)vb * kIngestChunk;
    // the chunk first (this thread's 32 bytes stay in registers for the '\n' scan)
    const uint64_t p = c0 + threadIdx.x * kBytesPerThread;
    uint4 v[kLoads];
#pragma unroll
    for (int j = 0; j < kLoads; j++) v[j] = load16(text, p + 16 * j, nbytes);
#pragma unroll
    for (int j = 0; j < kLoads; j++) L.text4[threadIdx.x * kLoads + j] = v[j];
    for (uint32_t i = kIngestChunk / 16 + threadIdx.x; i < (kIngestChunk + kIngestTail) / 16; i += kThreads) {
        const uint64_t q = c0 + (uint64_t)i * 16;
        if (q < nbytes) L.text4[i] = load16(text, q, nbytes);
    }
    const uint64_t m = p < nbytes ? nl_mask(v, p, nbytes - 1) : 0ull;
    const bool first = vb == 0 && threadIdx.x == 0 && nbytes > 0;
    const unsigned mine = (unsigned)__popcll(m) + (first ? 1u : 0u);
    unsigned nrec;
    unsigned at = block_excl_scan(mine, L.wave, &nrec);
    if (first) L.start[at++] = 0;
    for (uint64_t mm = m; mm; mm &= mm - 1) {
        if (at < CAP) L.start[at] = (uint16_t)(threadIdx.x * kBytesPerThread + __builtin_ctzll(mm) + 1);
        at++;
    }
    __syncthreads();
    return nrec;
}

// plain column stores (nontemporal ones measured within noise, round 5: 403-415 against 407-417 us)
template <typename T>
__device__ __forceinline__ void col_store(T* p, T v) {
    *p = v;
}
__device__ __forceinline__ void store_record(const IngestArgs& a, uint64_t idx, const ingest::Parsed& o,
                                             double* __restrict__ x, double* __restrict__ y,
                                             int64_t* __restrict__ ts, uint32_t* __restrict__ cell) {
    col_store(x + idx, o.x);
    col_store(y + idx, o.y);
    if (ts) col_store(ts + idx, (int64_t)o.ts);
    if (a.oid) col_store(a.oid + idx, o.oid);
    if (cell) {
        const int32_t cx = ingest::java_cell(o.x, a.min_x, a.cell_len);
        const int32_t cy = ingest::java_cell(o.y, a.min_y, a.cell_len);
        const bool ok = cx >= 0 && cx < a.n && cy >= 0 && cy < a.n;
        col_store(cell + idx, ok ? (uint32_t)cx * (uint32_t)a.n + (uint32_t)cy : 0xffffffffu);
    }
}

// The hot kernel: CSV fast paths only (swar_csv, then fast_csv), so no call, no scratch and 55
// VGPRs -- with the general grammar inlined the kernel took 256 VGPRs + 880 B of scratch per
// lane (2 waves per SIMD, 4.0 ms per batch), and as a call its scratch frame alone kept it at
// 1.3 ms.  A chunk with a record the fast paths do not decide (or any chunk of a GeoJSON / WKT
// batch) is listed for ingest_general, which re-parses all its records with the full grammar.
// The first round of records is parsed before the look-back, so the wait for the earlier
// chunks' counts overlaps the parse.
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8))) void ingest_fused(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                        IngestArgs a, IngestLookback lb,
                                                        double* __restrict__ x, double* __restrict__ y,
                                                        int64_t* __restrict__ ts, uint32_t* __restrict__ cell,
                                                        uint64_t cap, unsigned long long* __restrict__ total) {
    __shared__ ChunkLds<kFastStarts> L;
    __shared__ unsigned s_vb, s_flag;
    __shared__ unsigned long long s_base;
    if (threadIdx.x == 0) {
        s_vb = atomicAdd(lb.ticket, 1u);
        s_flag = 0;
    }
    __syncthreads();
    const unsigned vb = s_vb;
    const unsigned nrec = stage_chunk(text, nbytes, vb, L);
    const unsigned long long tag = lb.epoch << 42;
    if (threadIdx.x == 0) publish_status(lb.status + vb, tag | (vb == 0 ? kPrefixBit : 0ull) | nrec);
    const uint64_t c0 = (uint64_t)vb * kIngestChunk;
    const uint64_t stage_end = c0 + kIngestChunk + kIngestTail < nbytes ? c0 + kIngestChunk + kIngestTail : nbytes;
    const uint32_t stage_len = (uint32_t)(stage_end - c0);
    const uint8_t* st8 = reinterpret_cast<const uint8_t*>(L.text4);
    const uint8_t dl = (uint8_t)a.spec.delim;
    const bool fast = a.spec.format == ingest::kCsv && dl > ' ' && dl != '"' && dl != '.' && dl != '-' &&
                      (unsigned)(dl - '0') >= 10u;
    const bool listed_all = nrec <= kFastStarts;  // else the whole chunk goes to ingest_general
    const unsigned rounds = (nrec && listed_all) ? (nrec + kThreads - 1) / kThreads : 1u;  // block-uniform
    bool undecided = !listed_all;
    uint64_t rbase = 0;
    for (unsigned r = 0; r < rounds; r++) {
        const unsigned i = r * kThreads + threadIdx.x;
        ingest::Parsed o;
        o.x = o.y = 0.0;
        o.ts = 0;
        o.oid = ingest::kOidNull;
        int rc = ingest::kFallback;
        if (i < nrec && listed_all) {
            if (fast) {
                rc = swar_csv(st8, L.start[i], stage_len, a.spec, &o, c0);
                if (rc == kSwarNo) rc = fast_csv(st8, L.start[i], stage_len, a.spec, &o, c0);
            }
            undecided |= rc != ingest::kOk;
        }
        if (r == 0) {  // the record base: look-back by wave 0, behind its first round's parse
            if (threadIdx.x < kWave) {
                const unsigned long long excl = vb == 0 ? 0ull : lookback_prefix(lb.status, vb, lb.epoch, lb.nlisted + 1);
                if (threadIdx.x == 0) {
                    if (vb != 0) publish_status(lb.status + vb, tag | kPrefixBit | (excl + nrec));
                    s_base = excl;
                    if (vb == gridDim.x - 1) {
                        *total = excl + nrec;
                        __hip_atomic_store(lb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
                    }
                }
            }
            __syncthreads();
            rbase = s_base;
        }
        const uint64_t idx = rbase + i;
        if (i < nrec && listed_all && rc == ingest::kOk && idx < cap) store_record(a, idx, o, x, y, ts, cell);
    }
    if (__ballot(undecided) && lane_id() == 0) s_flag = 1u;
    __syncthreads();
    if (threadIdx.x == 0 && s_flag) {  // the chunk goes to ingest_general (rare for CSV)
        const unsigned j = atomicAdd(lb.nlisted, 1u);
        lb.listed[j] = make_ulonglong2(vb, rbase);
    }
}

// The general grammar (ingest_parse.h: quoted tokens, hex significands, exponents of any length,
// GeoJSON, WKT) over the chunks ingest_fused listed: every record of such a chunk is parsed again
// (the fast paths give the same values on the records they accept) and the first rejected record
// index is kept (bad holds its complement under atomicMax: zero = none).  A fixed grid that
// strides over the list; with an empty list every block exits after one load.
__global__ __launch_bounds__(kThreads) void ingest_general(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                          IngestArgs a, IngestLookback lb,
                                                          double* __restrict__ x, double* __restrict__ y,
                                                          int64_t* __restrict__ ts, uint32_t* __restrict__ cell,
                                                          uint64_t cap, unsigned long long* __restrict__ bad) {
    __shared__ ChunkLds<kIngestChunk> L;
    const unsigned nl = *lb.nlisted;
    for (unsigned j = blockIdx.x; j < nl; j += gridDim.x) {
        const ulonglong2 e = lb.listed[j];
        const unsigned vb = (unsigned)e.x;
        const uint64_t rbase = e.y;
        const unsigned nrec = stage_chunk(text, nbytes, vb, L);
        const uint64_t c0 = (uint64_t)vb * kIngestChunk;
        const uint64_t stage_end = c0 + kIngestChunk + kIngestTail < nbytes ? c0 + kIngestChunk + kIngestTail : nbytes;
        const LdsReader rd{reinterpret_cast<const uint8_t*>(L.text4), c0, (uint32_t)(stage_end - c0), text, nbytes};
        for (unsigned i = threadIdx.x; i < nrec; i += kThreads) {
            const uint64_t idx = rbase + i;
            ingest::Parsed o;
            o.ts = 0;
            if (ingest::parse_record(rd, c0 + L.start[i], a.spec, &o) != ingest::kOk) {
                atomicMax(bad, ~(unsigned long long)idx);
                continue;
            }
            if (idx < cap) store_record(a, idx, o, x, y, ts, cell);
        }
        __syncthreads();  // L is restaged for the next listed chunk
    }
}

// ---- objID spans -> strings (geohip_ingest_oid_compact) --------------------------------------
// Per record: the span's bytes without '"' (the reference deletes every quote of a CSV record
// before the split; a GeoJSON objID span holds none).  Lengths, a segmented exclusive scan into
// out_off (bit 63 = null objID), then the copy.
constexpr unsigned kOidTB = 256;
constexpr unsigned kOidPer = 8;                  // records per thread
constexpr unsigned kOidSeg = kOidTB * kOidPer;   // records per block

__device__ __forceinline__ bool oid_span(uint64_t v, uint64_t* off, uint64_t* len) {
    *len = v & ((1ull << ingest::kOidLenBits) - 1);
    *off = v >> ingest::kOidLenBits;
    return *len != ingest::kOidNull;
}

__global__ __launch_bounds__(kOidTB) void oid_len(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                 const uint64_t* __restrict__ spans, uint64_t m,
                                                 uint64_t* __restrict__ len, uint64_t* __restrict__ seg, uint64_t nseg) {
    uint64_t sum = 0;
    for (unsigned k = 0; k < kOidPer; k++) {
        const uint64_t i = (uint64_t)blockIdx.x * kOidSeg + (uint64_t)k * kOidTB + threadIdx.x;
        if (i >= m) break;
        uint64_t off, n, c = 0;
        if (oid_span(spans[i], &off, &n)) {
            if (off > nbytes || n > nbytes - off) {
                atomicOr(reinterpret_cast<unsigned long long*>(seg + nseg + 1), 1ull);
                n = 0;
            }
            for (uint64_t t = 0; t < n; t++) c += text[off + t] != '"' ? 1u : 0u;
        }
        len[i] = c;
        sum += c;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    __shared__ uint64_t s_sum[kOidTB / kWave];
    if (lane_id() == 0) s_sum[threadIdx.x / kWave] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (unsigned w = 0; w < kOidTB / kWave; w++) t += s_sum[w];
        seg[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(1024) void oid_scan_segs(uint64_t* __restrict__ seg, uint64_t nseg) {
    __shared__ uint64_t part[1024];
    const uint64_t per = (nseg + 1023) / 1024;
    const uint64_t b = threadIdx.x * per, e = b + per < nseg ? b + per : nseg;
    uint64_t s = 0;
    for (uint64_t u = b; u < e; u++) s += seg[u];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint64_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = part[threadIdx.x] - s;
    for (uint64_t u = b; u < e; u++) {
        const uint64_t c = seg[u];
        seg[u] = run;
        run += c;
    }
    if (threadIdx.x == 1023) seg[nseg] = part[1023];
}

__global__ __launch_bounds__(kOidTB) void oid_offsets(const uint64_t* __restrict__ spans, uint64_t m,
                                                     const uint64_t* __restrict__ len, const uint64_t* __restrict__ seg,
                                                     uint64_t nseg, uint64_t* __restrict__ out_off) {
    // thread t owns records b0 + t * kOidPer .. + kOidPer (contiguous), a block scan of their sums
    __shared__ uint64_t s_tot[kOidTB];
    const uint64_t b0 = (uint64_t)blockIdx.x * kOidSeg + (uint64_t)threadIdx.x * kOidPer;
    uint64_t mine = 0;
    for (unsigned k = 0; k < kOidPer; k++)
        if (b0 + k < m) mine += len[b0 + k];
    s_tot[threadIdx.x] = mine;
    __syncthreads();
    for (unsigned o = 1; o < kOidTB; o <<= 1) {
        const uint64_t v = threadIdx.x >= o ? s_tot[threadIdx.x - o] : 0;
        __syncthreads();
        s_tot[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = seg[blockIdx.x] + s_tot[threadIdx.x] - mine;
    for (unsigned k = 0; k < kOidPer; k++) {
        const uint64_t i = b0 + k;
        if (i >= m) break;
        uint64_t off, n;
        const bool real = oid_span(spans[i], &off, &n);
        out_off[i] = run | (real ? 0ull : 1ull << 63);
        run += len[i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out_off[m] = seg[nseg];
}

__global__ __launch_bounds__(kOidTB) void oid_write(const uint8_t* __restrict__ text, const uint64_t* __restrict__ spans,
                                                   uint64_t m, const uint64_t* __restrict__ out_off,
                                                   uint8_t* __restrict__ out, uint64_t cap) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOidTB + threadIdx.x; i < m; i += (uint64_t)gridDim.x * kOidTB) {
        uint64_t off, n;
        if (!oid_span(spans[i], &off, &n)) continue;
        uint64_t o = out_off[i] & ~(1ull << 63);
        for (uint64_t t = 0; t < n; t++) {
            const uint8_t c = text[off + t];
            if (c != '"' && o < cap) out[o++] = c;
        }
    }
}

}  // namespace

uint64_t oid_segments(uint64_t m) { return (m + kOidSeg - 1) / kOidSeg; }

hipError_t launch_oid_compact(geohip_ctx* ctx, const uint8_t* text, uint64_t nbytes, const uint64_t* spans, uint64_t m,
                              uint64_t* len, uint64_t* seg, uint64_t* out_off, uint8_t* out_text, uint64_t cap,
                              hipStream_t st) {
    const uint64_t nseg = oid_segments(m);
    if (out_text) {  // second call: the copy
        if (m) {
            const uint64_t g = (m + kOidTB - 1) / kOidTB;
            tlaunch(ctx, oid_write, (unsigned)(g < 65536 ? g : 65536), kOidTB, 0, st, text, spans, m,
                    (const uint64_t*)out_off, out_text, cap);
        }
        return hipGetLastError();
    }
    hipError_t e = hipMemsetAsync(seg + nseg, 0, 16, st);
    if (e != hipSuccess) return e;
    if (m) {
        tlaunch(ctx, oid_len, (unsigned)nseg, kOidTB, 0, st, text, nbytes, spans, m, len, seg, nseg);
        tlaunch(ctx, oid_scan_segs, 1, 1024, 0, st, seg, nseg);
        tlaunch(ctx, oid_offsets, (unsigned)nseg, kOidTB, 0, st, spans, m, (const uint64_t*)len, (const uint64_t*)seg,
                nseg, out_off);
    } else {
        e = hipMemsetAsync(out_off, 0, 8, st);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_ingest(geohip_ctx* ctx, const uint8_t* text, uint64_t nbytes, const IngestArgs& a,
                         const IngestLookback& lb, unsigned long long* total, double* x, double* y, int64_t* ts,
                         uint32_t* cell, uint64_t cap, unsigned long long* bad, hipStream_t st) {
    const uint64_t nchunks = ingest_chunks(nbytes);
    if (nchunks == 0) return hipMemsetAsync(total, 0, sizeof(unsigned long long), st);
    hipEvent_t ev0, ev1;
    ctx_timing_events(ctx, &ev0, &ev1);  // the step: both kernels (each also stamped by tlaunch)
    if (ev0) (void)hipEventRecord(ev0, st);
    tlaunch(ctx, ingest_fused, (unsigned)nchunks, kThreads, 0, st, text, nbytes, a, lb, x, y, ts, cell, cap, total);
    const unsigned g = nchunks < kGeneralBlocks ? (unsigned)nchunks : kGeneralBlocks;
    tlaunch(ctx, ingest_general, g, kThreads, 0, st, text, nbytes, a, lb, x, y, ts, cell, cap, bad);
    if (ev1) (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

}  // namespace geohip
