// device_common.h -- gfx950 device helpers shared by the libgeohip kernels.
//
// Everything here must be compiled with -ffp-contract=off (no FMA contraction), because
// the reference evaluates every fp64 expression in Java source order with separately
// rounded operations.  sqrt/division are IEEE correctly rounded on this path (checked on
// the device by tests/test_gpu_parity.py::test_fp64_primitives).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "geohip_internal.h"

namespace geohip {

constexpr int kWave = 64;
constexpr unsigned long long kSentinelD = ~0ull;  // > bits of any distance in [0, MAX_VALUE]
constexpr unsigned kSentinelI = ~0u;
constexpr double kDblMax = 1.7976931348623157e308;

// ---------------------------------------------------------------- fdlibm e_hypot -----------
__device__ __forceinline__ int32_t dhi(double d) { return __double2hiint(d); }
__device__ __forceinline__ uint32_t dlo(double d) { return (uint32_t)__double2loint(d); }
__device__ __forceinline__ double dmk(int32_t hi, uint32_t lo) { return __hiloint2double(hi, (int)lo); }
__device__ __forceinline__ double dsethi(double d, int32_t hi) { return dmk(hi, dlo(d)); }

// JDK 8 StrictMath.hypot (fdlibm 5.3 e_hypot.c) = JTS 1.16.1 Coordinate.distance kernel.
// The two "medium size" formulas are evaluated by operand selection so a wave does not
// diverge on which coordinate difference is larger; each selected operand is bitwise the
// value the corresponding fdlibm branch computes.
__device__ __forceinline__ double fdlibm_hypot(double x, double y) {
    int32_t ha = dhi(x) & 0x7fffffff;
    int32_t hb = dhi(y) & 0x7fffffff;
    double a, b;
    if (hb > ha) { a = y; b = x; int32_t j = ha; ha = hb; hb = j; } else { a = x; b = y; }
    a = dsethi(a, ha);
    b = dsethi(b, hb);
    if ((ha - hb) > 0x3c00000) return a + b;
    int32_t k = 0;
    if (ha > 0x5f300000) {
        if (ha >= 0x7ff00000) {
            double w = a + b;
            if (((ha & 0xfffff) | dlo(a)) == 0) w = a;
            if (((hb ^ 0x7ff00000) | dlo(b)) == 0) w = b;
            return w;
        }
        ha -= 0x25800000; hb -= 0x25800000; k += 600;
        a = dsethi(a, ha);
        b = dsethi(b, hb);
    }
    if (hb < 0x20b00000) {
        if (hb <= 0x000fffff) {
            if ((hb | dlo(b)) == 0) return a;
            double t1 = dmk(0x7fd00000, 0);
            b *= t1; a *= t1; k -= 1022;   // fdlibm keeps the unscaled ha/hb here
        } else {
            ha += 0x25800000; hb += 0x25800000; k -= 600;
            a = dsethi(a, ha);
            b = dsethi(b, hb);
        }
    }
    double w = a - b;
    const bool big = w > b;
    const double t1 = big ? dmk(ha, 0) : dmk(ha + 0x00100000, 0);
    const double aa = big ? a : a + a;
    const double t2 = aa - t1;
    const double y1 = dmk(hb, 0);
    const double y2 = b - y1;
    // big:  sqrt(t1*t1 - (b*(-b) - t2*(a+t1)))
    // else: sqrt(t1*y1 - (w*(-w) - (t1*y2 + t2*b)))
    const double P = big ? t1 * t1 : t1 * y1;
    const double Q = big ? b * (-b) : w * (-w);
    const double R = big ? t2 * (a + t1) : (t1 * y2 + t2 * b);
    w = __builtin_sqrt(P - (Q - R));
    if (k != 0) return dmk(0x3ff00000 + (k << 20), 0) * w;
    return w;
}

// p.point.distance(q.point): JTS DistanceOp with minDistance = Double.MAX_VALUE and strict <
// (DistanceFunctions.java:15-18): NaN / inf / MAX all read as MAX_VALUE.
__device__ __forceinline__ double jts_pp_distance(double ax, double ay, double bx, double by) {
    double d = fdlibm_hypot(ax - bx, ay - by);
    return d < kDblMax ? d : kDblMax;
}

__device__ __forceinline__ double coord_distance(double ax, double ay, double bx, double by) {
    return fdlibm_hypot(ax - bx, ay - by);
}

// Safe squared-distance screens.  With dx, dy as the kernels compute them, d2 = dx*dx + dy*dy
// in fp64 is within 3 ulp of the true square and fdlibm hypot is within 1 ulp of the true
// distance, so a 2^-40 relative margin on the bound squared separates "certainly above" and
// "certainly below" from the band where the exact JTS distance must be computed.  NaN d2
// fails both tests (goes to the exact path); an infinite bound never rejects.
constexpr double kSqHi = 1.0 + 0x1.0p-40;
constexpr double kSqLo = 1.0 - 0x1.0p-40;

// ---------------------------------------------------------------- classification ----------
__device__ __forceinline__ bool in_box(const Box& b, double x, double y) {
    bool bx = (x >= b.xlo) && (x <= b.xhi);
    bool by = (y >= b.ylo) && (y <= b.yhi);
    if (b.nan_x) bx = bx || (x != x);
    if (b.nan_y) by = by || (y != y);
    return bx && by;
}

// ---------------------------------------------------------------- wave64 primitives -------
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ unsigned lanes_below(unsigned long long mask) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

// Orders LDS traffic of one wave (lanes exchange data through wave-private LDS).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct KE {  // kNN entry: distance bits (monotone for d >= 0) and window index
    unsigned long long d;
    unsigned i;
};

__device__ __forceinline__ bool kless(const KE& a, const KE& b) {
    return a.d < b.d || (a.d == b.d && a.i < b.i);
}
// ---- cross-lane moves without the LDS crossbar --------------------------------------
// lane ^ j for j = 1, 2 (DPP quad_perm), 4 (row_half_mirror + quad_perm), 8 (row_mirror +
// row_half_mirror), 16 (ds_swizzle bit mode), 32 (v_permlane32_swap, gfx950).  j must fold to
// a constant (all callers sit in fully unrolled loops).
#define GEOHIP_DPP(v, ctrl) ((unsigned)__builtin_amdgcn_update_dpp(0, (int)(v), (ctrl), 0xF, 0xF, false))
__device__ __forceinline__ unsigned xor_lane(unsigned v, int j) {
    switch (j) {
        case 1: return GEOHIP_DPP(v, 0xB1);
        case 2: return GEOHIP_DPP(v, 0x4E);
        case 4: return GEOHIP_DPP(GEOHIP_DPP(v, 0x141), 0x1B);
        case 8: return GEOHIP_DPP(GEOHIP_DPP(v, 0x140), 0x141);
        case 16: return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
        default: {
            auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            return __lane_id() < 32 ? r[1] : r[0];
        }
    }
}
__device__ __forceinline__ unsigned long long xor_lane64(unsigned long long v, int j) {
    const unsigned lo = xor_lane((unsigned)v, j), hi = xor_lane((unsigned)(v >> 32), j);
    return ((unsigned long long)hi << 32) | lo;
}
// lane ^ 63 (reverse the wave)
__device__ __forceinline__ unsigned rev_lane(unsigned v) {
    return xor_lane((unsigned)__builtin_amdgcn_ds_swizzle((int)GEOHIP_DPP(v, 0x140), 0x401F), 32);
}
__device__ __forceinline__ unsigned long long rev_lane64(unsigned long long v) {
    return ((unsigned long long)rev_lane((unsigned)(v >> 32)) << 32) | rev_lane((unsigned)v);
}

// Inclusive prefix sum over the 64 lanes by DPP (row_shr 1/2/4/8 inside each 16-lane row with
// bound_ctrl zero fill, then row_bcast:15 / row_bcast:31 across rows): no LDS round trips.
__device__ __forceinline__ unsigned wave_incl_scan(unsigned x) {
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

__device__ __forceinline__ KE kxor(const KE& v, int m) {
    KE r;
    r.d = xor_lane64(v.d, m);
    r.i = xor_lane(v.i, m);
    return r;
}
__device__ __forceinline__ KE krev(const KE& v) {
    KE r;
    r.d = rev_lane64(v.d);
    r.i = rev_lane(v.i);
    return r;
}
__device__ __forceinline__ KE ksentinel() {
    KE r;
    r.d = kSentinelD;
    r.i = kSentinelI;
    return r;
}

// Bitonic sort of 64 keys held one per lane (ascending by lane).
__device__ __forceinline__ KE wave_sort64(KE v) {
    const int lane = lane_id();
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int j = size >> 1; j > 0; j >>= 1) {
            KE p = kxor(v, j);
            const bool want_min = ((lane & j) == 0) == ((lane & size) == 0);
            const bool pl = kless(p, v);
            if (want_min == pl) v = p;
        }
    }
    return v;
}

// A KPL*64-entry list: element e = s*64 + lane lives in slot s of that lane.
template <int KPL>
struct WList {
    KE s[KPL];
};

// Sort a bitonic list ascending (bitonic merge network).
template <int KPL>
__device__ __forceinline__ void wave_bitonic_merge(WList<KPL>& L) {
    const int lane = lane_id();
#pragma unroll
    for (int jj = KPL / 2; jj >= 1; jj >>= 1) {  // distances >= 64: in-lane slot pairs
#pragma unroll
        for (int s = 0; s < KPL; s++) {
            if ((s & jj) == 0) {
                KE a = L.s[s], b = L.s[s | jj];
                if (kless(b, a)) { L.s[s] = b; L.s[s | jj] = a; }
            }
        }
    }
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
#pragma unroll
        for (int s = 0; s < KPL; s++) {
            KE p = kxor(L.s[s], j);
            const bool want_min = (lane & j) == 0;
            if (want_min == kless(p, L.s[s])) L.s[s] = p;
        }
    }
}

// L <- the KPL*64 smallest of L u B, sorted; B is an ascending list of the same size.
template <int KPL>
__device__ __forceinline__ void wave_merge_lists(WList<KPL>& L, const WList<KPL>& B) {
    const int lane = lane_id();
#pragma unroll
    for (int s = 0; s < KPL; s++) {
        KE rv = krev(B.s[KPL - 1 - s]);  // B reversed
        if (kless(rv, L.s[s])) L.s[s] = rv;
    }
    wave_bitonic_merge<KPL>(L);
}

// L <- smallest of L u batch (64 sorted keys, one per lane), sorted.
template <int KPL>
__device__ __forceinline__ void wave_merge_batch(WList<KPL>& L, const KE& sorted_batch) {
    const int lane = lane_id();
    KE rv = krev(sorted_batch);
    if (kless(rv, L.s[KPL - 1])) L.s[KPL - 1] = rv;
    wave_bitonic_merge<KPL>(L);
}

// Full bitonic sort of a KPL*64-entry list (element e = s*64 + lane), ascending.
template <int KPL>
__device__ __forceinline__ void wave_sort_list(WList<KPL>& L) {
    const int lane = lane_id();
#pragma unroll
    for (int size = 2; size <= 64 * KPL; size <<= 1) {
#pragma unroll
        for (int j = size >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
                const int jj = j >> 6;
#pragma unroll
                for (int s = 0; s < KPL; s++) {
                    if ((s & jj) == 0) {
                        const bool up = ((s * 64) & size) == 0;
                        KE a = L.s[s], b = L.s[s | jj];
                        if (kless(b, a) == up) { L.s[s] = b; L.s[s | jj] = a; }
                    }
                }
            } else {
#pragma unroll
                for (int s = 0; s < KPL; s++) {
                    const int e = s * 64 + lane;
                    const bool up = (e & size) == 0;
                    KE p = kxor(L.s[s], j);
                    const bool want_min = ((lane & j) == 0) == up;
                    if (want_min == kless(p, L.s[s])) L.s[s] = p;
                }
            }
        }
    }
}

template <int KPL>
__device__ __forceinline__ KE wave_list_get(const WList<KPL>& L, int e) {  // e wave-uniform
    const int s = e >> 6, l = e & 63;
    KE r = L.s[0];
#pragma unroll
    for (int t = 1; t < KPL; t++)
        if (t == s) r = L.s[t];
    KE o;
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)r.d, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(r.d >> 32), l);
    o.d = ((unsigned long long)hi << 32) | lo;
    o.i = (unsigned)__builtin_amdgcn_readlane((int)r.i, l);
    return o;
}

// ---------------------------------------------------------------- decoupled look-back -----
// Status word of a chunk processed in ticket order: (epoch << 42) | kPrefixBit? | value, value =
// the chunk's own count (aggregate) or, with kPrefixBit, the counts of every chunk up to and
// including it (inclusive prefix).  Words of an earlier launch carry another epoch: not ready.
// (The ingest record bases and the streaming point-polygon pair / candidate offsets.)
constexpr unsigned long long kPrefixBit = 1ull << 41;
constexpr unsigned long long kValueMask = kPrefixBit - 1;

__device__ __forceinline__ void publish_status(unsigned long long* w, unsigned long long v) {
    // an atomic exchange is performed at the device coherence point: the other XCDs' polling
    // loads see it at once (a plain store may sit in this XCD's L2)
    (void)__hip_atomic_exchange(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave: the sum of the counts of the chunks before vb.  Lane l inspects chunk j - l; the
// window of 64 is consumed up to its nearest inclusive prefix (or entirely), once every word in
// that span is ready.  Chunks start in ticket order, so every chunk waited on is resident or
// done.  A wait past kLookbackSpins polls (seconds: a broken invariant, never a slow chunk) sets
// *fault and returns, so a bug ends the kernel with an error instead of hanging the device.
constexpr unsigned kLookbackSpins = 1u << 22;
__device__ __forceinline__ unsigned long long lookback_prefix(const unsigned long long* status, unsigned vb,
                                                              unsigned long long epoch, unsigned* fault) {
    const int lane = lane_id();
    unsigned long long excl = 0;
    long long j = (long long)vb - 1;
    unsigned spins = 0;
    while (j >= 0) {
        const long long t = j - lane;
        unsigned long long v = t >= 0 ? __hip_atomic_load(status + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : (epoch << 42) | kPrefixBit;  // before chunk 0: prefix 0
        const bool ready = (v >> 42) == epoch;
        const unsigned long long pm = __ballot(ready && (v & kPrefixBit));
        const unsigned long long span = pm ? (2ull << __builtin_ctzll(pm)) - 1ull : ~0ull;  // lanes 0 .. first prefix
        if (__ballot(!ready) & span) {
            if (++spins > kLookbackSpins) {
                if (lane == 0) *fault = 1u;
                return excl;
            }
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        unsigned long long c = ((span >> lane) & 1ull) ? (v & kValueMask) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        excl += c;
        if (pm) break;
        j -= kWave;
    }
    return excl;
}

// The exclusive prefix of the per-block counts of blocks 0 .. vb - 1 (status words (epoch << 40)
// | count, published by blocks that took their tickets earlier, so every block waited on is
// resident or done): one wave, lane l polls words l, l + 64, ... with all loads in flight, s_sleep
// back-off between rounds.  A wait past spin_limit rounds (seconds at kLookbackSpins: a broken
// invariant, never a slow block) sets *fault and returns what it has -- the kernel then ends with
// an error the host reports instead of hanging the device.  inject (measurement / tests only)
// waits for an epoch no block writes, to exercise that path.
template <int kPer>
__device__ __forceinline__ unsigned long long poll_block_counts(const unsigned long long* status, unsigned vb,
                                                                unsigned long long epoch, unsigned spin_limit,
                                                                unsigned inject, unsigned* fault) {
    const int lane = lane_id();
    const unsigned long long want = inject && vb ? (epoch ^ 0x800000ull) : epoch;
    unsigned long long v[kPer];
    unsigned pending = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const unsigned j = (unsigned)lane + (unsigned)k * kWave;
        v[k] = j < vb ? __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (want << 40);
    }
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if ((v[k] >> 40) != want) pending |= 1u << k;
    unsigned spins = 0;
    while (__ballot(pending != 0)) {
        if (++spins > spin_limit) {
            if (lane == 0) __hip_atomic_fetch_or(fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // kFaultLookback
            break;
        }
        __builtin_amdgcn_s_sleep(8);
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            if (pending & (1u << k)) {
                v[k] = __hip_atomic_load(status + lane + k * kWave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((v[k] >> 40) == want) pending &= ~(1u << k);
            }
        }
    }
    unsigned long long pre = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) pre += v[k] & ((1ull << 40) - 1);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
    return pre;
}

}  // namespace geohip
