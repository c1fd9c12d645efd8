// cell_kernels.hip -- tile-binned kernels of libgeohip for gfx950: point-point window join
// (PointPointJoinQuery.java:113-172 + JoinQuery.java:73-90) and point-polygon window range
// (PointPolygonRangeQuery.java:76-124).
//
// Both start from one binning pass of the window's points into square tiles of ts x ts grid
// cells (x-major tiles, at most 128 x 128 of them): a per-block LDS histogram (no per-point
// global atomics), a column-wise scan of the block histograms into per-(block, tile) offsets,
// and an LDS-cursor scatter into SoA x / y / idx / cell key.  Within a tile the points are in
// no particular order; the kernels test the exact cell of every point, so the tile is only a
// locality unit.
//
// Join: the query stream's replication (JoinQuery.getReplicatedPointQueryStream: every query
// copied to each cell of its Nbr block) becomes a tile -> query list; one workgroup per data
// tile stages its candidate queries in LDS and streams the tile's points once against them.
// Point-polygon: one workgroup per (polygon, tile) work item, ring in LDS, exactness-preserving
// screens before the JTS distance.  Pairs leave through per-wave LDS buffers, one global atomic
// per ~1K pairs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <string>
#include <vector>

#include "device_common.h"
#include "join.h"
#include "ppoly.h"
#include "sort.h"

namespace geohip {

constexpr int kTB = 256;             // threads per block (probe kernels, scans)
constexpr int kBinThreads = 1024;    // binning kernels
constexpr unsigned kMaxTiles = 16384;
constexpr unsigned kGlobalTiles = 4096;  // queries touching more tiles go to every tile's list

__device__ __forceinline__ int32_t d_java_d2i(double v) {
    if (v != v) return 0;
    if (v >= 2147483647.0) return INT32_MAX;
    if (v <= -2147483648.0) return INT32_MIN;
    return (int32_t)v;
}

// HelperClass.assignGridCellID per axis: (int)Math.floor((v - min)/l), exact division.
__device__ __forceinline__ int32_t d_axis_cell(double v, double mn, double l) {
    return d_java_d2i(__builtin_floor((v - mn) / l));
}
// The same cell through a multiply by il = fl(1/l): q = fl(t * il) is within |q| 2^-51 of the
// exact quotient t / l, so when q lies farther than |q| 2^-49 from every integer, floor(q) is
// floor(fl(t / l)); otherwise (and for NaN / inf / |q| >= 2^49) the division decides.
// (int) of a double as Java casts it -- NaN -> 0, out of range saturates -- which is what
// v_cvt_i32_f64 does: one instruction instead of d_java_d2i's compare chain.
__device__ __forceinline__ int32_t d_cvt_java(double f) {
    int32_t r;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(r) : "v"(f));
    return r;
}
__device__ __forceinline__ int32_t d_axis_cell_fast(double v, double mn, double l, double il) {
    const double t = v - mn;
    const double q = t * il;
    double f = __builtin_floor(q);
    const double e = __builtin_fabs(q) * 0x1.0p-49 + 0x1.0p-1000;
    const bool ok = (q - f > e) & ((f + 1.0) - q > e);
    if (__ballot(!ok)) {  // wave-uniform, rare: the division decides near integers, NaN, inf
        if (!ok) f = __builtin_floor(t / l);
    }
    return d_cvt_java(f);
}

// d_axis_cell_fast plus the point's subcell (0..3: which quarter of the cell, sub_of's edges):
// from q, the quotient the cell came from -- 4 (q - floor q) is exact in fp64, and it differs
// from the subcell edges' own arithmetic (sub_edge: mn + (c + i / 4) l, rounded twice) by at most
// 2^-51 (6 |q| + |mn| / l + 2) in those units, so outside the margin E below floor(4 (q - f)) is
// sub_of's answer; inside it (or when the cell itself took the division) sub_ok is false and the
// caller evaluates sub_of.
__device__ __forceinline__ int32_t d_axis_cell_sub(double v, double mn, double l, double il, double mnl, unsigned& sub,
                                                   bool& sub_ok) {
    const double t = v - mn;
    const double q = t * il;
    double f = __builtin_floor(q);
    const double e = __builtin_fabs(q) * 0x1.0p-49 + 0x1.0p-1000;
    const bool ok = (q - f > e) & ((f + 1.0) - q > e);
    const double t4 = (q - f) * 4.0;
    const double sf = __builtin_floor(t4);
    const double E = (__builtin_fabs(q) + mnl + 4.0) * 0x1.0p-44;
    sub_ok = ok && (sf < 1.0 || t4 - sf > E) && (sf > 2.0 || (sf + 1.0) - t4 > E);
    sub = sub_ok ? (unsigned)(int)sf : 0u;
    if (__ballot(!ok)) {  // wave-uniform, rare: the division decides near integers, NaN, inf
        if (!ok) f = __builtin_floor(t / l);
    }
    return d_cvt_java(f);
}

// Cell and subcell from ONE floor: q4 = fl(t * il4) with il4 = 4 il (exact) is 4 q exactly (a
// power-of-two scale commutes with rounding), so f4 = floor(q4) = 4 floor(q) + floor(4 (q - floor q))
// -- the cell in its high bits, the subcell in its low two.  When q4 lies farther than
// E = (|q4| + mnl + 4) 2^-44 from every integer, both d_axis_cell_sub's margins hold (its cell
// margin |q| 2^-49 is a multiple-of-4 distance of q4 / 4, its subcell margin is at most E), so
// both answers are d_axis_cell_sub's; otherwise (and for NaN / inf / huge values) that function
// decides.  The (int) of f4 saturates outside +-2^31: those cells lie outside every grid (nb <=
// 65535) as Java's saturated ones do.  (q4 - f4 is exact: f4 <= q4 < f4 + 1.)
__device__ __forceinline__ int32_t d_axis_cell_sub4(double v, double mn, double l, double il, double il4, double mnl,
                                                    unsigned& sub, bool& sub_ok) {
    const double q4 = (v - mn) * il4;
    const double f4 = __builtin_floor(q4);
    const double fr = q4 - f4;
    const double E = (__builtin_fabs(q4) + mnl + 4.0) * 0x1.0p-44;
    const bool ok = (fr > E) & ((1.0 - fr) > E);
    const int32_t fi = d_cvt_java(f4);
    int32_t c = fi >> 2;  // arithmetic: floor(f4 / 4)
    sub = (unsigned)fi & 3u;
    sub_ok = true;
    if (__ballot(!ok)) {  // wave-uniform, rare: the two-step form with its own fallbacks
        if (!ok) c = d_axis_cell_sub(v, mn, l, il, mnl, sub, sub_ok);
    }
    return c;
}

// small zero-fills inside timed steps (a kernel, so its time is stamped like the others)
__global__ void fill_words(unsigned* __restrict__ p, unsigned n, unsigned v) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}
// a step's zero block, and one more 64-bit word (an async call's device count) when z is not null
__global__ void zero_step(unsigned* __restrict__ p, unsigned n, unsigned long long* __restrict__ z,
                          unsigned* __restrict__ p2 = nullptr, unsigned n2 = 0) {
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0u;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += gridDim.x * blockDim.x) p2[i] = 0u;
    if (z && blockIdx.x == 0 && threadIdx.x == 0) *z = 0ull;
}
__global__ void set_u64(unsigned long long* __restrict__ p, unsigned long long v) { *p = v; }

// ------------------------------------------------------------------ scans ----------------
// exclusive scan, 3 phases: per-block totals, scan of totals, per-block rescan + offset
constexpr int kScanPer = 16;
constexpr int kScanSeg = kTB * kScanPer;

template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T* total) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < kTB; o <<= 1) {
        T a = t >= o ? sh[t - o] : T(0);
        __syncthreads();
        sh[t] += a;
        __syncthreads();
    }
    const T incl = sh[t];
    *total = sh[kTB - 1];
    __syncthreads();
    return incl - v;
}

template <typename T>
__global__ void scan_seg_totals(const T* __restrict__ in, uint64_t n, T* __restrict__ seg_tot) {
    __shared__ T sh[kTB];
    const uint64_t base = (uint64_t)blockIdx.x * kScanSeg + (uint64_t)threadIdx.x * kScanPer;
    T s = 0;
    for (int j = 0; j < kScanPer; j++)
        if (base + j < n) s += in[base + j];
    T tot;
    block_excl_scan(s, sh, &tot);
    if (threadIdx.x == 0) seg_tot[blockIdx.x] = tot;
}

template <typename T>
__global__ void scan_totals(T* __restrict__ seg_tot, uint64_t nseg, T* __restrict__ grand) {
    __shared__ T sh[kTB];
    T carry = 0;
    for (uint64_t b = 0; b < nseg; b += kTB) {
        const uint64_t i = b + threadIdx.x;
        const T v = i < nseg ? seg_tot[i] : T(0);
        T tot;
        const T ex = block_excl_scan(v, sh, &tot);
        if (i < nseg) seg_tot[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *grand = carry;
}

// out[i] = sum(in[0..i)); out[n] = total
template <typename T>
__global__ void scan_apply(const T* __restrict__ in, uint64_t n, const T* __restrict__ seg_off,
                           const T* __restrict__ grand, T* __restrict__ out) {
    __shared__ T sh[kTB];
    const uint64_t base = (uint64_t)blockIdx.x * kScanSeg + (uint64_t)threadIdx.x * kScanPer;
    T v[kScanPer];
    T s = 0;
    for (int j = 0; j < kScanPer; j++) {
        v[j] = base + j < n ? in[base + j] : T(0);
        s += v[j];
    }
    T tot;
    T run = seg_off[blockIdx.x] + block_excl_scan(s, sh, &tot);
    for (int j = 0; j < kScanPer; j++) {
        if (base + j < n) out[base + j] = run;
        run += v[j];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = *grand;
}

// ------------------------------------------------------------------ tile binning ---------
// Unsigned division by a launch constant 1 <= d < 2^31 without the ~30-instruction integer
// division sequence: round-up multiplier m = floor(2^32 (2^l - d) / d) + 1, l = ceil(log2 d),
// q = (t + ((n - t) >> 1)) >> (l - 1), t = mulhi(m, n) (Granlund-Montgomery; exact for every
// 32-bit n).  Five integer instructions; the fp64 reciprocal form it replaces cost ~12 VALU
// with three fp64 ones per division, and the binning passes were VALU-issue-bound.
struct FastDiv {
    unsigned m, d;
    unsigned s1, s2;
    __device__ __forceinline__ unsigned div(unsigned n) const {
        const unsigned t = __umulhi(m, n);
        return (t + ((n - t) >> s1)) >> s2;
    }
};
inline FastDiv make_fastdiv(unsigned d) {
    unsigned l = 0;
    while ((1ull << l) < d) l++;
    const unsigned m = (unsigned)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    return FastDiv{m, d, l ? 1u : 0u, l ? l - 1 : 0u};
}

struct TileGeom {
    double mnx, mny, l;  // grid the point cells are computed on
    double il;           // fl(1 / l) (d_axis_cell_fast)
    int32_t nb;          // key space: cells [0, nb)^2 (the query grid's n for the join)
    int32_t ts;          // cells per tile side
    int32_t nt;          // tiles per side
    uint32_t ntiles;     // nt * nt <= kMaxTiles
    FastDiv dts, dnb;    // / ts, / nb
};

__device__ __forceinline__ bool point_cell(const TileGeom& g, double x, double y, int32_t& cx, int32_t& cy) {
    cx = d_axis_cell_fast(x, g.mnx, g.l, g.il);
    cy = d_axis_cell_fast(y, g.mny, g.l, g.il);
    return cx >= 0 && cy >= 0 && cx < g.nb && cy < g.nb;
}
__device__ __forceinline__ unsigned tile_of(const TileGeom& g, int32_t cx, int32_t cy) {
    return g.dts.div((unsigned)cx) * (unsigned)g.nt + g.dts.div((unsigned)cy);
}

// Two binning levels, each a local LDS counting sort so every store leaves in runs: level 1
// sorts the raw window by band (128 consecutive tiles; out-of-grid points last), level 2 sorts
// each band by tile.  A direct one-level scatter into 16K tiles writes partial lines from
// every block (measured 0.3 TB/s on 50M uniform points).
constexpr int kBandBits = 7;
constexpr unsigned kBandTiles = 1u << kBandBits;
constexpr int kLocalBins = 132;   // >= bands + 1 (level 1), >= kBandTiles (level 2)
constexpr unsigned kL2Items = 32768;  // points per level-2 work item
constexpr unsigned kNoKey = 0xffffffffu;

struct SoA {
    double* x;
    double* y;
    unsigned* idx;
    unsigned* key;
};

struct BinPass {
    const double* x;       // level 1 input: the window
    const double* y;
    SoA src;               // level 2 input: level-1 output
    SoA dst;
    uint64_t n, chunk;     // level 1: points, points per block
    TileGeom g;
    unsigned nbands;       // bands of valid tiles; level-1 bin nbands = out of grid
    unsigned* hist;        // level 1: [block][nbands + 1]; level 2: [item][kBandTiles]
    const uint4* items;    // level 2: (band, begin, end, -)
    const unsigned* nitems;
    const unsigned* keep;  // optional cell bitmap (nb * nb bits): points of other cells are dropped
    unsigned keep_words;   // its words; level 1 copies it into LDS when it fits kKeepLds
};

// Level 1 reads the keep bitmap once per point at a random word: from LDS when the bitmap fits
// (nb <= 512), so the per-lane gathers do not go through the vector L1 (bin_*<1, KL = true>).
constexpr unsigned kKeepLds = 8192;

__device__ __forceinline__ unsigned key_tile(const TileGeom& g, unsigned key) {
    const unsigned nb = (unsigned)g.nb;
    const unsigned cx = g.dnb.div(key), cy = key - cx * nb;
    return g.dts.div(cx) * (unsigned)g.nt + g.dts.div(cy);
}

// level-1 point: key (kNoKey when out of the grid); bin: its band, nbands when out of the grid,
// nbands + 1 when its cell is not in the keep bitmap (dropped).  Two steps so the keep-bitmap
// loads of several points go out together (and ahead of any prefetch).
__device__ __forceinline__ unsigned l1_key(const BinPass& a, double px, double py, unsigned& tile) {
    int32_t cx, cy;
    tile = 0;
    if (point_cell(a.g, px, py, cx, cy)) {
        tile = tile_of(a.g, cx, cy);  // from the cell itself: no division of the key
        return (unsigned)cx * (unsigned)a.g.nb + (unsigned)cy;
    }
    return kNoKey;
}
// KL (a launch-time choice: one pointer that may be either would compile to flat loads)
template <bool KL>
__device__ __forceinline__ unsigned l1_keepword(const BinPass& a, const unsigned* kl, unsigned key) {
    if (!a.keep || key == kNoKey) return ~0u;
    return KL ? kl[key >> 5] : a.keep[key >> 5];
}
template <bool KL>
__device__ __forceinline__ void keep_stage(const BinPass& a, unsigned* kl) {
    if (KL)
        for (unsigned t = threadIdx.x; t < a.keep_words; t += kBinThreads) kl[t] = a.keep[t];
}
__device__ __forceinline__ unsigned l1_bin(const BinPass& a, unsigned key, unsigned kw, unsigned tile) {
    if (key == kNoKey) return a.nbands;
    if (!((kw >> (key & 31u)) & 1u)) return a.nbands + 1;
    return tile >> kBandBits;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations, not for its
// outstanding global loads (__syncthreads' workgroup fence would drain those too).  For phases
// whose cross-wave traffic is LDS alone.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// the range of points a block bins: level 1 a chunk of the window, level 2 one work item
template <int LEVEL>
__device__ __forceinline__ bool bin_range(const BinPass& a, uint64_t& b0, uint64_t& b1, unsigned& nbins,
                                          unsigned& band) {
    if (LEVEL == 1) {
        b0 = (uint64_t)blockIdx.x * a.chunk;
        b1 = b0 + a.chunk < a.n ? b0 + a.chunk : a.n;
        nbins = a.nbands + 2;
        band = 0;
        return true;
    }
    if (blockIdx.x >= *a.nitems) return false;
    const uint4 it = a.items[blockIdx.x];
    band = it.x;
    b0 = it.y;
    b1 = it.z;
    nbins = kBandTiles;
    return true;
}

template <bool B>
struct BoolC {
    static constexpr bool value = B;
};

template <int LEVEL, bool KL = false>
__global__ __launch_bounds__(kBinThreads) void bin_count(BinPass a) {
    __shared__ unsigned h[kBinThreads / kWave][kLocalBins];
    __shared__ unsigned kl[KL ? kKeepLds : 1];
    uint64_t b0, b1;
    unsigned nbins, band;
    if (!bin_range<LEVEL>(a, b0, b1, nbins, band)) return;
    keep_stage<KL>(a, kl);
    const int wid = threadIdx.x / kWave;
    for (unsigned t = threadIdx.x; t < (kBinThreads / kWave) * kLocalBins; t += kBinThreads) (&h[0][0])[t] = 0;
    __syncthreads();
    // kU points per thread with all their loads issued first (a single load pair per thread in
    // flight left the pass latency-bound at 2.5 TB/s; level 1 runs one block per CU: 8)
    constexpr unsigned kU = LEVEL == 1 ? 8 : 4;
    // FULL: every thread's kU points are in range (all but the block's last step), so the loads
    // carry no guards and their waits count down one at a time instead of vmcnt(0)
    auto step = [&](uint64_t i0, auto full) {
        constexpr bool FULL = decltype(full)::value;
        double px[kU], py[kU];
        unsigned key[kU], tl[kU];
#pragma unroll
        for (unsigned k = 0; k < kU; k++) {
            const uint64_t i = i0 + (uint64_t)k * kBinThreads;
            if (FULL || i < b1) {
                if (LEVEL == 1) {
                    px[k] = a.x[i];
                    py[k] = a.y[i];
                } else {
                    key[k] = a.src.key[i];
                }
            }
        }
        unsigned kw[kU];
        if (LEVEL == 1) {
#pragma unroll
            for (unsigned k = 0; k < kU; k++) {
                key[k] = l1_key(a, px[k], py[k], tl[k]);
                kw[k] = (FULL || i0 + (uint64_t)k * kBinThreads < b1) ? l1_keepword<KL>(a, kl, key[k]) : ~0u;
            }
        }
#pragma unroll
        for (unsigned k = 0; k < kU; k++) {
            const uint64_t i = i0 + (uint64_t)k * kBinThreads;
            if (FULL || i < b1) {
                const unsigned bin = LEVEL == 1 ? l1_bin(a, key[k], kw[k], tl[k]) : key_tile(a.g, key[k]) - (band << kBandBits);
                if (LEVEL == 2 || bin != a.nbands + 1) atomicAdd(&h[wid][bin], 1u);  // dropped: not counted
            }
        }
    };
    constexpr uint64_t kSpan = (uint64_t)kU * kBinThreads;
    uint64_t s0 = b0;
    for (; s0 + kSpan <= b1; s0 += kSpan) step(s0 + threadIdx.x, BoolC<true>{});
    if (s0 < b1) step(s0 + threadIdx.x, BoolC<false>{});
    __syncthreads();
    if (threadIdx.x < nbins) {
        unsigned c = 0;
        for (int w = 0; w < kBinThreads / kWave; w++) c += h[w][threadIdx.x];
        a.hist[(size_t)blockIdx.x * nbins + threadIdx.x] = c;
    }
}

// level 1: per band, totals over blocks, exclusive scan over bands -> start1[0..nbands+1],
// then hist[b][band] <- where block b writes its band-`band` points.  One block.
__global__ __launch_bounds__(kTB) void bin1_offsets(unsigned* __restrict__ hist, unsigned nblk, unsigned nbins,
                                                    unsigned* __restrict__ start1) {
    __shared__ unsigned sh[kTB];
    const unsigned t = threadIdx.x;
    // The column walks load kBatch rows into registers before using (and, in the second walk,
    // overwriting) them: one serial load -> store chain per row cost ~80 us for 256 rows.
    constexpr unsigned kBatch = 16;
    unsigned tot = 0;
    if (t < nbins)
        for (unsigned b0 = 0; b0 < nblk; b0 += kBatch) {
            unsigned v[kBatch];
#pragma unroll
            for (unsigned k = 0; k < kBatch; k++) v[k] = b0 + k < nblk ? hist[(size_t)(b0 + k) * nbins + t] : 0u;
#pragma unroll
            for (unsigned k = 0; k < kBatch; k++) tot += v[k];
        }
    unsigned all;
    const unsigned st = block_excl_scan(tot, sh, &all);
    if (t < nbins) {
        start1[t] = st;
        unsigned run = st;
        for (unsigned b0 = 0; b0 < nblk; b0 += kBatch) {
            unsigned v[kBatch];
#pragma unroll
            for (unsigned k = 0; k < kBatch; k++) v[k] = b0 + k < nblk ? hist[(size_t)(b0 + k) * nbins + t] : 0u;
#pragma unroll
            for (unsigned k = 0; k < kBatch; k++)
                if (b0 + k < nblk) {
                    hist[(size_t)(b0 + k) * nbins + t] = run;
                    run += v[k];
                }
        }
    }
    if (t == 0) start1[nbins] = all;
}

// level-2 work items: every band cut into pieces of kL2Items points.  One block.
__global__ __launch_bounds__(kTB) void bin2_plan(const unsigned* __restrict__ start1, unsigned nbands,
                                                 uint4* __restrict__ items, unsigned* __restrict__ wfirst,
                                                 unsigned* __restrict__ nitems) {
    __shared__ unsigned sh[kTB];
    const unsigned t = threadIdx.x;
    unsigned cnt = 0, b = 0, e = 0;
    if (t < nbands) {
        b = start1[t];
        e = start1[t + 1];
        cnt = (e - b + kL2Items - 1) / kL2Items;
    }
    unsigned all;
    const unsigned first = block_excl_scan(cnt, sh, &all);
    if (t < nbands) {
        wfirst[t] = first;
        for (unsigned k = 0; k < cnt; k++) {
            const unsigned lo = b + k * kL2Items;
            items[first + k] = make_uint4(t, lo, e - lo > kL2Items ? lo + kL2Items : e, 0u);
        }
    }
    if (t == 0) {
        wfirst[nbands] = all;
        *nitems = all;
    }
}

// level 2, per tile: total over the band's work items (tot), and, after the tile scan, the
// per-item write offsets (OFFS)
template <bool OFFS>
__global__ void bin2_tiles(unsigned* __restrict__ hist, const unsigned* __restrict__ wfirst, uint32_t ntiles,
                           unsigned* __restrict__ tot, const unsigned* __restrict__ start) {
    const unsigned t = blockIdx.x * kTB + threadIdx.x;
    if (t >= ntiles) return;
    const unsigned band = t >> kBandBits, loc = t & (kBandTiles - 1);
    const unsigned w0 = wfirst[band], w1 = wfirst[band + 1];
    if (!OFFS) {
        unsigned c = 0;
        for (unsigned w = w0; w < w1; w++) c += hist[(size_t)w * kBandTiles + loc];
        tot[t] = c;
    } else {
        unsigned run = start[t];
        for (unsigned w = w0; w < w1; w++) {
            const unsigned v = hist[(size_t)w * kBandTiles + loc];
            hist[(size_t)w * kBandTiles + loc] = run;
            run += v;
        }
    }
}

template <int N>
struct SortStage {
    double x[N];
    double y[N];
    unsigned idx[N];
    unsigned key[N];
    unsigned char bin[N];
};

// Local-sort scatter: SUB points at a time are counted by bin in LDS, staged in bin order,
// and stored so consecutive threads write consecutive addresses of one bin's run.  Level 1 runs
// one block per CU over the raw window: 4 points per thread per sub-chunk (64 KB of loads in
// flight per CU; 2 per thread left it latency-bound at ~3 TB/s); level 2 has many more blocks.
template <int LEVEL, bool KL = false>
__global__ __launch_bounds__(kBinThreads) void bin_scatter(BinPass a) {
    constexpr int PPT = LEVEL == 1 ? 4 : 2;
    constexpr int SUB = PPT * kBinThreads;
    __shared__ SortStage<SUB> st;
    __shared__ unsigned cur[kLocalBins], lh[kLocalBins], ls[kLocalBins];
    __shared__ unsigned kl[KL ? kKeepLds : 1];
    uint64_t b0, b1;
    unsigned nbins, band;
    if (!bin_range<LEVEL>(a, b0, b1, nbins, band)) return;
    keep_stage<KL>(a, kl);
    const unsigned* row = a.hist + (size_t)blockIdx.x * nbins;
    for (unsigned t = threadIdx.x; t < kLocalBins; t += kBinThreads) {
        cur[t] = t < nbins ? row[t] : 0u;
        lh[t] = 0;
    }
    __syncthreads();
    // the next sub-chunk's points are loaded while this one is sorted: the barriers below
    // order LDS only (lds_barrier), so those loads stay in flight across them
    double nx[PPT], ny[PPT];
    unsigned nidx[PPT], nkey[PPT];
    auto fetch = [&](uint64_t sb) {
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint64_t i = sb + threadIdx.x + (uint64_t)k * kBinThreads;
            if (i < b1) {
                if (LEVEL == 1) {
                    nx[k] = a.x[i];
                    ny[k] = a.y[i];
                } else {
                    nx[k] = a.src.x[i];
                    ny[k] = a.src.y[i];
                    nidx[k] = a.src.idx[i];
                    nkey[k] = a.src.key[i];
                }
            }
        }
    };
    if (b0 < b1) fetch(b0);
    for (uint64_t sb = b0; sb < b1; sb += SUB) {
        const unsigned m = b1 - sb < (uint64_t)SUB ? (unsigned)(b1 - sb) : (unsigned)SUB;
        double px[PPT], py[PPT];
        unsigned idx[PPT], key[PPT], bin[PPT], rk[PPT];
        unsigned kw[PPT], tl[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kBinThreads;
            px[k] = nx[k];
            py[k] = ny[k];
            idx[k] = LEVEL == 1 ? (unsigned)(sb + j) : nidx[k];
            key[k] = LEVEL == 1 ? l1_key(a, px[k], py[k], tl[k]) : nkey[k];
            kw[k] = (LEVEL == 1 && j < m) ? l1_keepword<KL>(a, kl, key[k]) : ~0u;  // issued before the prefetch
        }
        if (sb + SUB < b1) fetch(sb + SUB);
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kBinThreads;
            bin[k] = a.nbands + 1;  // level 1: dropped unless binned below
            if (j < m) {
                bin[k] = LEVEL == 1 ? l1_bin(a, key[k], kw[k], tl[k]) : key_tile(a.g, key[k]) - (band << kBandBits);
                if (LEVEL == 2 || bin[k] != a.nbands + 1) rk[k] = atomicAdd(&lh[bin[k]], 1u);
            }
        }
        lds_barrier();
        if (threadIdx.x < kWave) {  // exclusive scan of lh over <= 192 bins (3 per lane)
            const int l = threadIdx.x;
            const unsigned v0 = lh[l], v1 = lh[kWave + l], v2 = 2 * kWave + l < kLocalBins ? lh[2 * kWave + l] : 0u;
            const unsigned i0 = wave_incl_scan(v0);
            const unsigned t0 = (unsigned)__builtin_amdgcn_readlane((int)i0, kWave - 1);
            const unsigned i1 = wave_incl_scan(v1) + t0;
            const unsigned t1 = (unsigned)__builtin_amdgcn_readlane((int)i1, kWave - 1);
            const unsigned i2 = wave_incl_scan(v2) + t1;
            ls[l] = i0 - v0;
            ls[kWave + l] = i1 - v1;
            if (2 * kWave + l < kLocalBins) ls[2 * kWave + l] = i2 - v2;
        }
        lds_barrier();
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kBinThreads;
            if (j < m && (LEVEL == 2 || bin[k] != a.nbands + 1)) {  // dropped points are not staged
                const unsigned slot = ls[bin[k]] + rk[k];
                st.x[slot] = px[k];
                st.y[slot] = py[k];
                st.idx[slot] = idx[k];
                st.key[slot] = key[k];
                st.bin[slot] = (unsigned char)bin[k];
            }
        }
        lds_barrier();
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kBinThreads;
            if (j < (LEVEL == 2 ? m : ls[a.nbands + 1])) {  // the staged points: every bin before "dropped"
                const unsigned b = st.bin[j];
                const unsigned g = cur[b] + (j - ls[b]);
                a.dst.x[g] = st.x[j];
                a.dst.y[g] = st.y[j];
                a.dst.idx[g] = st.idx[j];
                a.dst.key[g] = st.key[j];
            }
        }
        lds_barrier();
        for (unsigned t = threadIdx.x; t < nbins; t += kBinThreads) {
            cur[t] += lh[t];
            lh[t] = 0;
        }
        lds_barrier();
    }
}

struct TileBins {
    const double* sx;
    const double* sy;
    const unsigned* sidx;
    const unsigned* skey;
    const unsigned* start;  // ntiles + 1
    int32_t nb;
    FastDiv dnb;            // / nb (key -> cx)
    int32_t ts, nt;         // cells per tile side, tiles per side
    double mnx, mny, l;     // the point grid (subcell edges)
};

// ------------------------------------------------------------------ pair output ----------
// Two passes, no contended counter: the count pass stores each block's pair count in
// bcount[slot0 + block]; an exclusive scan turns the counts into offsets boff; the write pass
// places a block's pairs at boff[slot] + a block-local (LDS) cursor.  Waves collect pairs in
// LDS buffers and copy them out coalesced.
struct PairSink {
    unsigned long long* bcount;       // count pass: pairs per block slot
    const unsigned long long* boff;   // write pass: first output pair of each block slot
    unsigned slot0;                   // slot of block 0 of this launch
    unsigned* out;                    // write pass: pairs, u32 x 2
    uint64_t cap;                     // pairs at or beyond cap are dropped (size reported by the scan)
    int aligned8;                     // out is 8-byte aligned: one 8-byte store per pair
    int swap;                         // store (b, a): the point-polygon join emits (point, polygon)
    unsigned point_base;              // added to every point index (pane stream positions)
};

template <bool WRITE>
__device__ __forceinline__ void pairs_flush(uint2* buf, unsigned long long& cnt, unsigned long long* bsh,
                                            const PairSink& s) {
    if (!WRITE || cnt == 0) return;
    wave_lds_sync();
    unsigned lo = 0, hi = 0;
    if (lane_id() == 0) {
        const unsigned long long b = s.boff[s.slot0 + blockIdx.x] + atomicAdd(bsh, cnt);
        lo = (unsigned)b;
        hi = (unsigned)(b >> 32);
    }
    const unsigned long long base = ((unsigned long long)__shfl(hi, 0) << 32) | __shfl(lo, 0);
    for (unsigned t = lane_id(); t < (unsigned)cnt; t += kWave) {
        const unsigned long long p = base + t;
        if (p < s.cap) {
            const uint2 b = make_uint2(buf[t].x, buf[t].y + s.point_base);  // (polygon, point)
            const uint2 v = s.swap ? make_uint2(b.y, b.x) : b;
            if (s.aligned8) {
                reinterpret_cast<uint2*>(s.out)[p] = v;
            } else {
                s.out[2 * p] = v.x;
                s.out[2 * p + 1] = v.y;
            }
        }
    }
    wave_lds_sync();
    cnt = 0;
}

template <bool WRITE, int CAP>
__device__ __forceinline__ void pairs_push(uint2* buf, unsigned long long& cnt, bool hit, unsigned a, unsigned b,
                                           unsigned long long* bsh, const PairSink& s) {
    const unsigned long long m = __ballot(hit);
    if (!WRITE) {
        cnt += (unsigned long long)__popcll(m);
        return;
    }
    if (m == 0) return;
    if (hit) buf[cnt + lanes_below(m)] = make_uint2(a, b);
    cnt += (unsigned long long)__popcll(m);
    if (cnt > (unsigned long long)(CAP - kWave)) pairs_flush<WRITE>(buf, cnt, bsh, s);
}

// every thread of the block: final flush (write) or the block's count (count)
template <bool WRITE>
__device__ __forceinline__ void pairs_end(uint2* buf, unsigned long long& cnt, unsigned long long* bsh,
                                          const PairSink& s) {
    if (WRITE) pairs_flush<WRITE>(buf, cnt, bsh, s);
    else if (lane_id() == 0 && cnt) atomicAdd(bsh, cnt);
    __syncthreads();
    if (!WRITE && threadIdx.x == 0) s.bcount[s.slot0 + blockIdx.x] = *bsh;
}

// ------------------------------------------------------------------ join -----------------
struct QRect {
    int32_t x0, x1, y0, y1;  // key space, clipped; x0 > x1 = empty
};

__device__ __forceinline__ bool rect_tiles(const QRect& R, const TileGeom& g, int32_t& tx0, int32_t& tx1, int32_t& ty0,
                                           int32_t& ty1) {
    if (R.x0 > R.x1 || R.y0 > R.y1) return false;
    tx0 = R.x0 / g.ts;
    tx1 = R.x1 / g.ts;
    ty0 = R.y0 / g.ts;
    ty1 = R.y1 / g.ts;
    return true;
}

// Query blocks on the device (PointPointJoinQuery.java:113-150 with JoinQuery.
// getReplicatedPointQueryStream, JoinQuery.java:73-90, and UniformGrid.getNeighboringCells,
// UniformGrid.java:261-293): the query's cell on the query grid, its key's round trip through
// HelperClass.getIntCellIndices when the key is not 10 characters, the int-wrapping
// [c - Lc, c + Lc] loops, clipped to the key space.  err: 1 = NumberFormatException,
// 2 = a loop that never terminates (the host reports GEOHIP_ERR_ARG); the query stays empty.
__device__ __forceinline__ int d_format05(int32_t v, char* out) {
    char digits[12];
    int nd = 0;
    int64_t a = v;
    const bool neg = a < 0;
    if (neg) a = -a;
    do {
        digits[nd++] = (char)('0' + (int)(a % 10));
        a /= 10;
    } while (a != 0);
    const int width = nd + (neg ? 1 : 0);
    int p = 0;
    if (neg) out[p++] = '-';
    for (int i = width; i < 5; i++) out[p++] = '0';
    while (nd > 0) out[p++] = digits[--nd];
    return p;
}
// Integer.parseInt(s.replaceFirst("^0+(?!$)", ""))
__device__ __forceinline__ bool d_java_parse(const char* s, int len, int32_t* out) {
    int skip = 0;
    while (skip < len - 1 && s[skip] == '0') skip++;
    s += skip;
    len -= skip;
    if (len <= 0) return false;
    bool neg = false;
    int p = 0;
    if (s[0] == '+' || s[0] == '-') {
        if (len == 1) return false;
        neg = s[0] == '-';
        p = 1;
    }
    int64_t v = 0;
    for (; p < len; p++) {
        if (s[p] < '0' || s[p] > '9') return false;
        v = v * 10 + (s[p] - '0');
        if (v > 2147483648LL) return false;
    }
    if (neg) v = -v;
    if (v > INT32_MAX || v < INT32_MIN) return false;
    *out = (int32_t)v;
    return true;
}

struct JqGeom {
    double mnx, mny, l;  // query grid
    int32_t nb, lc;      // key space side, candidate layers
    int all_cells;       // r == 0: every cell (UniformGrid.java:264-266)
};

// fault (async calls, else null): the ctx's fault word, kFaultQueryKey / kFaultQueryLoop
__global__ __launch_bounds__(kTB) void jq_rect(const double* __restrict__ qx, const double* __restrict__ qy,
                                               uint64_t nq, JqGeom g, QRect* __restrict__ rect,
                                               unsigned* __restrict__ err, unsigned* __restrict__ fault) {
    const uint64_t i = (uint64_t)blockIdx.x * kTB + threadIdx.x;
    if (i >= nq) return;
    QRect R{0, g.nb - 1, 0, g.nb - 1};
    if (!g.all_cells) {
        const int32_t cx = d_axis_cell(qx[i], g.mnx, g.l), cy = d_axis_cell(qy[i], g.mny, g.l);
        int32_t ci = cx, cj = cy;
        bool ok = true;
        if (!(cx >= -9999 && cx <= 99999 && cy >= -9999 && cy <= 99999)) {
            char key[24];
            int n = d_format05(cx, key);
            n += d_format05(cy, key + n);
            ok = d_java_parse(key, 5, &ci) && d_java_parse(key + 5, n - 5, &cj);
        }
        if (!ok) {
            atomicMax(err, 1u);
            if (fault) atomicOr(fault, kFaultQueryKey);
            R = QRect{1, 0, 1, 0};
        } else {
            const int32_t lo_i = (int32_t)(uint32_t)(uint64_t)((int64_t)ci - g.lc);
            const int32_t hi_i = (int32_t)(uint32_t)(uint64_t)((int64_t)ci + g.lc);
            const int32_t lo_j = (int32_t)(uint32_t)(uint64_t)((int64_t)cj - g.lc);
            const int32_t hi_j = (int32_t)(uint32_t)(uint64_t)((int64_t)cj + g.lc);
            if (lo_i > hi_i || lo_j > hi_j) {
                R = QRect{1, 0, 1, 0};
            } else if (hi_i == INT32_MAX || hi_j == INT32_MAX) {
                atomicMax(err, 2u);
                if (fault) atomicOr(fault, kFaultQueryLoop);
                R = QRect{1, 0, 1, 0};
            } else {
                R = QRect{lo_i > 0 ? lo_i : 0, hi_i < g.nb - 1 ? hi_i : g.nb - 1, lo_j > 0 ? lo_j : 0,
                          hi_j < g.nb - 1 ? hi_j : g.nb - 1};
            }
        }
    }
    rect[i] = R;
}

// Query replication as a tile -> query list (every query's block spans at most the host's
// per-query tile bound, <= kGlobalTiles).  FILL = 0: count per tile; FILL = 1: write the lists.
// One wave per query, its lanes over the query's tiles.
template <bool FILL>
__global__ __launch_bounds__(kTB) void jq_build(const QRect* __restrict__ rect, uint64_t nq, TileGeom g,
                                                unsigned* __restrict__ tcnt, const unsigned* __restrict__ qstart,
                                                unsigned* __restrict__ qlist) {
    // FILL: tcnt = the per-tile cursors (zeroed like the counts, a separate array)
    const uint64_t q = (uint64_t)blockIdx.x * (kTB / kWave) + threadIdx.x / kWave;
    if (q >= nq) return;  // wave-uniform
    const unsigned lane = (unsigned)lane_id();
    int32_t tx0, tx1, ty0, ty1;
    if (!rect_tiles(rect[q], g, tx0, tx1, ty0, ty1)) return;
    const unsigned ny = (unsigned)(ty1 - ty0 + 1);
    const unsigned ntl = (unsigned)(tx1 - tx0 + 1) * ny;
    for (unsigned l = lane; l < ntl; l += kWave) {
        const unsigned a = (unsigned)tx0 + l / ny, b = (unsigned)ty0 + l % ny;
        const unsigned t = a * (unsigned)g.nt + b;
        const unsigned k = atomicAdd(&tcnt[t], 1u);
        if (FILL) qlist[qstart[t] + k] = (unsigned)q;
    }
}

// queries whose blocks are too wide for per-tile lists: every tile checks all of them
__global__ void jq_global(uint64_t nq, unsigned* __restrict__ glist, unsigned* __restrict__ gcnt) {
    const uint64_t i = (uint64_t)blockIdx.x * kTB + threadIdx.x;
    if (i < nq) glist[i] = (unsigned)i;
    if (i == 0) *gcnt = (unsigned)nq;
}

// ---- join binning: 16-B point records in two data passes, no count pass ------------------
// The join reads, per point, only what its decisions use: the fp32 coordinates relative to the
// tile origin (the fp32 screen's operands, computed once here exactly as the screen defines
// them), the window index, and the cell inside the tile; the fp64 coordinates are gathered from
// the window by index for the rare exact decisions.  Record = uint4 {fl32(x - ox), fl32(y - oy),
// idx, lcx | lcy << 10 | (tile & 127) << 20} (ts <= 782 < 1024: grids of <= 99999 cells).
//   jb_bands  (one block per CU, its contiguous chunk of the window): each sub-chunk of kJbSub
//             points is sorted by band (128 consecutive tiles) in LDS and written back in place
//             (the same positions: one contiguous 64-KB store per sub-chunk); the sub-chunk's band
//             offsets go to soff; a block-wide LDS tile histogram is added to the tile counts once.
//   jb_scan   tile counts -> tile starts and per-tile cursors (one block); the counts are zeroed
//             before the step by its zero_step launch (the zero block), not here.
//   jb_tiles  one block per (band, group of kJbGroup level-1 blocks): the band's segments of
//             those blocks' sub-chunks, sorted by tile in LDS; each tile's run reserved with one
//             global atomic on its cursor, written contiguously.
// 16 + 16 B per point for level 1, 16 + 16 for level 2 (the SoA form moved 16 + 24 and 24 + 24,
// after two count passes).  The order of a tile's points depends on the cursor atomics -- the
// join's decisions are per point, and its pair order was never fixed.
constexpr unsigned kJbSub = 4096;     // points per local sort round (4 per thread)
constexpr unsigned kJbBlocks = 256;   // level-1 blocks
// Cache hints, each a same-box A/B of round 5 (2 reps): the window read nontemporally by
// jb_bands (jb_bands 92.7 -> 72.6 us); the tile-sorted records stored nontemporally by jb_tiles
// (jb_tiles 95 -> 87, join_fused 813 -> 800 us); not kept: level-1 records stored (jb_tiles 91 ->
// 107-123) or read (no gain) nontemporally.
constexpr unsigned kJbL2Threads = 512;  // level 2: rounds of kJbRound records, 4 blocks per CU
// records per level-2 round (same box, round 5: 512 118, 1024 92, 2048 109 us of jb_tiles)
constexpr unsigned kJbRound = 1024;
constexpr unsigned kJbL2Blocks = 1024;

struct JBin {
    const double* x;
    const double* y;
    uint64_t n, chunk;  // points; points per level-1 block
    TileGeom g;
    unsigned nbands, nsub, nblk;
    uint4* l1;          // level-1 records (block chunks, band-sorted per sub-chunk)
    unsigned* soff;     // [(block * nsub + sub) * (nbands + 1) + band] band starts inside the sub-chunk
    unsigned* tcnt;     // [ntiles] tile counts (zeroed by the step's fill_words launch)
    unsigned* tstart;   // [ntiles + 1]
    unsigned* tcur;     // [ntiles] level-2 cursors
    unsigned* spre;     // [nbands][nblk * nsub + 1] record prefix of each band's non-empty segments
    unsigned* sst;      // [nbands][nblk * nsub] their positions in l1
    unsigned* nne;      // [nbands] non-empty segments
    uint4* rinfo;       // level-2 rounds: (band, first segment, first record, end record)
    unsigned* nround;   // [1]
    uint4* recs;        // tile-sorted records
    // the join's work items, planned by the same launches: per tile ceil(points / kJP) x
    // ceil(queries / kJQ) items (istart by jb_scan, the item list by jb_segs)
    const unsigned* qstart;  // [ntiles + 1] per-tile query list starts
    const unsigned* gcnt;    // [1] queries every tile checks (global mode)
    unsigned* istart;        // [ntiles + 1]
    uint2* items;            // (tile, item within the tile)
};

__device__ __forceinline__ uint4 jb_record(const TileGeom& g, double x, double y, unsigned idx, bool& in, unsigned& tile) {
    int32_t cx, cy;
    in = point_cell(g, x, y, cx, cy);
    tile = 0;
    if (!in) return make_uint4(0u, 0u, 0u, 0u);
    const unsigned tx = g.dts.div((unsigned)cx), ty = g.dts.div((unsigned)cy);
    tile = tx * (unsigned)g.nt + ty;
    const int32_t X0 = (int32_t)tx * g.ts, Y0 = (int32_t)ty * g.ts;
    // the tile origin exactly as join_fused forms it
    const double ox = g.mnx + (double)X0 * g.l, oy = g.mny + (double)Y0 * g.l;
    const float ax = (float)(x - ox), ay = (float)(y - oy);
    const unsigned meta = (unsigned)(cx - X0) | ((unsigned)(cy - Y0) << 10) | ((tile & (kBandTiles - 1)) << 20);
    return make_uint4(__float_as_uint(ax), __float_as_uint(ay), idx, meta);
}

// exclusive scan of lh[0..nbins) (nbins <= 192) into ls by wave 0
__device__ __forceinline__ void lds_bins_scan(const unsigned* lh, unsigned* ls, unsigned nbins) {
    if (threadIdx.x < kWave) {
        const unsigned l = threadIdx.x;
        const unsigned v0 = l < nbins ? lh[l] : 0u, v1 = kWave + l < nbins ? lh[kWave + l] : 0u;
        const unsigned v2 = 2 * kWave + l < nbins ? lh[2 * kWave + l] : 0u;
        const unsigned i0 = wave_incl_scan(v0);
        const unsigned t0 = (unsigned)__builtin_amdgcn_readlane((int)i0, kWave - 1);
        const unsigned i1 = wave_incl_scan(v1) + t0;
        const unsigned t1 = (unsigned)__builtin_amdgcn_readlane((int)i1, kWave - 1);
        const unsigned i2 = wave_incl_scan(v2) + t1;
        if (l < nbins) ls[l] = i0 - v0;
        if (kWave + l < nbins) ls[kWave + l] = i1 - v1;
        if (2 * kWave + l < nbins) ls[2 * kWave + l] = i2 - v2;
        if (l == kWave - 1) ls[nbins] = i2;
    }
}

__global__ __launch_bounds__(kBinThreads) void jb_bands(JBin a) {
    constexpr int PPT = kJbSub / kBinThreads;
    __shared__ uint4 st[kJbSub];
    __shared__ unsigned th[kMaxTiles];
    __shared__ unsigned lh[kLocalBins], ls[kLocalBins + 1];
    const uint64_t b0 = (uint64_t)blockIdx.x * a.chunk;
    const uint64_t b1 = b0 + a.chunk < a.n ? b0 + a.chunk : a.n;
    const unsigned nbins = a.nbands + 1;  // + out of the key space (dropped)
    for (unsigned t = threadIdx.x; t < a.g.ntiles; t += kBinThreads) th[t] = 0;
    for (unsigned t = threadIdx.x; t < kLocalBins; t += kBinThreads) lh[t] = 0;
    __syncthreads();
    // the next sub-chunk's coordinates are loaded while this one is sorted (lds_barrier: LDS only)
    double nx[PPT], ny[PPT];
    // unconditional loads (index clamped into the chunk): a branch per load left the compiler a
    // wait for every earlier memory operation in front of each one
    auto fetch = [&](uint64_t sb) {
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint64_t i = sb + threadIdx.x + (uint64_t)k * kBinThreads;
            const uint64_t ic = i < b1 ? i : b1 - 1;
            // read once here (join_fused reads the records): past the caches
            nx[k] = __builtin_nontemporal_load(a.x + ic);
            ny[k] = __builtin_nontemporal_load(a.y + ic);
        }
    };
    if (b0 < b1) fetch(b0);
    for (unsigned s = 0; s < a.nsub; s++) {
        const uint64_t sb = b0 + (uint64_t)s * kJbSub;
        const unsigned m = sb < b1 ? (b1 - sb < (uint64_t)kJbSub ? (unsigned)(b1 - sb) : kJbSub) : 0u;
        uint4 rec[PPT];
        unsigned bin[PPT], rk[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kBinThreads;
            bin[k] = a.nbands;
            if (j < m) {
                bool in;
                unsigned tile;
                rec[k] = jb_record(a.g, nx[k], ny[k], (unsigned)(sb + j), in, tile);
                if (in) {
                    bin[k] = tile >> kBandBits;
                    atomicAdd(&th[tile], 1u);
                }
                rk[k] = atomicAdd(&lh[bin[k]], 1u);
            }
        }
        if (sb + kJbSub < b1) fetch(sb + kJbSub);
        lds_barrier();
        lds_bins_scan(lh, ls, nbins);
        lds_barrier();
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kBinThreads;
            if (j < m && bin[k] < a.nbands) st[ls[bin[k]] + rk[k]] = rec[k];
        }
        if (threadIdx.x < nbins) a.soff[((size_t)blockIdx.x * a.nsub + s) * nbins + threadIdx.x] = ls[threadIdx.x];
        lds_barrier();
        const unsigned kept = ls[a.nbands];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kBinThreads;
            if (j < kept) {
                a.l1[sb + j] = st[j];
            }
        }
        lds_barrier();
        for (unsigned t = threadIdx.x; t < nbins; t += kBinThreads) lh[t] = 0;
        lds_barrier();
    }
    __syncthreads();
    for (unsigned t = threadIdx.x; t < a.g.ntiles; t += kBinThreads) {
        const unsigned c = th[t];
        if (c) atomicAdd(&a.tcnt[t], c);
    }
}

// Exclusive scan of n <= kMaxTiles words by one block of kBinThreads: every value loaded up front
// (one global round trip: a pass-by-pass scan waited for one per pass, ~1 us each), then 16
// coalesced passes scanned together -- wave scans, one 256-entry scan of the (pass, wave) sums.
// store(i, v, exclusive prefix) per element; returns the total.  wsum: 256 words of LDS.
constexpr unsigned kScanPasses = kMaxTiles / kBinThreads;
template <typename L, typename S>
__device__ __forceinline__ unsigned block_scan_passes(unsigned n, unsigned* wsum, L&& load, S&& store) {
    constexpr unsigned kW = kBinThreads / kWave;  // 16 waves
    const unsigned wid = threadIdx.x / kWave, lane = (unsigned)lane_id();
    unsigned v[kScanPasses], incl[kScanPasses];
#pragma unroll
    for (unsigned p = 0; p < kScanPasses; p++) {
        const unsigned t = p * kBinThreads + threadIdx.x;
        v[p] = t < n ? load(t) : 0u;
    }
#pragma unroll
    for (unsigned p = 0; p < kScanPasses; p++) {
        incl[p] = wave_incl_scan(v[p]);
        if (lane == kWave - 1) wsum[p * kW + wid] = incl[p];
    }
    __syncthreads();
    // (pass, wave) sums in pass-major order: exclusive scan over 256 entries by 4 waves
    unsigned x = 0, xi = 0;
    if (threadIdx.x < kScanPasses * kW) {
        x = wsum[threadIdx.x];
        xi = wave_incl_scan(x);
    }
    __syncthreads();
    __shared__ unsigned wtot[kScanPasses * kW / kWave];
    if (threadIdx.x < kScanPasses * kW && lane == kWave - 1) wtot[wid] = xi;
    __syncthreads();
    if (threadIdx.x < kScanPasses * kW) {
        unsigned b = 0;
        for (unsigned w = 0; w < wid; w++) b += wtot[w];
        wsum[threadIdx.x] = b + xi - x;
    }
    __syncthreads();
    unsigned total = 0;
    for (unsigned w = 0; w < kScanPasses * kW / kWave; w++) total += wtot[w];
#pragma unroll
    for (unsigned p = 0; p < kScanPasses; p++) {
        const unsigned t = p * kBinThreads + threadIdx.x;
        if (t < n) store(t, v[p], wsum[p * kW + wid] + incl[p] - v[p]);
    }
    return total;
}

// Tile starts and cursors from the tile counts, then the join's item starts from the same counts
// and the query list starts (one block; was a separate join_plan launch).
constexpr unsigned kJP = 1024;  // points per join work item (4 waves x 4 chunks of 64)
constexpr unsigned kJQ = 128;   // queries per join work item
__global__ __launch_bounds__(kBinThreads) void jb_scan(JBin a) {
    __shared__ unsigned wsum[kScanPasses * (kBinThreads / kWave)];
    __shared__ unsigned sitems[kMaxTiles];  // item counts, formed while the tile counts load
    const unsigned gq = *a.gcnt;
    const unsigned total = block_scan_passes(
        a.g.ntiles, wsum,
        [&](unsigned t) {
            const unsigned np = a.tcnt[t];
            const unsigned nq = a.qstart[t + 1] - a.qstart[t] + gq;
            sitems[t] = (np == 0 || nq == 0) ? 0u : ((np + kJP - 1) / kJP) * ((nq + kJQ - 1) / kJQ);
            return np;
        },
        [&](unsigned t, unsigned, unsigned ex) {
            a.tstart[t] = ex;
            a.tcur[t] = ex;
        });
    if (threadIdx.x == 0) a.tstart[a.g.ntiles] = total;
    __syncthreads();  // wsum is reused; sitems complete
    const unsigned items = block_scan_passes(
        a.g.ntiles, wsum, [&](unsigned t) { return sitems[t]; }, [&](unsigned t, unsigned, unsigned ex) { a.istart[t] = ex; });
    if (threadIdx.x == 0) a.istart[a.g.ntiles] = items;
}

// Level-2 rounds: each band's records, in (level-1 block, sub-chunk) order, cut into rounds of
// kJbSub; per band the non-empty segments (a sub-chunk's run of the band) with their record
// prefix and window position.  One block per band: its round base from the band totals (the
// tile starts), its segments scanned and compacted, a descriptor per round
// (band, first segment, first record, end record).
__global__ __launch_bounds__(kBinThreads) void jb_segs(JBin a) {
    __shared__ unsigned wsum[2][kBinThreads / kWave];
    __shared__ unsigned sh_rbase;
    const unsigned b = blockIdx.x, nbins = a.nbands + 1, nseg = a.nblk * a.nsub;
    const int wid = threadIdx.x / kWave, lane = lane_id();
    auto band_total = [&](unsigned t) {
        const unsigned e = (t + 1) * kBandTiles < a.g.ntiles ? (t + 1) * kBandTiles : a.g.ntiles;
        return a.tstart[e] - a.tstart[t * kBandTiles];
    };
    // round base: the rounds of bands < b (b <= 128 bands: one per thread of the first waves)
    if (threadIdx.x == 0) sh_rbase = 0;
    __syncthreads();
    if (threadIdx.x < b) {
        const unsigned rb = (band_total(threadIdx.x) + kJbRound - 1) / kJbRound;
        if (rb) atomicAdd(&sh_rbase, rb);
    }
    __syncthreads();
    const unsigned rbase = sh_rbase, T = band_total(b);
    if (b == a.nbands - 1 && threadIdx.x == 0) a.nround[0] = rbase + (T + kJbRound - 1) / kJbRound;
    unsigned* spre = a.spre + (size_t)b * (nseg + 1);
    unsigned* sst = a.sst + (size_t)b * nseg;
    unsigned carry_len = 0, carry_ne = 0;
    constexpr unsigned kG = 4;  // passes whose segment rows are loaded together (one round trip)
    for (unsigned g0 = 0; g0 < nseg; g0 += kG * kBinThreads) {
        unsigned len[kG], gst[kG];
#pragma unroll
        for (unsigned u = 0; u < kG; u++) {
            const unsigned sg = g0 + u * kBinThreads + threadIdx.x;
            len[u] = 0;
            gst[u] = 0;
            if (sg < nseg) {
                const unsigned blk = sg / a.nsub, sub = sg - blk * a.nsub;
                const unsigned* row = a.soff + (size_t)sg * nbins;
                const unsigned lo = row[b], hi = row[b + 1];
                len[u] = hi - lo;
                gst[u] = (unsigned)((uint64_t)blk * a.chunk + (uint64_t)sub * kJbSub) + lo;
            }
        }
#pragma unroll
        for (unsigned u = 0; u < kG; u++) {
            if (g0 + u * kBinThreads >= nseg) break;  // block-uniform
            const unsigned ne = len[u] ? 1u : 0u;
            const unsigned il = wave_incl_scan(len[u]), in = wave_incl_scan(ne);
            if (lane == kWave - 1) {
                wsum[0][wid] = il;
                wsum[1][wid] = in;
            }
            __syncthreads();
            unsigned bl = carry_len, bn = carry_ne, tl = 0, tn = 0;
            for (int w = 0; w < kBinThreads / kWave; w++) {
                if (w < wid) {
                    bl += wsum[0][w];
                    bn += wsum[1][w];
                }
                tl += wsum[0][w];
                tn += wsum[1][w];
            }
            if (ne) {
                const unsigned pre = bl + il - len[u], idx = bn + in - ne;
                spre[idx] = pre;
                sst[idx] = gst[u];
                // the rounds whose first record lies in this segment
                for (unsigned k = (pre + kJbRound - 1) / kJbRound; (uint64_t)k * kJbRound < (uint64_t)pre + len[u]; k++) {
                    const unsigned v0 = k * kJbRound;
                    a.rinfo[rbase + k] = make_uint4(b, idx, v0, T - v0 < kJbRound ? T : v0 + kJbRound);
                }
            }
            carry_len += tl;
            carry_ne += tn;
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        spre[carry_ne] = carry_len;  // = T: the end of the last segment
        a.nne[b] = carry_ne;
    }
    // the join's work items of this band's tiles (was a separate join_item_fill launch)
    const unsigned t0 = b * kBandTiles, t1 = t0 + kBandTiles < a.g.ntiles ? t0 + kBandTiles : a.g.ntiles;
    for (unsigned t = t0 + (unsigned)wid; t < t1; t += kBinThreads / kWave) {
        const unsigned ib = a.istart[t], ie = a.istart[t + 1];
        for (unsigned k = ib + (unsigned)lane; k < ie; k += kWave) a.items[k] = make_uint2(t, k - ib);
    }
}

// Level 2: persistent blocks over the rounds (static stride: every round holds <= kJbRound records).
// A round's segments come into LDS in windows of kJbSegBatch; each record finds its segment by a
// wave-uniform binary search and a per-lane forward step; the round is sorted by tile in LDS and
// each tile's run reserved with one atomic on its cursor.
__global__ __launch_bounds__(kJbL2Threads) void jb_tiles(JBin a) {
    constexpr int PPT = kJbRound / kJbL2Threads;
    constexpr unsigned kWin = kJbL2Threads;  // segments per window
    __shared__ uint4 st[kJbRound];
    __shared__ unsigned wst[kWin], wpre[kWin + 1];
    __shared__ unsigned lh[kBandTiles], ls[kBandTiles + 1], base[kBandTiles];
    const unsigned nseg = a.nblk * a.nsub;
    const unsigned nround = a.nround[0];
    const int wid = threadIdx.x / kWave;
    for (unsigned t = threadIdx.x; t < kBandTiles; t += kJbL2Threads) lh[t] = 0;
    uint4 ninfo = blockIdx.x < nround ? a.rinfo[blockIdx.x] : make_uint4(0u, 0u, 0u, 0u);
    for (unsigned r = blockIdx.x; r < nround; r += gridDim.x) {
        const uint4 info = ninfo;
        if (r + gridDim.x < nround) ninfo = a.rinfo[r + gridDim.x];  // the next round's, in flight meanwhile
        const unsigned b = info.x, v0 = info.z, v1 = info.w;
        const unsigned nne = a.nne[b];
        const unsigned* spre = a.spre + (size_t)b * (nseg + 1);
        const unsigned* sst = a.sst + (size_t)b * nseg;
        uint4 rec[PPT];
        unsigned bin[PPT], rk[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            rec[k] = make_uint4(0u, 0u, 0u, 0u);
            bin[k] = rk[k] = 0u;
        }
        unsigned wb = info.y;  // the window's first segment
        for (;;) {
            const unsigned wl = nne - wb < kWin ? nne - wb : kWin;
            __syncthreads();  // the previous window is no longer read
            if (threadIdx.x < wl) {
                wst[threadIdx.x] = sst[wb + threadIdx.x];
                wpre[threadIdx.x] = spre[wb + threadIdx.x];
            }
            if (threadIdx.x == 0) wpre[wl] = spre[wb + wl];
            __syncthreads();
            const unsigned wlo = wpre[0], whi = wpre[wl];
            // the PPT record addresses first, then their loads together, then the bins: one
            // global round trip per window instead of one per record (each bin's LDS atomic
            // used to wait for its record before the next load was issued)
            unsigned src[PPT];
            bool has[PPT];
#pragma unroll
            for (int k = 0; k < PPT; k++) {
                const unsigned v = v0 + threadIdx.x + k * kJbL2Threads;
                const unsigned vw = v0 + (unsigned)(wid * kWave) + k * kJbL2Threads;  // the wave's first
                has[k] = false;
                src[k] = 0;
                if (vw + kWave > wlo && vw < whi && vw < v1) {  // wave-uniform: some lane in this window
                    const unsigned key = vw > wlo ? vw : wlo;
                    unsigned lo = 0, hi = wl;  // largest j with wpre[j] <= key
                    while (hi - lo > 1) {
                        const unsigned mid = (lo + hi) >> 1;
                        if (wpre[mid] <= key) lo = mid;
                        else hi = mid;
                    }
                    if (v >= wlo && v < whi && v < v1) {
                        unsigned j = lo;
                        while (wpre[j + 1] <= v) j++;
                        has[k] = true;
                        src[k] = wst[j] + (v - wpre[j]);
                    }
                }
            }
            uint4 got[PPT];
#pragma unroll
            for (int k = 0; k < PPT; k++) {  // unconditional (src 0 when none): no branch per load
                got[k] = a.l1[src[k]];
            }
#pragma unroll
            for (int k = 0; k < PPT; k++) {
                rec[k].x = has[k] ? got[k].x : rec[k].x;  // selects, not stores under a branch (kept in VGPRs)
                rec[k].y = has[k] ? got[k].y : rec[k].y;
                rec[k].z = has[k] ? got[k].z : rec[k].z;
                rec[k].w = has[k] ? got[k].w : rec[k].w;
                const unsigned bk = (got[k].w >> 20) & (kBandTiles - 1);
                bin[k] = has[k] ? bk : bin[k];
                if (has[k]) rk[k] = atomicAdd(&lh[bk], 1u);
            }
            if (whi >= v1 || wb + wl >= nne) break;
            wb += wl;
        }
        __syncthreads();
        lds_bins_scan(lh, ls, kBandTiles);
        if (threadIdx.x < kBandTiles && lh[threadIdx.x]) {
            base[threadIdx.x] = atomicAdd(&a.tcur[b * kBandTiles + threadIdx.x], lh[threadIdx.x]);
        }
        __syncthreads();
        const unsigned m = v1 - v0;
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kJbL2Threads;
            if (j < m) st[ls[bin[k]] + rk[k]] = rec[k];
        }
        lds_barrier();
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const unsigned j = threadIdx.x + k * kJbL2Threads;
            if (j < m) {
                const uint4 q = st[j];
                const unsigned bq = (q.w >> 20) & (kBandTiles - 1);
                const unsigned p = base[bq] + (j - ls[bq]);
                typedef unsigned u4v __attribute__((ext_vector_type(4)));
                u4v v = {q.x, q.y, q.z, q.w};
                // bounded even if the counts were not the binning's own; nontemporal (see kJbRound)
                if (p < a.n) __builtin_nontemporal_store(v, reinterpret_cast<u4v*>(a.recs + p));
            }
        }
        lds_barrier();
        for (unsigned t = threadIdx.x; t < kBandTiles; t += kJbL2Threads) lh[t] = 0;
    }
}

// ---- single-pass join: balanced work items, decoupled look-back, staged pair runs ---------
// Work item = (tile, up to kJP of its points, up to kJQ of its candidate queries).  Dense tiles
// become many items (the C3 Gaussian window has tiles with thousands of points and hundreds of
// queries), so the grid stays balanced.  A persistent grid takes items in order from a ticket;
// each item
//   1. classifies its queries against the tile's box (rect vs the tile's cells, then box
//      distances with proven margins): MISS (no point of the tile can pair), ALL (every point
//      pairs: the block covers the tile and the tile lies inside the circle) or PART,
//   2. counts its pairs: |ALL| per valid point, and for PART queries per point the block test
//      and a packed-fp32 distance screen on coordinates relative to the tile origin (error
//      bound per item, below), the exact fp64 / JTS distance only in the screen's band,
//   3. takes its output run with one atomic add of its count (output order: item runs in the
//      order items finish counting, pairs inside a run in a fixed order),
//   4. recomputes the same decisions and writes (point, query) pairs through a per-wave LDS
//      stage that leaves in contiguous runs (512-byte stores).
// Emit (p, q) iff key(p) lies in q's Nbr block and (approximate or dist(p, q) <= r)
// (PointPointJoinQuery.java:156-160).
//
// fp32 screen: a = fl32(p - o), b = fl32(q - o) per axis (o = tile origin), d2' = dx'^2 + dy'^2
// in fp32.  With A >= |p - o| + |q - o| on both axes over the item and u = 2^-24,
// |dx' - dx| <= e = 2.05 u A, so |d2' - d2| <= 4 e A + 2 e^2 + 3 u d2'.  d2' below lo (above hi)
// puts the true d2 below r2lo (above r2hi), where the fp64 screens already decide (kSqLo/kSqHi).
constexpr unsigned kJCh = kJP / kWave / (kTB / kWave);  // chunks per wave and item
// persistent grid of the write pass: 31.2 KB of LDS with 352-pair stages, 5 blocks per CU (89
// VGPRs allow 5 waves per SIMD).  C3 kernel sums, one box, round 4 (nontemporal pair stores):
// stage 512 at 4 blocks per CU 1278 us; 640 / 768 / 896 at 3: 1265 / 1262 / 1262; 1024 at 2: 1360;
// 320 at 5: 1333.  Round 5, plain stores (same box, 2 reps): 768 at 3: 1176-1184; 512 at 4:
// 1081-1089; 448 at 4: 1078-1091; 352 at 5: 1066-1067 -- with cached stores occupancy beats runs
constexpr unsigned kJBlocksW = 1280;
constexpr unsigned kJBlocksC = 1280;  // count pass (4 KB LDS, 83 VGPRs: 5 blocks per CU)

// query list starts per tile (one block)
__global__ __launch_bounds__(kBinThreads) void jq_starts(const unsigned* __restrict__ qcnt, uint32_t ntiles,
                                                          unsigned* __restrict__ qstart) {
    __shared__ unsigned wsum[kScanPasses * (kBinThreads / kWave)];
    const unsigned total = block_scan_passes(
        ntiles, wsum, [&](unsigned t) { return qcnt[t]; }, [&](unsigned t, unsigned, unsigned ex) { qstart[t] = ex; });
    if (threadIdx.x == 0) qstart[ntiles] = total;
}


struct JoinRun {
    const uint4* recs;       // tile-sorted point records (jb_tiles)
    const unsigned* tstart;  // [ntiles + 1]
    const double* px;        // the window (fp64 coordinates of the exact decisions, by index)
    const double* py;
    TileGeom geo;
    const unsigned* qstart;
    const unsigned* qlist;
    const unsigned* glist;
    const unsigned* gcnt;
    const double* qx;
    const double* qy;
    const QRect* rect;
    double r, r2lo, r2hi;
    const unsigned* istart;  // [ntiles] = item count
    const uint2* items;
    uint32_t ntiles;
    unsigned* ticket;
    unsigned long long* total;   // output cursor = pair total
    unsigned* out;
    uint64_t cap;
    int aligned8;
};

typedef float jf2 __attribute__((ext_vector_type(2)));

// a jb_record: tile-relative fp32 coordinates, window index, cell (tile origin X0, Y0 + local)
__device__ __forceinline__ void jrec_load(const uint4 r, int32_t X0, int32_t Y0, float& ax, float& ay, unsigned& pid,
                                          int32_t& cx, int32_t& cy) {
    ax = __uint_as_float(r.x);
    ay = __uint_as_float(r.y);
    pid = r.z;
    cx = X0 + (int32_t)(r.w & 1023u);
    cy = Y0 + (int32_t)((r.w >> 10) & 1023u);
}

struct JPart {  // a PART query: block as (x0, x1 - x0, y0, y1 - y0), tile-relative fp32 coordinates
    int32_t x0, wx, y0, wy;
};

// pair (point, query) at output position p (< cap)
__device__ __forceinline__ void jpair_store(const JoinRun& a, unsigned long long p, unsigned pid, unsigned q) {
    if (a.aligned8) {  // one 8-byte store per pair (plain: nontemporal stores measured 1028 against
                       // 933 us for C3's join_fused, same box -- the L2 merges the runs' partial lines)
        reinterpret_cast<unsigned long long*>(a.out)[p] = ((unsigned long long)q << 32) | pid;
    } else {
        a.out[2 * p] = pid;
        a.out[2 * p + 1] = q;
    }
}


// hit ballots of one point chunk against PART queries j .. j + 3 (padded past the count): the
// four blocks and screen operands read together, one wave-uniform branch for the rare band
template <bool APPROX>
__device__ __forceinline__ void jpart_quad(const JoinRun& a, const JPart* __restrict__ pr, const jf2* __restrict__ pb,
                                           const unsigned* __restrict__ pq, unsigned j, int32_t cx, int32_t cy,
                                           float ax, float ay, unsigned pid, float lo, float hi,
                                           unsigned long long (&m)[4]) {
    // branch-free: every block is read whatever the lane (invalid lanes carry cx = -1 and fail)
    const unsigned ux = (unsigned)cx, uy = (unsigned)cy;
    bool h[4], band[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const JPart R = pr[j + u];
        const bool in = (ux - (unsigned)R.x0 <= (unsigned)R.wx) & (uy - (unsigned)R.y0 <= (unsigned)R.wy);
        if (APPROX) {
            h[u] = in;
            band[u] = false;
        } else {
            const jf2 b = pb[j + u];
            const float dx = ax - b.x, dy = ay - b.y;
            const float d2 = dx * dx + dy * dy;
            h[u] = in && d2 < lo;
            band[u] = in && !(d2 < lo) && !(d2 > hi);
        }
    }
    if (!APPROX && __ballot(band[0] || band[1] || band[2] || band[3])) {  // rare: fp64 screens, then JTS
        const double px = a.px[pid], py = a.py[pid];
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (band[u]) {
                const unsigned q = pq[j + u];
                const double ox = a.qx[q], oy = a.qy[q];
                const double ex = px - ox, ey = py - oy, e2 = ex * ex + ey * ey;
                h[u] = e2 <= a.r2lo || (!(e2 > a.r2hi) && jts_pp_distance(px, py, ox, oy) <= a.r);
            }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) m[u] = __ballot(h[u]);
}

// A wave's pair stage: pairs leave in contiguous runs of full 512-B wave stores.  (One store per
// (chunk, query) straight from the ballots -- no stage -- measured slower: 1.13 ms against 1.04 ms
// for C3's write pass; the partial-wave stores are ~3x as many instructions for the same bytes.)
constexpr unsigned kJStage = 352;   // pairs per wave (6 KB)
__device__ __forceinline__ void jstage_flush(const JoinRun& a, uint2* st, unsigned& cnt, unsigned long long& pos) {
    wave_lds_sync();
    for (unsigned t = (unsigned)lane_id(); t < cnt; t += kWave) {
        const unsigned long long p = pos + t;
        if (p < a.cap) {
            const uint2 v = st[t];
            jpair_store(a, p, v.x, v.y);
        }
    }
    wave_lds_sync();
    pos += cnt;
    cnt = 0;
}

// The pairs of one chunk of 64 points: ALL queries (the in-box ballot vm) and PART queries (the
// kept hit ballots), from position pos on (advanced).  A full chunk's ALL pairs go straight out as
// 512-B wave stores; the rest through the stage (st, sc), flushed when fewer than 4 x 64 slots
// remain (the most one step adds).
__device__ __forceinline__ void jemit_chunk(const JoinRun& a, unsigned long long vm, unsigned pid,
                                            const unsigned* __restrict__ lall, unsigned nall,
                                            const unsigned* __restrict__ lpq, unsigned npart,
                                            const ulonglong2* __restrict__ masks, uint2* st, unsigned& sc,
                                            unsigned long long& pos) {
    const unsigned lane = (unsigned)lane_id();
    const bool in_box = (vm >> lane) & 1ull;
    const unsigned vrank = lanes_below(vm), vcnt = (unsigned)__popcll(vm);
    if (vcnt == kWave) {
        unsigned j = 0;
        for (; j + 4 <= nall; j += 4) {  // four queries' ids in one LDS read
            const uint4 q4 = *reinterpret_cast<const uint4*>(&lall[j]);
            const unsigned long long p = pos + lane;
            if (p < a.cap) jpair_store(a, p, pid, q4.x);
            if (p + kWave < a.cap) jpair_store(a, p + kWave, pid, q4.y);
            if (p + 2 * kWave < a.cap) jpair_store(a, p + 2 * kWave, pid, q4.z);
            if (p + 3 * kWave < a.cap) jpair_store(a, p + 3 * kWave, pid, q4.w);
            pos += 4 * kWave;
        }
        for (; j < nall; j++) {
            const unsigned long long p = pos + lane;
            if (p < a.cap) jpair_store(a, p, pid, lall[j]);
            pos += kWave;
        }
    } else {
        for (unsigned j = 0; j < nall; j++) {
            if (in_box) st[sc + vrank] = make_uint2(pid, lall[j]);
            sc += vcnt;
            if (sc > kJStage - 4 * kWave) jstage_flush(a, st, sc, pos);
        }
    }
    for (unsigned j = 0; j < npart; j += 4) {  // four queries per step, reads first
        const ulonglong2 ma = masks[j / 2], mb = masks[j / 2 + 1];
        const unsigned long long mq[4] = {ma.x, ma.y, mb.x, mb.y};
        const unsigned qq[4] = {lpq[j], lpq[j + 1], lpq[j + 2], lpq[j + 3]};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if ((mq[u] >> lane) & 1ull) st[sc + lanes_below(mq[u])] = make_uint2(pid, qq[u]);
            sc += (unsigned)__popcll(mq[u]);
        }
        if (sc > kJStage - 4 * kWave) jstage_flush(a, st, sc, pos);
    }
}

template <bool APPROX, bool WRITE>
__global__ __launch_bounds__(kTB) void join_fused(JoinRun a) {
    __shared__ __attribute__((aligned(16))) unsigned lall[kJQ];  // ALL queries
    __shared__ unsigned lpq[kJQ + 4];    // PART queries (+ padding to a multiple of 4)
    __shared__ JPart lpr[kJQ + 4];
    __shared__ jf2 lpb[kJQ + 4];
    __shared__ uint2 stage[WRITE ? kTB / kWave : 1][WRITE ? kJStage : 1];
    __shared__ ulonglong2 lmask[WRITE ? kTB / kWave : 1][WRITE ? kJCh : 1][WRITE ? kJQ / 2 : 1];  // PART ballots
    __shared__ unsigned sh_item, sh_nall, sh_npart, sh_amax, sh_wc[2][kTB / kWave];
    __shared__ unsigned long long sh_wcnt[kTB / kWave], sh_off;
    const int wid = threadIdx.x / kWave, lane = lane_id();
    const unsigned nitems = a.istart[a.ntiles];
    const unsigned gq = *a.gcnt;
    const TileGeom& g = a.geo;
    const double slack = 0x1.0p-30 * (__builtin_fabs(g.mnx) + __builtin_fabs(g.mny) + ((double)g.nb + 2.0) * g.l);
#ifdef GEOHIP_JOIN_TRACE  // measurement build (scripts/join_tail.py): per block start, end, items, last item start
    unsigned long long* tr = reinterpret_cast<unsigned long long*>(a.out) + (a.cap - 4 * 2048);
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_last = t_start;
    unsigned n_items = 0;
#endif
    for (bool first = true;; first = false) {
        if (threadIdx.x == 0) {  // the block's first item by its index, the rest from the ticket
            sh_item = first ? blockIdx.x : gridDim.x + atomicAdd(a.ticket, 1u);
            sh_amax = 0;
        }
        __syncthreads();
        // uniform in fact and, through readfirstlane, to the compiler: a loop exit it treats as
        // divergent gets structured with lane 0 outside the barrier loop (hangs)
        const unsigned it = (unsigned)__builtin_amdgcn_readfirstlane((int)sh_item);
        if (it >= nitems) break;
#ifdef GEOHIP_JOIN_TRACE
        t_last = __builtin_amdgcn_s_memrealtime();
        n_items++;
#endif
        const uint2 d = a.items[it];
        const unsigned tile = d.x;
        const unsigned qs = a.qstart[tile], nql = a.qstart[tile + 1] - qs, nqt = nql + gq;
        const unsigned nqc = (nqt + kJQ - 1) / kJQ;
        const unsigned pc = d.y / nqc, qc = d.y - pc * nqc;
        const unsigned ds = a.tstart[tile] + pc * kJP;
        const unsigned de0 = a.tstart[tile + 1];
        const unsigned de = ds + kJP < de0 ? ds + kJP : de0;
        const unsigned q0 = qc * kJQ;
        const unsigned nbq = nqt - q0 < kJQ ? nqt - q0 : kJQ;
        // the tile's cells and its coordinate box (slack covers the cell rounding of its points)
        const int32_t tx = (int32_t)(tile / (unsigned)g.nt), ty = (int32_t)(tile % (unsigned)g.nt);
        const int32_t X0 = tx * g.ts, Y0 = ty * g.ts;
        const int32_t X1 = X0 + g.ts - 1 < g.nb - 1 ? X0 + g.ts - 1 : g.nb - 1;
        const int32_t Y1 = Y0 + g.ts - 1 < g.nb - 1 ? Y0 + g.ts - 1 : g.nb - 1;
        const double ox = g.mnx + (double)X0 * g.l, oy = g.mny + (double)Y0 * g.l;
        const double bx0 = ox - slack, by0 = oy - slack;
        const double bx1 = g.mnx + (double)(X1 + 1) * g.l + slack, by1 = g.mny + (double)(Y1 + 1) * g.l + slack;
        // 1. classify the item's queries
        int cls = 0;  // 0 miss, 1 all, 2 part
        unsigned q = 0;
        QRect R{1, 0, 1, 0};
        double qxv = 0.0, qyv = 0.0;
        if (threadIdx.x < nbq) {
            const unsigned t = q0 + threadIdx.x;
            q = t < nql ? a.qlist[qs + t] : a.glist[t - nql];
            R = a.rect[q];
            qxv = a.qx[q];
            qyv = a.qy[q];
            const bool inter = R.x0 <= R.x1 && R.y0 <= R.y1 && R.x0 <= X1 && R.x1 >= X0 && R.y0 <= Y1 && R.y1 >= Y0;
            const bool cover = R.x0 <= X0 && R.x1 >= X1 && R.y0 <= Y0 && R.y1 >= Y1;
            if (APPROX) {
                cls = !inter ? 0 : (cover ? 1 : 2);
            } else if (inter) {
                const double ex0 = __builtin_fmax(__builtin_fmax(bx0 - qxv, qxv - bx1), 0.0);
                const double ey0 = __builtin_fmax(__builtin_fmax(by0 - qyv, qyv - by1), 0.0);
                const double dmin2 = ex0 * ex0 + ey0 * ey0;
                const double ex1 = __builtin_fmax(__builtin_fabs(qxv - bx0), __builtin_fabs(qxv - bx1));
                const double ey1 = __builtin_fmax(__builtin_fabs(qyv - by0), __builtin_fabs(qyv - by1));
                const double dmax2 = ex1 * ex1 + ey1 * ey1;
                if (dmin2 * (1.0 - 0x1.0p-40) > a.r2hi) cls = 0;
                else if (cover && dmax2 * (1.0 + 0x1.0p-40) < a.r2lo) cls = 1;
                else cls = 2;
            }
        }
        // compaction in query order: ALL and PART lists
        {
            const unsigned long long ma = __ballot(cls == 1), mp = __ballot(cls == 2);
            if (lane == 0) {
                sh_wc[0][wid] = (unsigned)__popcll(ma);
                sh_wc[1][wid] = (unsigned)__popcll(mp);
            }
            __syncthreads();
            unsigned ba = 0, bp = 0, ta = 0, tp = 0;
            for (int w = 0; w < kTB / kWave; w++) {
                if (w < wid) {
                    ba += sh_wc[0][w];
                    bp += sh_wc[1][w];
                }
                ta += sh_wc[0][w];
                tp += sh_wc[1][w];
            }
            if (cls == 1) lall[ba + lanes_below(ma)] = q;
            if (cls == 2) {
                const unsigned k = bp + lanes_below(mp);
                lpq[k] = q;
                lpr[k] = JPart{R.x0, R.x1 - R.x0, R.y0, R.y1 - R.y0};
                const float fx = (float)(qxv - ox), fy = (float)(qyv - oy);
                lpb[k] = jf2{fx, fy};
                const float m = __builtin_fmaxf(__builtin_fabsf(fx), __builtin_fabsf(fy));
                atomicMax(&sh_amax, m == m ? __float_as_uint(m) : 0x7f800000u);  // NaN -> no fp32 screen
            }
            if (threadIdx.x == 0) {
                sh_nall = ta;
                sh_npart = tp;
                for (unsigned u = tp; u < tp + 4; u++) {  // padding: never inside
                    lpr[u] = JPart{INT32_MAX, 0, INT32_MAX, 0};
                    lpb[u] = jf2{0.f, 0.f};
                    lpq[u] = 0;
                }
            }
        }
        __syncthreads();
        const unsigned nall = sh_nall, npart = sh_npart;
        // fp32 screen bounds of this item (A: point side <= the box extent, query side measured)
        float lo = -1.0f, hi = __builtin_inff();
        if (!APPROX) {
            const double pa = (bx1 - bx0) + (by1 - by0);
            const double A = pa + 2.0 * (double)__uint_as_float(sh_amax) * (1.0 + 0x1.0p-20);
            const double e = 2.05 * 0x1.0p-24 * A;
            const double err = 4.0 * e * A + 2.0 * e * e;
            if (err == err && err < 0x1.0p100) {
                if (a.r2lo > 0.0) {
                    const double l = (a.r2lo - err) * (1.0 - 0x1.0p-21);
                    lo = l > 0.0 ? __double2float_rd(l) : -1.0f;
                }
                if (a.r2hi < 0x1.0p100) hi = __double2float_ru((a.r2hi + err) * (1.0 + 0x1.0p-21));
            } else {
                lo = -1.0f;  // every in-block lane takes the exact path (NaN hi: never "certainly above")
                hi = __builtin_nanf("");
            }
        }
        // 2. count: the wave's chunks w, w + 4, ... of 64 points.  The write pass keeps every
        //    decision of this phase -- each chunk's window indices and in-box ballot in registers,
        //    the PART hit ballots in LDS -- so the emission issues no global load: on gfx9 a load's
        //    wait also waits for every store issued before it, so a load in the emission would hold
        //    the wave until its previous pair stores had drained.
        const unsigned nch = (de - ds + 63) / 64;
        unsigned long long cnt = 0;
        uint4 rk[kJCh];
        unsigned pidk[kJCh];
        unsigned long long vmk[kJCh];
#pragma unroll
        for (unsigned k = 0; k < kJCh; k++) {  // the wave's records first: their loads in flight together
            const unsigned c = (unsigned)wid + k * (kTB / kWave);
            const unsigned i = ds + c * 64 + (unsigned)lane;
            rk[k] = make_uint4(0u, 0u, 0u, 0u);
            if (c < nch && i < de) rk[k] = a.recs[i];  // (nontemporal: no gain, round 5)
        }
#pragma unroll
        for (unsigned k = 0; k < kJCh; k++) {
            const unsigned c = (unsigned)wid + k * (kTB / kWave);
            vmk[k] = 0;
            pidk[k] = 0;
            if (c >= nch) continue;  // wave-uniform
            const unsigned i = ds + c * 64 + (unsigned)lane;
            const bool valid = i < de;
            float ax = 0.f, ay = 0.f;
            unsigned pid = 0;
            int32_t cx = -1, cy = -1;
            if (valid) jrec_load(rk[k], X0, Y0, ax, ay, pid, cx, cy);
            // ALL queries pair every point of the chunk whose coordinates lie in the tile box: a
            // NaN coordinate is keyed to cell 0 by the (int) cast yet has no distance <= r
            // (the approximate join pairs it by cell alone; fl32 of NaN - o is NaN, of a finite
            // difference never)
            const bool in_box = valid && (APPROX || (ax == ax && ay == ay));
            const unsigned long long vm = __ballot(in_box);
            vmk[k] = vm;
            pidk[k] = pid;
            cnt += (unsigned long long)nall * (unsigned)__popcll(vm);
            for (unsigned j = 0; j < npart; j += 4) {
                unsigned long long m[4];
                jpart_quad<APPROX>(a, lpr, lpb, lpq, j, cx, cy, ax, ay, pid, lo, hi, m);
                if (WRITE && lane == 0) {
                    lmask[WRITE ? wid : 0][WRITE ? k : 0][WRITE ? j / 2 : 0] = make_ulonglong2(m[0], m[1]);
                    lmask[WRITE ? wid : 0][WRITE ? k : 0][WRITE ? j / 2 + 1 : 0] = make_ulonglong2(m[2], m[3]);
                }
                cnt += (unsigned)(__popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]) + __popcll(m[3]));
            }
        }
        if (lane == 0) sh_wcnt[wid] = cnt;
        __syncthreads();
        unsigned long long tot = 0;
        for (int w = 0; w < kTB / kWave; w++) tot += sh_wcnt[w];
        // 3. the item's output run: one atomic per item (a decoupled look-back in item order made
        //    every item wait for the count phase of all earlier ones: +0.25 ms on C3, measured)
        if (threadIdx.x == 0) sh_off = tot ? atomicAdd(a.total, tot) : 0ull;
        if (WRITE) __syncthreads();
        // 4. emit the kept decisions (LDS reads and global stores only)
        if (WRITE && cnt) {
            unsigned long long pos = sh_off;
            for (int w = 0; w < wid; w++) pos += sh_wcnt[w];
            uint2* st = stage[WRITE ? wid : 0];
            unsigned sc = 0;
#pragma unroll
            for (unsigned k = 0; k < kJCh; k++) {
                const unsigned c = (unsigned)wid + k * (kTB / kWave);
                if (c >= nch) continue;
                jemit_chunk(a, vmk[k], pidk[k], lall, nall, lpq, npart, lmask[WRITE ? wid : 0][WRITE ? k : 0], st, sc,
                            pos);
            }
            if (sc) jstage_flush(a, st, sc, pos);
        }
        __syncthreads();  // every wave leaves the item together (LDS reuse, uniform loop)
    }
#ifdef GEOHIP_JOIN_TRACE
    if (WRITE && threadIdx.x == 0 && blockIdx.x < 2048) {
        tr[blockIdx.x] = t_start;
        tr[2048 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        tr[4096 + blockIdx.x] = n_items;
        tr[6144 + blockIdx.x] = t_last;
    }
#endif
}

// ------------------------------------------------------------------ point-polygon --------
// Exact sign of x1*y2 - y1*x2 (RobustDeterminant.signOfDet2x2): error-free products by fma,
// summed as a Shewchuk expansion; the most significant nonzero component carries the sign.
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
    s = a + b;
    const double bv = s - a;
    const double av = s - bv;
    e = (a - av) + (b - bv);
}

__device__ __forceinline__ int exact_det_sign(double x1, double y1, double x2, double y2) {
    const double p = x1 * y2;
    const double ep = __builtin_fma(x1, y2, -p);
    const double q = y1 * x2;
    const double eq = __builtin_fma(y1, x2, -q);
    // grow [ep, p] by -eq, then by -q
    double h0, h1, h2, h3, Q, t;
    two_sum(-eq, ep, Q, h0);
    two_sum(Q, p, t, h1);
    Q = t;
    h2 = Q;  // expansion [h0, h1, h2]
    double g0, g1, g2;
    two_sum(-q, h0, Q, g0);
    two_sum(Q, h1, t, g1);
    Q = t;
    two_sum(Q, h2, t, g2);
    h3 = t;  // [g0, g1, g2, h3]
    if (h3 != 0) return h3 > 0 ? 1 : -1;
    if (g2 != 0) return g2 > 0 ? 1 : -1;
    if (g1 != 0) return g1 > 0 ? 1 : -1;
    if (g0 != 0) return g0 > 0 ? 1 : -1;
    return 0;
}

struct PolyDev {
    uint32_t voff, nv;      // closed ring in vx/vy
    double bb[4];           // minx, miny, maxx, maxy
    uint32_t goff, ng;      // G rects (cell space, may lie outside the grid)
    uint32_t coff, nc;      // C rects (clipped)
    int32_t wx0, wx1, wy0, wy1;  // walk region (clipped union), empty if wx0 > wx1
    uint32_t outside;       // some G rect reaches outside [0,n)^2
    uint32_t ns;            // y slabs (0: no slab lists, every segment is visited)
    double sy0, sinv;       // slab of y = clamp(floor((y - sy0) * sinv), 0, ns - 1)
    double E;               // distance lists hold every segment within E of the slab in y
    uint32_t loff, llen;    // slab block in the u16 list blob (SlabView)
    uint32_t nring;         // closed rings in the vertex run: shell first, then the holes
    uint32_t eoff;          // nring > 1: ring envelopes at renv[4 * eoff ...] (minx, miny, maxx, maxy)
    double gb[4];           // box of every ring (= bb unless a hole leaves the shell's envelope):
                            // the distance screens and slab lists are built on it
    uint32_t cls;           // per-cell classes of the walk region at pcls[cls ...] (x-major,
                            // (wy1 - wy0 + 1) per column), kNoCls: none (classify_cells)
    uint32_t pad_cls;
};

// Per-cell classes of a polygon's exact-evaluation cells, decided once on the host for every
// point a cell's exact coordinate box can hold (classify_cells): kClsHit -- every such point is
// within r of the polygon (JTS distance <= r), kClsMiss -- none is, kClsMixed -- per point.
// One u32 per cell: 2 bits per subcell of a 4 x 4 split (subcell 4 sx + sy at bits 2 (4 sx + sy));
// a cell decided as a whole repeats its class in all 16 fields.
constexpr uint8_t kClsMixed = 0, kClsHit = 1, kClsMiss = 2;
constexpr uint32_t kNoCls = 0xffffffffu;
constexpr uint32_t kWordHit = 0x55555555u, kWordMiss = 0xAAAAAAAAu;
// Subcell split of cell c of an axis: edge i (1..3) = mn + (c + i / 4) l, evaluated identically on
// host and device (no contraction); a point of the cell is in subcell #{i : v >= edge i}, so each
// subcell is an exact interval of doubles.
__host__ __device__ __forceinline__ double sub_edge(double mn, double l, int32_t c, int i) {
    return mn + ((double)c + 0.25 * (double)i) * l;
}
__host__ __device__ __forceinline__ int sub_of(double v, double mn, double l, int32_t c) {
    return (v >= sub_edge(mn, l, c, 1) ? 1 : 0) + (v >= sub_edge(mn, l, c, 2) ? 1 : 0) + (v >= sub_edge(mn, l, c, 3) ? 1 : 0);
}

// Refinement of the mixed subcells (ppoly_cand_refine): a mixed subcell is split again 4 x 4 on
// the sixteenth-cell edges sub16_edge (the subcell edges are every fourth of them, bit-identical:
// 0.0625 * 4 i == 0.25 i), each part classified by the same BoxClassifier.  Per walk-region cell
// a pair rf[2 cell] = the first of its refinement words or kNoRefine (no part of a mixed subcell
// decided), rf[2 cell + 1] = its class word; one word per MIXED subcell (2 bits per part: 4 tx +
// ty), in subcell order, so subcell s's word is rank(s) words in, rank = the mixed subcells below s
// in the class word (refine_rank).  (16 words per refined cell took 2.55 MB for C4 and its gathers
// 24 of the refinement's 63 us.)  Each such word comes with the first of its second-level words
// (one per mixed part, in part order, 2 bits per 64th-cell sub-part), or kNoRefine.
constexpr uint32_t kNoRefine = 0xffffffffu;
// mixed subcells of a class word below subcell s (fields of value kClsMixed = 0)
__host__ __device__ __forceinline__ uint32_t refine_mixed(uint32_t word) { return ~(word | (word >> 1)) & 0x55555555u; }
__host__ __device__ __forceinline__ uint32_t refine_rank(uint32_t word, int s) {
    return (uint32_t)__builtin_popcount(refine_mixed(word) & ((1u << (2 * s)) - 1u));
}
__host__ __device__ __forceinline__ double sub16_edge(double mn, double l, int32_t c, int j) {
    return mn + ((double)c + 0.0625 * (double)j) * l;
}
// part t (0..3) of subcell s of cell c: #{i in 1..3 : v >= sub16_edge(4 s + i)}
__host__ __device__ __forceinline__ int sub16_of(double v, double mn, double l, int32_t c, int s) {
    return (v >= sub16_edge(mn, l, c, 4 * s + 1) ? 1 : 0) + (v >= sub16_edge(mn, l, c, 4 * s + 2) ? 1 : 0) +
           (v >= sub16_edge(mn, l, c, 4 * s + 3) ? 1 : 0);
}
// Second level: a mixed part is split 4 x 4 again on the 64th-cell edges (every fourth is a part
// edge, bit-identical: 0.015625 * 4 j == 0.0625 j); sub-part u (0..3) of part q (0..15 along the
// axis, q = 4 s + t) of cell c: #{i in 1..3 : v >= sub64_edge(4 q + i)}
__host__ __device__ __forceinline__ double sub64_edge(double mn, double l, int32_t c, int j) {
    return mn + ((double)c + 0.015625 * (double)j) * l;
}
__host__ __device__ __forceinline__ int sub64_of(double v, double mn, double l, int32_t c, int q) {
    return (v >= sub64_edge(mn, l, c, 4 * q + 1) ? 1 : 0) + (v >= sub64_edge(mn, l, c, 4 * q + 2) ? 1 : 0) +
           (v >= sub64_edge(mn, l, c, 4 * q + 3) ? 1 : 0);
}

// Polygons with holes: rings are stored back to back in one vertex run, with a ring id per
// vertex (u16, < kMaxRings); segment (v[e], v[e+1]) exists iff both ends carry the same id (the
// junction between two rings is not an edge).  Crossing parity and boundary flags are kept per
// ring as 64-bit masks over a chunk of 64 rings (ring = 64 c + bit), so segments may still be
// visited in any order; a polygon of more than 64 rings takes one pass per chunk until a chunk
// decides (rings_locate_chunk).
constexpr uint32_t kMaxRings = 65535;
typedef uint16_t ring_id_t;

// A polygon's y-slab index (u16): cbeg[ns + 1] | dbeg[ns + 1] | segment ids.  Crossing list of
// slab s: segments (v[e], v[e+1]) whose y-range meets the slab (padded) -- every segment that
// RayCrossingCounter.countSegment can count or flag for a point whose y falls in the slab.
// Distance list: segments whose y-range widened by E meets the slab; a point whose screen
// radius is <= E cannot be within it of any other segment.  Built by plan_slabs (host).
struct SlabView {
    const uint16_t* p;
    uint32_t ns;
    __device__ __forceinline__ uint32_t cbeg(uint32_t s) const { return p[s]; }
    __device__ __forceinline__ uint32_t dbeg(uint32_t s) const { return p[ns + 1 + s]; }
    __device__ __forceinline__ uint32_t id(uint32_t k) const { return p[2 * (ns + 1) + k]; }
};

__host__ __device__ __forceinline__ uint32_t slab_of(double y, double sy0, double sinv, uint32_t ns) {
    const double f = (y - sy0) * sinv;
    if (!(f >= 0.0)) return 0;  // also NaN
    if (f >= (double)ns) return ns - 1;
    return (uint32_t)f;
}

// Screens that only ever reject (never accept) a "distance <= r" test against geometry lying
// inside a box B.  The true distance to anything in B is at least the distance to B; every JTS
// distance this library computes (fdlibm hypot, Distance.pointToSegment) is within
// 2^-50 * (|p - A|_1 + |B - A|_1) + 2^-51 d of the true one, so a margin of
// 2^-44 * (|p - bbmin|_1 + 2 * |bb extent|_1 + r) on the radius keeps every computed
// d <= r out of the rejected set.  NaN anywhere reads as "not rejected" (exact path).
__device__ __forceinline__ double screen_lim2(double px, double py, const double bb[4], double r) {
    const double m = ((__builtin_fabs(px - bb[0]) + __builtin_fabs(py - bb[1])) +
                      2.0 * ((bb[2] - bb[0]) + (bb[3] - bb[1])) + __builtin_fabs(r)) * 0x1.0p-44;
    const double lim = r + m;
    return lim * lim;
}
__device__ __forceinline__ double box_dist2(double px, double py, double x0, double y0, double x1, double y1) {
    const double ex = __builtin_fmax(__builtin_fmax(x0 - px, px - x1), 0.0);
    const double ey = __builtin_fmax(__builtin_fmax(y0 - py, py - y1), 0.0);
    return ex * ex + ey * ey;
}

// Sign of x1*y2 - y1*x2 for exact inputs: the rounded determinant decides when it clears
// the forward error bound 2^-51.4 * (|x1*y2| + |y1*x2|) (plus an absolute term for underflow);
// otherwise exact_det_sign.  Same result as RobustDeterminant.signOfDet2x2.
__device__ __forceinline__ int det_sign(double x1, double y1, double x2, double y2) {
    const double dl = x1 * y2, dr = y1 * x2;
    const double det = dl - dr;
    const double eb = 3.3306690738754716e-16 * (__builtin_fabs(dl) + __builtin_fabs(dr)) + 0x1.0p-1020;
    if (det > eb) return 1;
    if (det < -eb) return -1;
    return exact_det_sign(x1, y1, x2, y2);
}

// One segment of RayCrossingCounter.countSegment(p1, p2) for point p.
__device__ __forceinline__ void count_segment(double px, double py, double p1x, double p1y, double p2x, double p2y,
                                              bool& boundary, int& crossings) {
    const bool live = !(p1x < px && p2x < px);
    const bool at_p2 = px == p2x && py == p2y;
    const bool horiz = p1y == py && p2y == py;
    const bool on_h = horiz && px >= __builtin_fmin(p1x, p2x) && px <= __builtin_fmax(p1x, p2x);
    const bool strad = (p1y > py && p2y <= py) || (p2y > py && p1y <= py);
    if (live && !at_p2 && strad) {
        const double x1 = p1x - px, y1 = p1y - py, x2 = p2x - px, y2 = p2y - py;
        int sg = det_sign(x1, y1, x2, y2);
        boundary = boundary || sg == 0;
        if (y2 < y1) sg = -sg;
        crossings += sg > 0 ? 1 : 0;
    }
    boundary = boundary || (live && (at_p2 || on_h));
}

// Distance.pointToSegment(p, A, B) <= r, behind the box screen (lim2 = screen_lim2).
__device__ __forceinline__ bool segment_within(double px, double py, double ax, double ay, double bx, double by,
                                               double r, double lim2) {
    if (box_dist2(px, py, __builtin_fmin(ax, bx), __builtin_fmin(ay, by), __builtin_fmax(ax, bx),
                  __builtin_fmax(ay, by)) > lim2)
        return false;
    // Certified screens without division or square root.  D = true distance from p to the
    // segment; the JTS value d is within dJ = 2^-50 (|p-A|_1 + |B-A|_1) + 2^-51 D of it (see
    // screen_lim2), so D < r - dl decides "d <= r" and D > r + dl decides "d > r", dl >= 4 dJ.
    // Bounds on D: <= |p-A|, |p-B|; = the line distance |cross| / |B-A| when the projection is
    // certainly interior; >= the line distance always.  Every product below is of terms <= M
    // (M = |p-A|_1 + |B-A|_1), so each computed quantity is within 2^-50 M^2 of its value: E =
    // 2^-45 M^2 covers it, and the (1 -/+ 2^-45) factors cover the roundings of the squared
    // bounds.  NaN or an infinity anywhere fails every decision (the exact path runs).
    {
        const double dax = px - ax, day = py - ay, dbx = px - bx, dby = py - by;
        const double ex = bx - ax, ey = by - ay;
        const double M = __builtin_fabs(dax) + __builtin_fabs(day) + __builtin_fabs(ex) + __builtin_fabs(ey);
        const double E = M * M * 0x1.0p-45;
        const double dl = M * 0x1.0p-48 + __builtin_fabs(r) * 0x1.0p-49;
        const double rl = r - dl, rh = r + dl;
        const double rl2 = rl * rl * (1.0 - 0x1.0p-45), rh2 = rh * rh * (1.0 + 0x1.0p-45);
        const double da2 = dax * dax + day * day, db2 = dbx * dbx + dby * dby;
        const double len2 = ex * ex + ey * ey;
        const double dot = dax * ex + day * ey;
        const double crs = __builtin_fabs(day * ex - dax * ey);
        const bool interior = dot - E > 0.0 && dot + E < len2 - E;
        if (rl > 0.0) {
            if (da2 + E < rl2 || db2 + E < rl2) return true;  // an endpoint is closer than r
            if (interior && (crs + E) * (crs + E) < rl2 * (len2 - E) * (1.0 - 0x1.0p-50)) return true;
        }
        if (crs > E && (crs - E) * (crs - E) > rh2 * (len2 + E) * (1.0 + 0x1.0p-50)) return false;  // line
        if (dot + E < 0.0 && da2 - E > rh2) return false;        // nearest point A
        if (dot - E > len2 + E && db2 - E > rh2) return false;   // nearest point B
    }
    double d;
    if (ax == bx && ay == by) {
        d = coord_distance(px, py, ax, ay);
    } else {
        const double len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay);
        const double rr = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2;
        if (rr <= 0.0) d = coord_distance(px, py, ax, ay);
        else if (rr >= 1.0) d = coord_distance(px, py, bx, by);
        else {
            const double s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2;
            d = __builtin_fabs(s) * __builtin_sqrt(len2);
        }
    }
    return d <= r;
}

// fp32 segment boxes for the distance pre-screen: box of segment (v[e], v[e+1]) relative to
// the polygon's origin o = (gb[0], gb[1]), each coordinate rounded to fp32 once (error <=
// 2^-24 |c - o| + 2^-53 |c - o|: IEEE subtraction and conversion are each within half an ulp of
// their result).  The last vertex has no segment: an all-NaN box, which never rejects.
__device__ __forceinline__ float4 seg_box32(const double* __restrict__ vx, const double* __restrict__ vy, uint32_t e,
                                            uint32_t nv, double ox, double oy) {
    if (e + 1 >= nv) return make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
    const double ax = vx[e], ay = vy[e], bx = vx[e + 1], by = vy[e + 1];
    return make_float4((float)(__builtin_fmin(ax, bx) - ox), (float)(__builtin_fmin(ay, by) - oy),
                       (float)(__builtin_fmax(ax, bx) - ox), (float)(__builtin_fmax(ay, by) - oy));
}
// The point's side of that screen.  u = p - o and every box coordinate carry at most ~2^-23.9 of
// their magnitude, the fp32 subtractions 2^-24 of theirs, so the fp32 box distance is within
// S = 2^-18 (|u| + |v| + ext) (+ an absolute term for fp32 underflow) of the true box distance,
// ext = the polygon box's half-perimeter >= every |box coordinate|.  Rejected: fp32 distance^2 >
// (lim + S)^2 (1 + 2^-19) -- the squares' own fp32 rounding (<= 2^-22) is inside that factor.
// NaN anywhere never rejects (fmaxf drops one NaN operand, a NaN bound compares false).
struct Fp32Screen {
    float u, v, lim2;
    __device__ __forceinline__ bool rejects(const float4 b) const {
        const float ex = __builtin_fmaxf(__builtin_fmaxf(b.x - u, u - b.z), 0.0f);
        const float ey = __builtin_fmaxf(__builtin_fmaxf(b.y - v, v - b.w), 0.0f);
        return ex * ex + ey * ey > lim2;
    }
};
__device__ __forceinline__ Fp32Screen fp32_screen(double px, double py, const double gb[4], double lim2) {
    const double u = px - gb[0], v = py - gb[1];
    const double ext = (gb[2] - gb[0]) + (gb[3] - gb[1]);
    const double S = (__builtin_fabs(u) + __builtin_fabs(v) + ext) * 0x1.0p-18 + 0x1.0p-100;
    const double ls = __builtin_sqrt(lim2) * (1.0 + 0x1.0p-40) + S;
    return Fp32Screen{(float)u, (float)v, (float)(ls * ls * (1.0 + 0x1.0p-19))};
}

// JTS DistanceOp(point, polygon) predicate "distance <= r" (r < MAX_VALUE):
// PointLocator (envelope, RayCrossingCounter over the ring) -> 0 when not EXTERIOR; else the
// min over segments of Distance.pointToSegment.  A boundary hit anywhere makes the answer true
// whatever the other segments count, so segments are visited in any order and only those of
// the point's slab lists; boolean-equivalent early exit on the first segment within r.
__device__ __forceinline__ bool point_polygon_within(double px, double py, const double* __restrict__ vx,
                                     const double* __restrict__ vy, const PolyDev& P, const SlabView& sv, double r,
                                     const float4* __restrict__ sb = nullptr) {
    const int nv = (int)P.nv;
    const bool in_env = !(px > P.bb[2] || px < P.bb[0] || py > P.bb[3] || py < P.bb[1]);
    const uint32_t s = sv.ns ? slab_of(py, P.sy0, P.sinv, sv.ns) : 0u;
    if (in_env) {
        bool boundary = false;
        int crossings = 0;
        if (sv.ns) {
            // two segments per step: both ids, then all eight coordinates, in flight together
            // (crossing counts add and boundary flags OR: order-independent)
            const uint32_t k1 = sv.cbeg(s + 1);
            uint32_t k = sv.cbeg(s);
            for (; k + 2 <= k1; k += 2) {
                const uint32_t e0 = sv.id(k), e1 = sv.id(k + 1);
                const double p0x = vx[e0 + 1], p0y = vy[e0 + 1], q0x = vx[e0], q0y = vy[e0];
                const double p1x = vx[e1 + 1], p1y = vy[e1 + 1], q1x = vx[e1], q1y = vy[e1];
                count_segment(px, py, p0x, p0y, q0x, q0y, boundary, crossings);
                count_segment(px, py, p1x, p1y, q1x, q1y, boundary, crossings);
            }
            if (k < k1) {
                const uint32_t e = sv.id(k);
                count_segment(px, py, vx[e + 1], vy[e + 1], vx[e], vy[e], boundary, crossings);
            }
        } else {
            for (int i = 1; i < nv; i++) count_segment(px, py, vx[i], vy[i], vx[i - 1], vy[i - 1], boundary, crossings);
        }
        if (boundary || (crossings & 1)) return true;  // distance 0
    }
    const double lim2 = screen_lim2(px, py, P.gb, r);
    if (sv.ns && lim2 <= P.E * P.E) {
        const uint32_t k1 = sv.dbeg(s + 1);
        uint32_t k = sv.dbeg(s);
        if (sb) {
            // fp32 pre-screen (sb: segment boxes relative to (gb[0], gb[1]), see seg_box32): the
            // box distance of the fp32 point and box is within S of the true box distance, so
            // "fp32 box distance > lim + S" rejects only segments the fp64 screen rejects too;
            // the survivors (usually none or one per point) take the fp64 path unchanged
            const float4* __restrict__ sbb = sb;
            const Fp32Screen f = fp32_screen(px, py, P.gb, lim2);
            for (; k + 2 <= k1; k += 2) {
                const uint32_t e0 = sv.id(k), e1 = sv.id(k + 1);
                const bool r0 = f.rejects(sbb[e0]), r1 = f.rejects(sbb[e1]);
                if (!r0 && segment_within(px, py, vx[e0], vy[e0], vx[e0 + 1], vy[e0 + 1], r, lim2)) return true;
                if (!r1 && segment_within(px, py, vx[e1], vy[e1], vx[e1 + 1], vy[e1 + 1], r, lim2)) return true;
            }
            if (k < k1) {
                const uint32_t e = sv.id(k);
                if (!f.rejects(sbb[e]) && segment_within(px, py, vx[e], vy[e], vx[e + 1], vy[e + 1], r, lim2))
                    return true;
            }
            return false;
        }
        for (; k + 2 <= k1; k += 2) {  // "any segment within r": pairs, same answer
            const uint32_t e0 = sv.id(k), e1 = sv.id(k + 1);
            const double a0x = vx[e0], a0y = vy[e0], b0x = vx[e0 + 1], b0y = vy[e0 + 1];
            const double a1x = vx[e1], a1y = vy[e1], b1x = vx[e1 + 1], b1y = vy[e1 + 1];
            if (segment_within(px, py, a0x, a0y, b0x, b0y, r, lim2) ||
                segment_within(px, py, a1x, a1y, b1x, b1y, r, lim2))
                return true;
        }
        if (k < k1) {
            const uint32_t e = sv.id(k);
            if (segment_within(px, py, vx[e], vy[e], vx[e + 1], vy[e + 1], r, lim2)) return true;
        }
        return false;
    }
    for (int i = 0; i < nv - 1; i++)
        if (segment_within(px, py, vx[i], vy[i], vx[i + 1], vy[i + 1], r, lim2)) return true;
    return false;
}

// PointLocator.locateInPolygon (JTS 1.16.1) from per-ring masks of the rings [64 c, 64 c + 64):
// bit j of bnd = some segment of ring 64 c + j flags the point as on it, bit j of par = odd
// crossing count of that ring.  Chunk 0 holds the shell (bit 0): shell boundary -> on the polygon;
// even shell parity -> outside.  Then the holes in order: a hole whose envelope excludes the point
// is EXTERIOR to it (locateInPolygonRing's envelope test), boundary -> on the polygon, interior ->
// outside.  Returns 1 (distance 0), 0 (outside), or -1: no ring of the chunk decides (the next
// chunk's holes go on; after the last chunk the point is inside).
__device__ __forceinline__ int rings_locate_chunk(double px, double py, unsigned long long bnd, unsigned long long par,
                                                  const double* __restrict__ renv, uint32_t c) {
    unsigned long long m = bnd | par;
    if (c == 0) {
        if (bnd & 1ull) return 1;
        if (!(par & 1ull)) return 0;
        m &= ~1ull;
    }
    while (m) {
        const int h = __builtin_ctzll(m);
        m &= m - 1;
        const double* e = renv + 4 * (64 * (size_t)c + h);
        if (px > e[2] || px < e[0] || py > e[3] || py < e[1]) continue;
        return ((bnd >> h) & 1ull) ? 1 : 0;  // on hole h / inside hole h
    }
    return -1;
}

// point_polygon_within for a polygon with holes (P.nring > 1): the same crossing and distance
// lists (plan_slabs leaves the ring junctions out of them), crossings kept per ring.  Distance:
// any segment of any ring within r (DistanceOp's per-ring envelope skip only drops rings whose
// envelope is farther than the running minimum, which never holds a segment within r of p
// except through a rounding tie between the envelope and segment distances).
__device__ __forceinline__ bool point_polygon_within_rings(double px, double py, const double* __restrict__ vx,
                                                        const double* __restrict__ vy,
                                                        const ring_id_t* __restrict__ vr,
                                                        const double* __restrict__ renv, const PolyDev& P,
                                                        const SlabView& sv, double r) {
    const int nv = (int)P.nv;
    const bool in_env = !(px > P.bb[2] || px < P.bb[0] || py > P.bb[3] || py < P.bb[1]);
    const uint32_t s = sv.ns ? slab_of(py, P.sy0, P.sinv, sv.ns) : 0u;
    if (in_env) {
        const uint32_t nch = (P.nring + 63) / 64;
        int loc = -1;
        for (uint32_t c = 0; c < nch && loc < 0; c++) {
            unsigned long long bnd = 0, par = 0;
            auto seg = [&](uint32_t e) {
                const uint32_t rid = vr[e];
                if ((rid >> 6) != c) return;
                bool b = false;
                int cr = 0;
                count_segment(px, py, vx[e + 1], vy[e + 1], vx[e], vy[e], b, cr);
                const unsigned long long bit = 1ull << (rid & 63);
                bnd |= b ? bit : 0ull;
                par ^= (cr & 1) ? bit : 0ull;
            };
            if (sv.ns) {
                for (uint32_t k = sv.cbeg(s); k < sv.cbeg(s + 1); k++) seg(sv.id(k));
            } else {
                for (int e = 0; e < nv - 1; e++)
                    if (vr[e] == vr[e + 1]) seg((uint32_t)e);
            }
            loc = rings_locate_chunk(px, py, bnd, par, renv, c);
        }
        if (loc != 0) return true;  // on a ring, or inside with no hole claiming the point
    }
    const double lim2 = screen_lim2(px, py, P.gb, r);
    if (sv.ns && lim2 <= P.E * P.E) {
        for (uint32_t k = sv.dbeg(s); k < sv.dbeg(s + 1); k++) {
            const uint32_t e = sv.id(k);
            if (segment_within(px, py, vx[e], vy[e], vx[e + 1], vy[e + 1], r, lim2)) return true;
        }
        return false;
    }
    for (int e = 0; e < nv - 1; e++)
        if (vr[e] == vr[e + 1] && segment_within(px, py, vx[e], vy[e], vx[e + 1], vy[e + 1], r, lim2)) return true;
    return false;
}

// DistanceFunctions.getPointPolygonBBoxMinEuclideanDistance (DistanceFunctions.java:150-200)
__device__ __forceinline__ double pp_euclid(double lon, double lat, double lon1, double lat1) {
    const double dy = lat1 - lat, dx = lon1 - lon;
    return __builtin_sqrt(dy * dy + dx * dx);
}
__device__ __forceinline__ double bbox_border(double x, double y, double x1, double y1, double x2, double y2) {
    if (x1 == x2) return pp_euclid(x, y, x1, y);
    if (y1 == y2) return pp_euclid(x, y, x, y1);
    return 4.9406564584124654e-324;
}
__device__ __forceinline__ double bbox_distance(double x, double y, const double bb[4]) {
    const double x1 = bb[0], y1 = bb[1], x2 = bb[2], y2 = bb[3];
    if (x <= x1) {
        if (y <= y1) return pp_euclid(x, y, x1, y1);
        if (y >= y2) return pp_euclid(x, y, x1, y2);
        return bbox_border(x, y, x1, y1, x1, y2);
    } else if (x >= x2) {
        if (y <= y1) return pp_euclid(x, y, x2, y1);
        if (y >= y2) return pp_euclid(x, y, x2, y2);
        return bbox_border(x, y, x2, y1, x2, y2);
    }
    if (y <= y1) return bbox_border(x, y, x1, y1, x2, y1);
    if (y >= y2) return bbox_border(x, y, x1, y2, x2, y2);
    return 0.0;
}

__device__ __forceinline__ bool in_rects(const int32_t* __restrict__ rr, uint32_t n, int32_t cx, int32_t cy) {
    for (uint32_t i = 0; i < n; i++)
        if (cx >= rr[4 * i] && cx <= rr[4 * i + 1] && cy >= rr[4 * i + 2] && cy <= rr[4 * i + 3]) return true;
    return false;
}

constexpr int kMaxLdsVerts = 512;   // larger rings are read from global memory
constexpr int kMaxLdsSlab = 2048;   // u16 slab-list entries staged in LDS
constexpr int kMaskWords = 512;     // hit-mask words kept in LDS (tiles up to 32768 points)
constexpr int kCandQ = 128;         // per-wave queue of points needing the exact polygon distance
constexpr int kPolyPairs = 512;     // per-wave pair buffer of the polygon kernels
constexpr int kTileCls = 1024;      // tile cells whose classes ppoly_eval stages (ts <= 32)

struct PolyWork {
    uint32_t poly, tile;  // tile | kWorkAllHit: every point of the tile is a hit (no point is read)
};
constexpr uint32_t kWorkAllHit = 0x80000000u;

struct CandQueue {
    double x[kCandQ];
    double y[kCandQ];
    unsigned pos[kCandQ];
};

// hit-mask words of each work item: ceil(points of its tile / 64)
__global__ void ppoly_words(const PolyWork* __restrict__ work, uint32_t nwork, const unsigned* __restrict__ tstart,
                            unsigned long long* __restrict__ words) {
    const uint32_t w = blockIdx.x * kTB + threadIdx.x;
    if (w >= nwork) return;
    const uint32_t t = work[w].tile & ~kWorkAllHit;
    words[w] = (tstart[t + 1] - tstart[t] + 63) / 64;
}

// Count pass, one workgroup per (polygon, tile): ring and slab lists in LDS; every wave
// classifies 64 of the tile's points per pass (G -> hit; C -> approximate bbox distance, or
// the envelope screen then a per-wave queue) and evaluates the exact JTS distance on full
// waves of queued points.  Hits become a bitmask over the tile's points (word k = points
// [64k, 64k + 64) of the tile) and a per-work-item count; the write pass (ppoly_emit) only
// reads the mask.
// Emit (polygon, p) iff key(p) in G, or key(p) in C and d <= r (PointPolygonRangeQuery.java:105-121).
template <bool APPROX>
__global__ __launch_bounds__(kTB) void ppoly_eval(TileBins tb, const PolyWork* __restrict__ work,
                                                  const PolyDev* __restrict__ polys, const double* __restrict__ vx,
                                                  const double* __restrict__ vy, const ring_id_t* __restrict__ vring,
                                                  const double* __restrict__ renv, const int32_t* __restrict__ rects,
                                                  const uint16_t* __restrict__ slabs, const uint32_t* __restrict__ pcls,
                                                  double r, int r_is_max, const unsigned long long* __restrict__ wofs,
                                                  unsigned long long* __restrict__ mask,
                                                  unsigned long long* __restrict__ bcount) {
    __shared__ uint32_t lcls[kTileCls];  // the cell class words of this tile (P.cls)
    __shared__ double lvx[kMaxLdsVerts];
    __shared__ double lvy[kMaxLdsVerts];
    __shared__ ring_id_t lvr[kMaxLdsVerts];
    __shared__ float4 lsb[kMaxLdsVerts];  // fp32 segment boxes (single-ring polygons staged in LDS)
    __shared__ uint16_t lsl[kMaxLdsSlab];
    __shared__ unsigned long long lmask[kMaskWords];
    __shared__ CandQueue cq[kTB / kWave];
    __shared__ unsigned long long bsh;
    const PolyWork w = work[blockIdx.x];
    const PolyDev P = polys[w.poly];
    const uint32_t tile = w.tile & ~kWorkAllHit;
    const bool all_hit = (w.tile & kWorkAllHit) != 0;
    const unsigned ds = tb.start[tile], de = tb.start[tile + 1];
    const unsigned nwords = (de - ds + 63) / 64;
    const bool lds_mask = nwords <= (unsigned)kMaskWords;
    unsigned long long* gm = mask + wofs[blockIdx.x];
    const bool v_lds = P.nv <= (uint32_t)kMaxLdsVerts;
    const bool s_lds = P.llen <= (uint32_t)kMaxLdsSlab;
    const bool holes = P.nring > 1;
    if (v_lds)
        for (uint32_t t = threadIdx.x; t < P.nv; t += kTB) {
            lvx[t] = vx[P.voff + t];
            lvy[t] = vy[P.voff + t];
            if (holes) lvr[t] = vring[P.voff + t];
            else if (!APPROX) lsb[t] = seg_box32(vx + P.voff, vy + P.voff, t, P.nv, P.gb[0], P.gb[1]);
        }
    if (s_lds)
        for (uint32_t t = threadIdx.x; t < P.llen; t += kTB) lsl[t] = slabs[P.loff + t];
    if (lds_mask)
        for (uint32_t t = threadIdx.x; t < nwords; t += kTB) lmask[t] = 0;
    if (threadIdx.x == 0) bsh = 0;
    const int32_t ts = tb.ts;
    const int32_t tx0 = (int32_t)(tile / (uint32_t)tb.nt) * ts, ty0 = (int32_t)(tile % (uint32_t)tb.nt) * ts;
    const bool use_cls = !APPROX && !all_hit && P.cls != kNoCls && ts * ts <= kTileCls;
    if (use_cls) {
        const int32_t ch = P.wy1 - P.wy0 + 1;
        for (int32_t t = threadIdx.x; t < ts * ts; t += kTB) {
            const int32_t cx = tx0 + t / ts, cy = ty0 + t % ts;
            lcls[t] = (cx >= P.wx0 && cx <= P.wx1 && cy >= P.wy0 && cy <= P.wy1)
                          ? pcls[P.cls + (uint32_t)((cx - P.wx0) * ch + (cy - P.wy0))]
                          : 0u;
        }
    }
    __syncthreads();
    const double* rvx = v_lds ? lvx : vx + P.voff;
    const double* rvy = v_lds ? lvy : vy + P.voff;
    const ring_id_t* rvr = v_lds ? lvr : vring + P.voff;
    const double* rre = renv + 4 * (size_t)P.eoff;
    const SlabView sv{s_lds ? lsl : slabs + P.loff, P.ns};
    unsigned long long* mk = lds_mask ? lmask : gm;  // global words: zeroed by the host, atomics only
    const int wid = threadIdx.x / kWave, lane = lane_id();
    CandQueue& Q = cq[wid];
    unsigned qn = 0;
    const unsigned nb = (unsigned)tb.nb;
    const int32_t* grect = rects + 4 * P.goff;
    const int32_t* crect = rects + 4 * P.coff;
    auto drain = [&](unsigned take) {  // evaluate the top `take` queued points (wave-uniform)
        const unsigned from = qn - take;
        if ((unsigned)lane < take) {
            const double px = Q.x[from + lane], py = Q.y[from + lane];
            const unsigned pos = Q.pos[from + lane];
            const bool in = holes ? point_polygon_within_rings(px, py, rvx, rvy, rvr, rre, P, sv, r)
                                  : point_polygon_within(px, py, rvx, rvy, P, sv, r, v_lds ? lsb : nullptr);
            if (in) atomicOr(&mk[pos >> 6], 1ull << (pos & 63));
        }
        wave_lds_sync();
        qn = from;
    };
    // the first G and C rectangle in registers (one each unless the plan is unusual)
    int32_t g0[4] = {1, 0, 1, 0}, c0[4] = {1, 0, 1, 0};
    if (P.ng) for (int t = 0; t < 4; t++) g0[t] = grect[t];
    if (P.nc) for (int t = 0; t < 4; t++) c0[t] = crect[t];
    auto in_r = [](const int32_t (&q)[4], int32_t x, int32_t y) { return x >= q[0] && x <= q[1] && y >= q[2] && y <= q[3]; };
    // key and coordinates of the next pass are loaded while the current one is classified
    unsigned key_n = 0;
    double px_n = 0.0, py_n = 0.0;
    auto fetch = [&](unsigned base) {
        const unsigned i = base + lane;
        if (i < de) {
            key_n = tb.skey[i];
            px_n = tb.sx[i];
            py_n = tb.sy[i];
        }
    };
    if (all_hit) {
        // every cell of the tile is guaranteed or a whole-cell hit (the plan checked cell 0
        // rows/columns are guaranteed, so NaN points there are hits too): whole mask words
        for (uint32_t t = threadIdx.x; t < nwords; t += kTB) {
            const unsigned left = de - ds - 64 * t;
            const unsigned long long v = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
            if (lds_mask) lmask[t] = v;
            else gm[t] = v;
        }
    }
    if (!all_hit && ds + wid * kWave < de) fetch(ds + wid * kWave);
    for (unsigned base = ds + wid * kWave; !all_hit && base < de; base += kTB) {
        const unsigned i = base + lane;
        const unsigned key = key_n;
        const double px = px_n, py = py_n;
        if (base + kTB < de) fetch(base + kTB);
        bool hit = false, need = false;
        if (i < de) {
            const int32_t cx = (int32_t)tb.dnb.div(key), cy = (int32_t)(key - (unsigned)cx * nb);
            bool g = in_r(g0, cx, cy);
            if (P.ng > 1 && !g) g = in_rects(grect + 4, P.ng - 1, cx, cy);
            bool c = !g && in_r(c0, cx, cy);
            if (P.nc > 1 && !g && !c) c = in_rects(crect + 4, P.nc - 1, cx, cy);
            if (g || c) {
                // a decided cell class applies to every point in the cell's coordinate box: not
                // to NaN coordinates (cell 0 by Java's (int) NaN)
                uint32_t k = kClsMixed;
                if (use_cls && !g && px == px && py == py) {
                    const uint32_t wd = lcls[(cx - tx0) * ts + (cy - ty0)];
                    if (wd == kWordHit) k = kClsHit;
                    else if (wd == kWordMiss) k = kClsMiss;
                    else if (wd != 0u) {
                        const int sx = sub_of(px, tb.mnx, tb.l, cx), sy = sub_of(py, tb.mny, tb.l, cy);
                        k = (wd >> (2 * (4 * sx + sy))) & 3u;
                    }
                }
                if (g || r_is_max || k == kClsHit) hit = true;
                else if (APPROX) hit = bbox_distance(px, py, P.bb) <= r;
                else if (k != kClsMiss)
                    need = !(box_dist2(px, py, P.gb[0], P.gb[1], P.gb[2], P.gb[3]) > screen_lim2(px, py, P.gb, r));
            }
        }
        const unsigned long long m = __ballot(hit);
        if (m && lane == 0) atomicOr(&mk[(base - ds) >> 6], m);
        if (!APPROX) {
            const unsigned long long mq = __ballot(need);
            if (need) {
                const unsigned slot = qn + lanes_below(mq);
                Q.x[slot] = px;
                Q.y[slot] = py;
                Q.pos[slot] = i - ds;
            }
            qn += (unsigned)__popcll(mq);
            wave_lds_sync();
            if (qn >= (unsigned)kWave) drain(kWave);
        }
    }
    if (!APPROX && qn) drain(qn);
    __syncthreads();
    if (!lds_mask) __threadfence();
    __syncthreads();
    unsigned long long c = 0;
    for (uint32_t t = threadIdx.x; t < nwords; t += kTB) {
        unsigned long long v;
        if (lds_mask) {
            v = lmask[t];
            gm[t] = v;
        } else {
            v = __hip_atomic_load(&gm[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        c += (unsigned long long)__popcll(v);
    }
    if (c) atomicAdd(&bsh, c);
    __syncthreads();
    if (threadIdx.x == 0) bcount[blockIdx.x] = bsh;
}

// Write pass: pairs (polygon, point) of every set bit of the work item's hit mask.
__global__ __launch_bounds__(kTB) void ppoly_emit(TileBins tb, const PolyWork* __restrict__ work,
                                                  const unsigned long long* __restrict__ wofs,
                                                  const unsigned long long* __restrict__ mask, PairSink sink) {
    __shared__ uint2 pbuf[kTB / kWave][kPolyPairs];
    __shared__ unsigned long long bsh;
    const PolyWork w = work[blockIdx.x];
    const uint32_t tile = w.tile & ~kWorkAllHit;
    const unsigned ds = tb.start[tile], de = tb.start[tile + 1];
    const unsigned nwords = (de - ds + 63) / 64;
    const unsigned long long* gm = mask + wofs[blockIdx.x];
    if (threadIdx.x == 0) bsh = 0;
    __syncthreads();
    const int wid = threadIdx.x / kWave, lane = lane_id();
    uint2* buf = pbuf[wid];
    unsigned long long cnt = 0;
    for (unsigned k = wid; k < nwords; k += kTB / kWave) {
        const unsigned long long word = gm[k];
        if (word == 0) continue;
        const bool hit = (word >> lane) & 1ull;
        const unsigned pid = hit ? tb.sidx[ds + k * 64 + lane] : 0u;
        pairs_push<true, kPolyPairs>(buf, cnt, hit, w.poly, pid, &bsh, sink);
    }
    pairs_end<true>(buf, cnt, &bsh, sink);
}

// out-of-grid points vs guaranteed rects reaching outside the grid (Lg == 0 bbox keys).
// DIST (point-polygon join, exact): the polygon's rect list is (coff, nc) and a matching point
// also needs the JTS distance <= r (the join has no guaranteed-cell shortcut).
template <bool WRITE, bool DIST = false>
__global__ __launch_bounds__(kTB) void ppoly_outside(const double* __restrict__ x, const double* __restrict__ y,
                                                     const unsigned* __restrict__ oidx, unsigned nout, double mnx,
                                                     double mny, double l, const PolyDev* __restrict__ polys,
                                                     uint32_t npoly, const int32_t* __restrict__ rects, PairSink sink,
                                                     const double* __restrict__ vx = nullptr,
                                                     const double* __restrict__ vy = nullptr,
                                                     const uint16_t* __restrict__ slabs = nullptr, double r = 0.0,
                                                     const ring_id_t* __restrict__ vring = nullptr,
                                                     const double* __restrict__ renv = nullptr) {
    __shared__ uint2 pbuf[WRITE ? kTB / kWave : 1][WRITE ? kPolyPairs : 1];
    __shared__ unsigned long long bsh;
    const int wid = threadIdx.x / kWave;
    uint2* buf = pbuf[WRITE ? wid : 0];
    unsigned long long cnt = 0;
    if (threadIdx.x == 0) bsh = 0;
    __syncthreads();
    for (uint32_t p = blockIdx.x; p < npoly; p += gridDim.x) {
        const PolyDev P = polys[p];
        if (!P.outside) continue;
        for (unsigned t0 = wid * kWave; t0 < nout; t0 += kTB) {
            const unsigned t = t0 + lane_id();
            bool hit = false;
            unsigned pid = 0;
            if (t < nout) {
                pid = oidx[t];
                const double px = x[pid], py = y[pid];
                const int32_t cx = d_axis_cell(px, mnx, l), cy = d_axis_cell(py, mny, l);
                hit = DIST ? in_rects(rects + 4 * P.coff, P.nc, cx, cy) : in_rects(rects + 4 * P.goff, P.ng, cx, cy);
                if (DIST && hit) {
                    const SlabView sv{slabs + P.loff, P.ns};
                    hit = P.nring > 1 ? point_polygon_within_rings(px, py, vx + P.voff, vy + P.voff, vring + P.voff,
                                                                   renv + 4 * (size_t)P.eoff, P, sv, r)
                                      : point_polygon_within(px, py, vx + P.voff, vy + P.voff, P, sv, r);
                }
            }
            pairs_push<WRITE, kPolyPairs>(buf, cnt, hit, p, pid, &bsh, sink);
        }
    }
    pairs_end<WRITE>(buf, cnt, &bsh, sink);
}

// ====================================================== point-polygon: streaming path =======
// The window is read once, in arrival order, with no tile binning.  A host-built cell table
// (PolyCache::cell_off / cell_ent, cached with the polygon plan) lists per key cell the
// polygons whose rectangles hold it, C cells of class kClsMiss left out: entry (poly | kEntC?,
// class word).  Per point, its cell's entries: a G entry (or, exact, a C entry whose subcell
// class is kClsHit; approximate, a C entry whose bbox distance is <= r) is a pair at once; a C
// entry of a mixed subcell is a candidate (point, polygon) for the exact JTS test.  Candidates
// (a few % of the points for C4) are grouped by polygon (ppoly_cand_count / _plan / _scatter)
// and evaluated with the polygon's rings in LDS (ppoly_cand_eval), as ppoly_eval does per tile.
// Pairs and candidates leave through per-wave LDS buffers, one global atomic per buffer.
// The same decisions as ppoly_eval (PointPolygonRangeQuery.java:105-121; the join's
// PointPolygonJoinQuery.java:183-195 through jmode's rectangle lists).
constexpr uint32_t kEntC = 0x80000000u;    // entry.x: C cell (class word in entry.y); else G
constexpr unsigned kCandGone = 0xffffffffu;  // a candidate slot decided by the refinement, left to the
                                             // redo pass, or past a range's end: the grouping skips it
constexpr int kStreamNW = 8;               // waves per block
constexpr unsigned kStreamPts = 256;       // points per wave iteration (4 per lane)
// 4096-point chunks: 2 iterations per wave (8192 spilled 33 VGPRs in the two-phase chunk; 2048
// measured 626-629 against 591-594 us of C4 kernels, round 5)
constexpr unsigned kLocalBits = 12;  // point within its chunk
constexpr unsigned kStreamChunk = 1u << kLocalBits;  // points per chunk
constexpr unsigned kStreamBlocksPerCU = 2;  // resident blocks per CU (LDS, registers)
constexpr unsigned kSPairCap = 2 * kStreamChunk;  // block-staged pairs per chunk (4 B each: poly << 12 | point),
                                                  // kSPairCap / kStreamNW per wave
constexpr unsigned kSCandCap = kStreamChunk / 4;  // block-staged candidates per chunk (per wave likewise)
constexpr uint32_t kStreamMaxPolys = 1u << (32 - kLocalBits);
// candidates per evaluation work item (512 / 256 measured slower: 640 / 652 against 622 us of
// C4 kernels, round 5)
constexpr unsigned kCandItem = 1024;
constexpr unsigned kCandLdsPolys = 16384;  // polygons whose per-polygon counters fit LDS
constexpr unsigned kEvalBlocks = 1024;     // grid of the evaluation pass (strides over its items)
static_assert(kStreamChunk == (1u << kLocalBits), "chunk-local point ids");
static_assert(kStreamChunk % (kStreamNW * kStreamPts) == 0, "chunk = waves x iterations x points");

// A cell's table head (8 B, one gather per point): x == kNoEntry -- no entry; x & kMulti -- x's
// low 30 bits entries at cell_ent[y ...]; else the cell's only entry (x = poly | kEntC?, y = its
// class word).  2 MB for 500 x 500 cells.
constexpr uint32_t kNoEntry = 0xffffffffu;
constexpr uint32_t kMulti = 0x40000000u;

struct StreamOut {
    unsigned* out;                  // pairs, u32 x 2 (swap: (point, polygon))
    uint64_t cap;
    int aligned8, swap;
    unsigned point_base;            // added to every point index of a pair (pane stream positions)
    unsigned long long* ptotal;     // pairs: reservation cursor (zero before; an async call's count)
    unsigned long long* ctotal;     // candidates: reservation cursor (zero before)
    unsigned* flushes;              // wave stages flushed before their chunk's end (profiling count)
    uint64_t ccap;                  // candidate buffer: a chunk whose candidates pass it goes to the redo pass
    unsigned* cpoly;                // candidates in chunk order: polygon (the grouping reads these),
    double4* crec;                  // and (x, y, point bits, -) -- one 32-byte sector per gather
    unsigned* covf;                 // per wave: the chunk's candidates staged before its end (packed
    unsigned covf_wave;             // words), covf_wave each -- a chunk's worth at most
    unsigned* redo;                 // chunks whose candidates did not fit the buffer (ppoly_stream_redo)
    unsigned* nredo;                // their count (zero before)
};

struct StreamArgs {
    const double* x;
    const double* y;
    uint64_t n;
    TileGeom g;
    const unsigned* keep;           // cells with entries (bitmap, keep_words words)
    unsigned keep_words;
    const uint2* head;              // nb * nb
    const uint2* ent;
    const PolyDev* polys;
    const uint32_t* opoly;          // polygons whose rectangles reach outside the grid
    uint32_t nopoly;
    const int32_t* rects;
    int jmode;                      // 0 range, 1 join exact, 2 join approximate
    double r;
    StreamOut o;
    // the rings, for the redo pass's candidates (decided there as ppoly_cand_eval decides the
    // others)
    const double* vx;
    const double* vy;
    const ring_id_t* vring;
    const double* renv;
    const uint16_t* slabs;
};

// Pairs and candidates of the current chunk are staged in LDS (4 B each: poly << kLocalBits |
// chunk-local point): each wave owns a region of the block's stage and counts its entries in a
// wave-uniform register -- no LDS atomic per push.  The block reserves the waves' entries with one
// atomic per kind at the chunk's end; a wave whose region fills before that (cells of many
// polygons) flushes it with its own reservation and goes on -- no chunk is ever run twice (the
// round-5 form re-ran an overflowing chunk with direct stores: every chunk of a window of 3000
// overlapping polygons re-ran).
struct StreamSink {
    unsigned* pk;                   // this wave's LDS region
    unsigned cap;                   // its capacity (a push adds <= 64)
    unsigned n;                     // entries staged (wave-uniform)
    unsigned ovn;                   // candidates: this chunk's entries in the wave's overflow list
                                    // (kOvnLost: the list filled, the chunk goes to the redo pass)
};
constexpr unsigned kOvnLost = 0xffffffffu;
constexpr uint32_t kSpillEnt = 16;  // spill-list entries per chunk point (a window of cells with more
                                    // polygons than that may send chunks to the redo pass)

__device__ __forceinline__ void stream_emit_pair(const StreamOut& o, unsigned long long p, unsigned poly, unsigned idx) {
    if (p >= o.cap) return;
    idx += o.point_base;
    const uint2 v = o.swap ? make_uint2(idx, poly) : make_uint2(poly, idx);
    if (o.aligned8) {  // one 8-byte store per pair (plain, as the join's: nontemporal 617 against 613 us
                       // of C4 kernels, same box)
        reinterpret_cast<unsigned long long*>(o.out)[p] = ((unsigned long long)v.y << 32) | v.x;
    } else {
        o.out[2 * p] = v.x;
        o.out[2 * p + 1] = v.y;
    }
}

// one global reservation of m slots on *total by lane 0, broadcast (wave-uniform)
__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* total, unsigned m) {
    unsigned lo = 0, hi = 0;
    if (lane_id() == 0) {
        const unsigned long long b = atomicAdd(total, (unsigned long long)m);
        lo = (unsigned)b;
        hi = (unsigned)(b >> 32);
    }
    return ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)hi) << 32) |
           (unsigned)__builtin_amdgcn_readfirstlane((int)lo);
}

// the wave's spill list (StreamOut::covf): the chunk's candidates whose LDS region filled before
// the chunk's end, kept as packed words until the chunk's one reservation
__device__ __forceinline__ unsigned* stream_ovf(const StreamOut& o) {
    return o.covf + ((size_t)blockIdx.x * kStreamNW + threadIdx.x / kWave) * o.covf_wave;
}

// entries [0, m) of a staged region (chunk c0) to their slots from base on (wave-cooperative)
__device__ __forceinline__ void stream_store_pairs(const StreamArgs& a, const unsigned* pk, unsigned m,
                                                   unsigned long long base, uint64_t c0) {
    for (unsigned t = (unsigned)lane_id(); t < m; t += kWave) {
        const unsigned v = pk[t];
        stream_emit_pair(a.o, base + t, v >> kLocalBits, (unsigned)(c0 + (v & (kStreamChunk - 1))));
    }
}
// packed candidate words [0, m) (LDS or the spill list) to slots base + t of the candidate buffer
__device__ __forceinline__ void stream_store_cands(const StreamArgs& a, const unsigned* pk, unsigned m,
                                                   unsigned long long base, uint64_t c0) {
    for (unsigned t = (unsigned)lane_id(); t < m; t += kWave) {
        const unsigned v = pk[t];
        const unsigned idx = (unsigned)(c0 + (v & (kStreamChunk - 1)));
        a.o.cpoly[base + t] = v >> kLocalBits;
        a.o.crec[base + t] = make_double4(a.x[idx], a.y[idx], __longlong_as_double((long long)idx), 0.0);
    }
}

// ppoly_stream_redo: the staged candidates decided at once by the exact test ppoly_cand_eval runs
// (PointPolygonRangeQuery.java:116, DistanceFunctions.java:33-36), hits reserved and stored
__device__ __forceinline__ void stream_decide_cands(const StreamArgs& a, const unsigned* pk, unsigned m, uint64_t c0) {
    for (unsigned t0 = 0; t0 < m; t0 += kWave) {
        const unsigned t = t0 + (unsigned)lane_id();
        bool hit = false;
        unsigned poly = 0, idx = 0;
        if (t < m) {
            const unsigned v = pk[t];
            poly = v >> kLocalBits;
            idx = (unsigned)(c0 + (v & (kStreamChunk - 1)));
            const PolyDev P = a.polys[poly];
            const double px = a.x[idx], py = a.y[idx];
            const SlabView sv{a.slabs + P.loff, P.ns};
            hit = P.nring > 1 ? point_polygon_within_rings(px, py, a.vx + P.voff, a.vy + P.voff, a.vring + P.voff,
                                                           a.renv + 4 * (size_t)P.eoff, P, sv, a.r)
                              : point_polygon_within(px, py, a.vx + P.voff, a.vy + P.voff, P, sv, a.r);
        }
        const unsigned long long mh = __ballot(hit);
        if (mh) {
            const unsigned long long pb = wave_reserve(a.o.ptotal, (unsigned)__popcll(mh));
            if (hit) stream_emit_pair(a.o, pb + lanes_below(mh), poly, idx);
        }
    }
}

// A wave's region full before the chunk's end: pairs get their own reservation and are stored;
// candidates go to the wave's spill list (the chunk reserves them all at its end, so a chunk's
// candidates either all fit the buffer or are all left to ppoly_stream_redo); in the redo kernel
// the candidates are decided at once.
template <bool CAND, bool REDO>
__device__ __forceinline__ void stream_flush(const StreamArgs& a, StreamSink& k, uint64_t c0) {
    wave_lds_sync();
    if (CAND && REDO) {
        stream_decide_cands(a, k.pk, k.n, c0);
    } else if (CAND) {
        if (k.ovn != kOvnLost) {  // wave-uniform
            if (k.ovn + k.n <= a.o.covf_wave) {
                unsigned* ovf = stream_ovf(a.o) + k.ovn;
                for (unsigned t = (unsigned)lane_id(); t < k.n; t += kWave) ovf[t] = k.pk[t];
                k.ovn += k.n;
            } else {
                k.ovn = kOvnLost;  // the spill list is full: the chunk's candidates go to the redo pass
            }
        }
    } else {
        const unsigned long long b = wave_reserve(a.o.ptotal, k.n);
        stream_store_pairs(a, k.pk, k.n, b, c0);
        if (lane_id() == 0) atomicAdd(a.o.flushes, 1u);
    }
    wave_lds_sync();
    k.n = 0;
}

// wave-uniform: lanes with `hit` stage a pair, lanes with `need` a candidate (never both):
// two ballots, one LDS store per lane
template <bool CANDS, bool REDO>
__device__ __forceinline__ void stream_push(const StreamArgs& a, StreamSink& ps, StreamSink& cs, bool hit, bool need,
                                            unsigned poly, unsigned loc, uint64_t c0) {
    if (REDO) hit = false;  // the redo kernel's chunks stored their pairs in the stream already
    const unsigned long long mp = __ballot(hit);
    const unsigned long long mc = CANDS ? __ballot(need) : 0ull;
    if (!(mp | mc)) return;
    const unsigned w = (poly << kLocalBits) | loc;
    if (CANDS) {
        unsigned* dst = hit ? ps.pk + ps.n + lanes_below(mp) : cs.pk + cs.n + lanes_below(mc);
        if (hit || need) *dst = w;
    } else if (hit) {
        ps.pk[ps.n + lanes_below(mp)] = w;
    }
    ps.n += (unsigned)__popcll(mp);
    if (CANDS) cs.n += (unsigned)__popcll(mc);
    if (!REDO && ps.n > ps.cap - kWave) stream_flush<false, REDO>(a, ps, c0);
    if (CANDS && cs.n > cs.cap - kWave) stream_flush<true, REDO>(a, cs, c0);
}

// Entry balance of the exact walk (round 5; it replaced each lane walking its own points' entries
// as one list, entries addressed from the heads' prefix: 512 -> 460 us): per wave iteration, the multi-entry cells'
// entries are numbered across the wave and every lane takes kBalItems of them per step, so a step
// serves the wave's entries evenly (a lane's own list had ~7 entries on average and ~14 at the
// wave's maximum: half of every step's lanes idle) and an iteration needs one round of entry
// gathers, not one per entry of the longest list.  Per wave in LDS: one record per multi-entry
// slot (kBalRecs) and a bitmap of the entries that start a record (kBalWords x 64 entries); an
// iteration that exceeds either takes the per-lane walk.
constexpr unsigned kBalRecs = 128;
constexpr unsigned kBalWords = 16;
// entries per lane per balanced step (same box: 1 450, 2 448, 3 457, 4 463, 6 479 us)
constexpr unsigned kBalItems = 2;

// the class decision of one entry (ex, word) for a point with subcell / NaN bits sw:
// PointPolygonRangeQuery.java:105-121 -- G -> pair; C -> by the subcell class (mixed: candidate)
// (branch-free: selects instead of the early returns, whose exec-mask bookkeeping cost more
// scalar instructions than the decision itself; kWordHit / kWordMiss are the all-hit / all-miss
// fields, so the subcell's field covers them)
__device__ __forceinline__ void stream_decide(uint32_t ex, uint32_t word, unsigned sw, bool& hit, bool& need) {
    constexpr unsigned kNanBit = 16u;
    static_assert(kWordHit == 0x55555555u && kClsHit == 1 && kWordMiss == 0xAAAAAAAAu && kClsMiss == 2,
                  "uniform class words are their fields repeated");
    // a decided class holds for every point in the cell's coordinate box: not for NaN
    // coordinates (cell 0 by Java's (int) NaN)
    const unsigned field = (word >> (2u * (sw & 15u))) & 3u;
    const unsigned kc = (sw & kNanBit) ? (unsigned)kClsMixed : field;
    const bool some = ex != kNoEntry, g = (ex & kEntC) == 0u;
    hit = some & (g | (kc == kClsHit));
    need = some & !g & (kc == kClsMixed);
}

// One chunk's points (all waves of the block).  Phase A: every point of the wave's iterations --
// coordinates (next iteration's in flight), cell, subcell, and its table head gather issued;
// phase B: the entries, with all the wave's heads already in flight from phase A (a head gather
// per iteration waited on at once cost ~1 us of latency per iteration under the streaming
// traffic).  Phase B needs no coordinates except for the approximate bbox test and the rare
// out-of-grid polygons (reloaded).
// Coordinates of the first wave iteration of chunk [c0, c1) (loaded by stream_chunk itself, or by the
// kernel ahead of the previous chunk's write-out: its loads then return before those stores).
struct StreamPre {
    double x[4], y[4];
};
template <bool APPROX, bool KL, bool REDO = false>
__device__ __forceinline__ void stream_chunk(const StreamArgs& a, const unsigned* kl, uint64_t c0, uint64_t c1,
                                             StreamSink& ps, StreamSink& cs, uint2* brec, unsigned long long* bbm,
                                             const StreamPre* pre) {
    const int wid = threadIdx.x / kWave, lane = lane_id();
    const TileGeom& g = a.g;
    const unsigned nb = (unsigned)g.nb;
    constexpr unsigned kIters = kStreamChunk / (kStreamNW * kStreamPts);
    auto load = [&](unsigned t, double (&qx)[4], double (&qy)[4]) {
        const uint64_t base = c0 + (uint64_t)(t * kStreamNW + wid) * kStreamPts;
        const uint64_t i0 = base + 2 * (uint64_t)lane, i1 = i0 + 128;
        if (base + kStreamPts <= c1) {
            // plain loads (nontemporal: 472 against 460 us of ppoly_stream, round 5)
            const double2 ax = *reinterpret_cast<const double2*>(a.x + i0);
            const double2 bx = *reinterpret_cast<const double2*>(a.x + i1);
            const double2 ay = *reinterpret_cast<const double2*>(a.y + i0);
            const double2 by = *reinterpret_cast<const double2*>(a.y + i1);
            qx[0] = ax.x; qx[1] = ax.y; qx[2] = bx.x; qx[3] = bx.y;
            qy[0] = ay.x; qy[1] = ay.y; qy[2] = by.x; qy[3] = by.y;
        } else {
            const uint64_t id[4] = {i0, i0 + 1, i1, i1 + 1};
#pragma unroll
            for (int s = 0; s < 4; s++) {
                qx[s] = id[s] < c1 ? a.x[id[s]] : 0.0;
                qy[s] = id[s] < c1 ? a.y[id[s]] : 0.0;
            }
        }
    };
    auto loc_of = [&](unsigned t, int s) {
        return (t * kStreamNW + (unsigned)wid) * kStreamPts + 2u * (unsigned)lane + (unsigned)(s & 1) +
               128u * (unsigned)(s >> 1);
    };
    const double mnlx = __builtin_fabs(g.mnx) * g.il, mnly = __builtin_fabs(g.mny) * g.il;
    const double il4 = g.il * 4.0;
    // point state for phase B: bits 0-3 subcell (4 sx + sy), 4 NaN coordinate, 5 outside the grid
    constexpr unsigned kNanBit = 16u, kOutBit = 32u;
    uint2 hd[kIters][4];
    unsigned st[kIters];  // one byte per point
    double nx[4], ny[4];
    if (pre) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            nx[s] = pre->x[s];
            ny[s] = pre->y[s];
        }
    } else {
        load(0, nx, ny);
    }
#pragma unroll
    for (unsigned t = 0; t < kIters; t++) {
        double qx[4], qy[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            qx[s] = nx[s];
            qy[s] = ny[s];
        }
        if (t + 1 < kIters) load(t + 1, nx, ny);
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const bool v = c0 + loc_of(t, s) < c1;
            unsigned sx = 0, sy = 0;
            bool okx = false, oky = false;
            const int32_t cx = d_axis_cell_sub4(qx[s], g.mnx, g.l, g.il, il4, mnlx, sx, okx);
            const int32_t cy = d_axis_cell_sub4(qy[s], g.mny, g.l, g.il, il4, mnly, sy, oky);
            const bool in = v && cx >= 0 && cy >= 0 && cx < g.nb && cy < g.nb;
            const bool nan = !(qx[s] == qx[s] && qy[s] == qy[s]);
            unsigned w = (nan ? kNanBit : 0u) | ((v && !in) ? kOutBit : 0u);
            hd[t][s] = make_uint2(kNoEntry, 0u);
            if (in) {
                const unsigned key = (unsigned)cx * nb + (unsigned)cy;
                bool has = true;
                if (KL) has = (kl[key >> 5] >> (key & 31u)) & 1u;
                else if (a.keep) has = (a.keep[key >> 5] >> (key & 31u)) & 1u;
                if (has) hd[t][s] = a.head[key];
                if (has && !nan && !APPROX) {
                    // the subcell from the cell computation's quotient, exact outside a margin
                    // around the subcell edges; the edges' own arithmetic inside it (rare)
                    if (__ballot(!(okx && oky))) {
                        if (!okx) sx = (unsigned)sub_of(qx[s], g.mnx, g.l, cx);
                        if (!oky) sy = (unsigned)sub_of(qy[s], g.mny, g.l, cy);
                    }
                    w |= 4u * sx + sy;
                }
            }
            st[t] = s == 0 ? w : (st[t] | (w << (8 * s)));
        }
    }
    if (!APPROX) {
        // Phase B (exact, balanced): per iteration, single-entry slots decided by their own lanes
        // (the head is the entry: no gather), multi-entry slots recorded for the wave
#pragma unroll
        for (unsigned t = 0; t < kIters; t++) {
            unsigned cnt[4], lc = 0, ln = 0;
#pragma unroll
            for (int sl = 0; sl < 4; sl++) {
                const uint2 h = hd[t][sl];
                const bool multi = h.x != kNoEntry && (h.x & kMulti);
                cnt[sl] = multi ? (h.x & ~kMulti) : 0u;
                lc += cnt[sl];
                ln += multi ? 1u : 0u;
                bool hit = false, need = false;
                if (!multi) stream_decide(h.x, h.y, st[t] >> (8 * sl), hit, need);
                const unsigned loc = loc_of(t, sl);
                stream_push<true, REDO>(a, ps, cs, hit, need, h.x & ~kEntC, loc, c0);
            }
            const unsigned ic = wave_incl_scan(lc), in = wave_incl_scan(ln);
            const unsigned T = (unsigned)__builtin_amdgcn_readlane((int)ic, kWave - 1);
            const unsigned R = (unsigned)__builtin_amdgcn_readlane((int)in, kWave - 1);
            if (T == 0) continue;
            if (T > kBalWords * kWave || R > kBalRecs) {
                // rare (cells of many polygons): each lane walks its own multi-entry slots
#pragma unroll
                for (int sl = 0; sl < 4; sl++) {
                    unsigned e = cnt[sl] ? hd[t][sl].y : 0u;
                    const unsigned e1 = e + cnt[sl];
                    const unsigned sw = st[t] >> (8 * sl), loc = loc_of(t, sl);
                    while (__ballot(e < e1)) {
                        uint2 en = make_uint2(kNoEntry, 0u);
                        if (e < e1) en = a.ent[e++];
                        bool hit, need;
                        stream_decide(en.x, en.y, sw, hit, need);
                        stream_push<true, REDO>(a, ps, cs, hit, need, en.x & ~kEntC, loc, c0);
                    }
                }
                continue;
            }
            // records (first entry, loc | sw << 12 | start << 17) and the entry-start bitmap
            if ((unsigned)lane < (T + kWave - 1) / kWave) bbm[lane] = 0ull;
            wave_lds_sync();
            unsigned p = ic - lc, r = in - ln;
#pragma unroll
            for (int sl = 0; sl < 4; sl++) {
                if (cnt[sl]) {
                    brec[r] = make_uint2(hd[t][sl].y, loc_of(t, sl) | (((st[t] >> (8 * sl)) & 31u) << 12) | (p << 17));
                    atomicOr(&bbm[p >> 6], 1ull << (p & 63u));
                    r++;
                    p += cnt[sl];
                }
            }
            wave_lds_sync();
            // entries w = w0 + 64 u + lane: the record = starts at or below w, minus one
            unsigned carry = 0;
            const unsigned long long le = ~0ull >> (63 - lane);
            for (unsigned w0 = 0; w0 < T; w0 += kBalItems * kWave) {  // wave-uniform
                uint2 en[kBalItems];
                unsigned ry[kBalItems];
#pragma unroll
                for (unsigned u = 0; u < kBalItems; u++) {
                    const unsigned wb = w0 + u * kWave, w = wb + (unsigned)lane;
                    const unsigned long long word = wb < T ? bbm[wb >> 6] : 0ull;
                    const unsigned rr = carry + (unsigned)__popcll(word & le) - 1u;
                    carry += (unsigned)__popcll(word);
                    en[u] = make_uint2(kNoEntry, 0u);
                    ry[u] = 0u;
                    if (w < T) {
                        const uint2 rec = brec[rr];
                        ry[u] = rec.y;
                        en[u] = a.ent[rec.x + (w - (rec.y >> 17))];
                    }
                }
#pragma unroll
                for (unsigned u = 0; u < kBalItems; u++) {
                    bool hit, need;
                    stream_decide(en[u].x, en[u].y, ry[u] >> 12, hit, need);
                    const unsigned loc = ry[u] & (kStreamChunk - 1);
                    stream_push<true, REDO>(a, ps, cs, hit, need, en[u].x & ~kEntC, loc, c0);
                }
            }
            wave_lds_sync();  // the records and bitmap are reused by the next iteration
        }
    }
#pragma unroll
    for (unsigned t = 0; t < kIters; t++) {
        double qx[4] = {0.0, 0.0, 0.0, 0.0}, qy[4] = {0.0, 0.0, 0.0, 0.0};
        const bool any_out = __ballot((st[t] & (kOutBit * 0x01010101u)) != 0) != 0;
        if (APPROX || (a.nopoly && any_out)) load(t, qx, qy);  // reloaded (L2): bbox test, outside points
#pragma unroll
        for (int s = 0; s < 4; s++) {
            if (!APPROX) break;  // exact: the worklist above walked the entries
            const unsigned loc = loc_of(t, s);
            const unsigned sw = st[t] >> (8 * s);
            const bool nan = sw & kNanBit;
            const unsigned sub = sw & 15u;
            // entry cursor: the head's entry (single) or cell_ent[e, e1) (multi)
            uint32_t ex = hd[t][s].x, word = hd[t][s].y;
            unsigned e = 0, e1 = 0;
            if (ex != kNoEntry && (ex & kMulti)) {
                e = word;
                e1 = e + (ex & ~kMulti);
                const uint2 en = a.ent[e++];
                ex = en.x;
                word = en.y;
            }
            while (__ballot(ex != kNoEntry)) {
                bool hit = false, need = false;
                unsigned poly = 0;
                if (ex != kNoEntry) {
                    poly = ex & ~kEntC;
                    if (!(ex & kEntC)) {
                        hit = true;
                    } else if (APPROX) {
                        hit = bbox_distance(qx[s], qy[s], a.polys[poly].bb) <= a.r;
                    } else {
                        // a decided class holds for every point in the cell's coordinate box: not
                        // for NaN coordinates (cell 0 by Java's (int) NaN)
                        uint32_t k = kClsMixed;
                        if (!nan) {
                            if (word == kWordHit) k = kClsHit;
                            else if (word == kWordMiss) k = kClsMiss;
                            else k = (word >> (2 * sub)) & 3u;
                        }
                        hit = k == kClsHit;
                        need = k == kClsMixed;
                    }
                    if (e < e1) {  // the cell's next entry
                        const uint2 en = a.ent[e++];
                        ex = en.x;
                        word = en.y;
                    } else {
                        ex = kNoEntry;
                    }
                }
                stream_push<!APPROX, REDO>(a, ps, cs, hit, need, poly, loc, c0);
            }
        }
        // points outside the grid against the polygons whose rectangles reach outside it (rare)
        if (a.nopoly && any_out) {
            for (int s = 0; s < 4; s++) {
                const bool o = (st[t] >> (8 * s)) & kOutBit;
                int32_t cx = 0, cy = 0;
                if (o) {
                    cx = d_axis_cell(qx[s], g.mnx, g.l);
                    cy = d_axis_cell(qy[s], g.mny, g.l);
                }
                for (uint32_t j = 0; j < a.nopoly; j++) {
                    const uint32_t p = a.opoly[j];
                    const PolyDev& P = a.polys[p];
                    // range: the guaranteed rectangles; join exact: the checked list (+ the exact
                    // test); join approximate: every rectangle is in the G list
                    bool in = false;
                    if (o)
                        in = a.jmode == 1 ? in_rects(a.rects + 4 * P.coff, P.nc, cx, cy)
                                          : in_rects(a.rects + 4 * P.goff, P.ng, cx, cy);
                    const bool dist = !APPROX && a.jmode == 1;
                    stream_push<!APPROX, REDO>(a, ps, cs, in && !dist, in && dist, p, loc_of(t, s), c0);
                }
            }
        }
    }
}

// Persistent blocks take the kStreamChunk-point chunks blockIdx.x, + gridDim.x, ...  Per chunk: pairs
// and candidates staged in LDS (4 B each), then one atomic reservation each on the pair and
// candidate totals (the output is unordered: no look-back, no chunk waits for another) and
// coalesced stores.  A chunk whose stage overflowed runs again with its reservations made from
// the counts, storing every pair / candidate straight to its slot.
// the register budget held to 4 waves per SIMD (LDS allows 4; 5-6 spilled, 670-700 us; 3: 1.07 ms)
template <bool APPROX, bool KL>
__global__ __launch_bounds__(kStreamNW * kWave) __attribute__((amdgpu_waves_per_eu(4))) void ppoly_stream(StreamArgs a) {
    __shared__ unsigned kl[KL ? kKeepLds : 1];
    __shared__ unsigned ppk[kSPairCap];
    __shared__ unsigned cpk[APPROX ? 1 : kSCandCap];
    __shared__ unsigned s_wp[kStreamNW], s_wc[kStreamNW];  // per-wave staged counts
    __shared__ unsigned long long s_pb, s_cb;
    constexpr bool kBal = !APPROX;
    __shared__ uint2 brec[kBal ? kStreamNW * kBalRecs : 1];             // balanced walk: records
    __shared__ unsigned long long bbm[kBal ? kStreamNW * kBalWords : 1];  // and entry-start bitmaps
    constexpr unsigned kWPair = kSPairCap / kStreamNW, kWCand = kSCandCap / kStreamNW;
    const int wid = threadIdx.x / kWave, lane = lane_id();
    if (KL)
        for (unsigned t = threadIdx.x; t < a.keep_words; t += kStreamNW * kWave) kl[t] = a.keep[t];
    const unsigned nchunks = (unsigned)((a.n + kStreamChunk - 1) / kStreamChunk);
    // the first wave iteration's coordinates of the block's next chunk, loaded before the current
    // chunk's reservation and pair stores (gfx9: one vmcnt for loads and stores -- loads issued
    // after the stores would wait for them to drain)
    StreamPre pre;
    auto prefetch = [&](unsigned v) {
        const uint64_t b0 = (uint64_t)v * kStreamChunk + (uint64_t)wid * kStreamPts;
        const uint64_t b1 = (uint64_t)v * kStreamChunk + kStreamChunk < a.n ? (uint64_t)v * kStreamChunk + kStreamChunk : a.n;
        const uint64_t i0 = b0 + 2 * (uint64_t)lane, i1 = i0 + 128;
        if (b0 + kStreamPts <= b1) {
            const double2 ax = *reinterpret_cast<const double2*>(a.x + i0);
            const double2 bx = *reinterpret_cast<const double2*>(a.x + i1);
            const double2 ay = *reinterpret_cast<const double2*>(a.y + i0);
            const double2 by = *reinterpret_cast<const double2*>(a.y + i1);
            pre.x[0] = ax.x; pre.x[1] = ax.y; pre.x[2] = bx.x; pre.x[3] = bx.y;
            pre.y[0] = ay.x; pre.y[1] = ay.y; pre.y[2] = by.x; pre.y[3] = by.y;
        } else {
            const uint64_t id[4] = {i0, i0 + 1, i1, i1 + 1};
#pragma unroll
            for (int s = 0; s < 4; s++) {
                pre.x[s] = id[s] < b1 ? a.x[id[s]] : 0.0;
                pre.y[s] = id[s] < b1 ? a.y[id[s]] : 0.0;
            }
        }
    };
    if (blockIdx.x < nchunks) prefetch(blockIdx.x);
    for (unsigned vb = blockIdx.x; vb < nchunks; vb += gridDim.x) {
        __syncthreads();  // the previous chunk's stage is drained (and the bitmap staged)
        const uint64_t c0 = (uint64_t)vb * kStreamChunk;
        const uint64_t c1 = c0 + kStreamChunk < a.n ? c0 + kStreamChunk : a.n;
        StreamSink ps{ppk + wid * kWPair, kWPair, 0u, 0u};
        StreamSink cs{cpk + (APPROX ? 0 : wid * kWCand), APPROX ? kWave : kWCand, 0u, 0u};
        uint2* wrec = kBal ? brec + wid * kBalRecs : brec;
        unsigned long long* wbm = kBal ? bbm + wid * kBalWords : bbm;
        stream_chunk<APPROX, KL>(a, kl, c0, c1, ps, cs, wrec, wbm, &pre);
        if (vb + gridDim.x < nchunks) prefetch(vb + gridDim.x);
        if (lane == 0) {
            s_wp[wid] = ps.n;
            // staged in LDS + spilled before the chunk's end (or kOvnLost)
            s_wc[wid] = cs.ovn == kOvnLost ? kOvnLost : cs.n + cs.ovn;
        }
        __syncthreads();
        unsigned np = 0, nc = 0, pex = 0, cex = 0;  // totals; this wave's offsets in the chunk
        bool lost = false;                          // block-uniform: a wave's spill list filled
#pragma unroll
        for (int w = 0; w < kStreamNW; w++) {
            const unsigned wp = s_wp[w], wc0 = s_wc[w];
            lost = lost || wc0 == kOvnLost;
            const unsigned wc = wc0 == kOvnLost ? 0u : wc0;
            pex += w < wid ? wp : 0u;
            cex += w < wid ? wc : 0u;
            np += wp;
            nc += wc;
        }
        if (lost) nc = 0;  // nothing reserved: the redo pass decides every candidate of the chunk
        if (threadIdx.x == 0) {
            s_pb = np ? atomicAdd(a.o.ptotal, (unsigned long long)np) : 0ull;
            s_cb = nc ? atomicAdd(a.o.ctotal, (unsigned long long)nc) : 0ull;
            // a chunk whose candidates do not all fit the buffer (or its spill lists) leaves them
            // all to the redo pass
            if (!APPROX && (lost || (nc && s_cb + nc > a.o.ccap))) a.o.redo[atomicAdd(a.o.nredo, 1u)] = vb;
        }
        __syncthreads();
        // each wave stores its own region: coalesced runs of the output
        stream_store_pairs(a, ppk + wid * kWPair, ps.n, s_pb + pex, c0);
        if (!APPROX && !lost) {
            const unsigned long long cb = s_cb + cex;
            const unsigned wc = cs.n + cs.ovn;
            if (s_cb + nc <= a.o.ccap) {
                stream_store_cands(a, cpk + wid * kWCand, cs.n, cb, c0);
                if (cs.ovn) stream_store_cands(a, stream_ovf(a.o), cs.ovn, cb + cs.n, c0);
            } else {  // its slots below the capacity are marked gone (the grouping skips them)
                for (unsigned t = (unsigned)lane; t < wc && cb + t < a.o.ccap; t += kWave) a.o.cpoly[cb + t] = kCandGone;
            }
        }
    }
}

// The chunks ppoly_stream left to redo (their candidates did not fit the candidate buffer, which
// is sized from the previous call's count): each is walked again with pairs off (the stream stored
// them) and its candidates decided at once by the exact test.  Rare by construction (a first call,
// or a window with many more candidates than the last); with an empty list every block exits at
// once.  No call runs the step twice.
template <bool KL>
__global__ __launch_bounds__(kStreamNW * kWave) void ppoly_stream_redo(StreamArgs a) {
    __shared__ unsigned kl[KL ? kKeepLds : 1];
    __shared__ unsigned cpk[kSCandCap];
    __shared__ uint2 brec[kStreamNW * kBalRecs];
    __shared__ unsigned long long bbm[kStreamNW * kBalWords];
    constexpr unsigned kWCand = kSCandCap / kStreamNW;
    const unsigned nredo = *a.o.nredo;
    if (blockIdx.x >= nredo) return;
    const int wid = threadIdx.x / kWave;
    if (KL)
        for (unsigned t = threadIdx.x; t < a.keep_words; t += kStreamNW * kWave) kl[t] = a.keep[t];
    unsigned dummy = 0;
    for (unsigned i = blockIdx.x; i < nredo; i += gridDim.x) {
        __syncthreads();
        const unsigned vb = a.o.redo[i];
        const uint64_t c0 = (uint64_t)vb * kStreamChunk;
        const uint64_t c1 = c0 + kStreamChunk < a.n ? c0 + kStreamChunk : a.n;
        StreamSink ps{&dummy, 0x7fffffffu, 0u, 0u};  // pairs off
        StreamSink cs{cpk + wid * kWCand, kWCand, 0u, 0u};
        stream_chunk<false, KL, true>(a, kl, c0, c1, ps, cs, brec + wid * kBalRecs, bbm + wid * kBalWords, nullptr);
        wave_lds_sync();
        stream_decide_cands(a, cs.pk, cs.n, c0);
    }
}

// Pairs of the exact tests: per-wave LDS buffers appended behind the stream's pairs, one global
// atomic per buffer on the pair total (the stream's last chunk wrote it before this launch).
constexpr unsigned kSPairs = 512;
__device__ __forceinline__ void spairs_flush(uint2* buf, unsigned& cnt, const StreamOut& o) {
    wave_lds_sync();
    unsigned lo = 0, hi = 0;
    if (lane_id() == 0) {
        const unsigned long long b = atomicAdd(o.ptotal, (unsigned long long)cnt);
        lo = (unsigned)b;
        hi = (unsigned)(b >> 32);
    }
    const unsigned long long base = ((unsigned long long)__shfl(hi, 0) << 32) | __shfl(lo, 0);
    for (unsigned t = lane_id(); t < cnt; t += kWave) stream_emit_pair(o, base + t, buf[t].x, buf[t].y);
    wave_lds_sync();
    cnt = 0;
}
template <unsigned CAP = kSPairs>
__device__ __forceinline__ void spairs_push(uint2* buf, unsigned& cnt, bool hit, unsigned poly, unsigned idx,
                                            const StreamOut& o) {
    const unsigned long long m = __ballot(hit);
    if (!m) return;
    if (hit) buf[cnt + lanes_below(m)] = make_uint2(poly, idx);
    cnt += (unsigned)__popcll(m);
    if (cnt > CAP - (unsigned)kWave) spairs_flush(buf, cnt, o);
}

// Grouping of the candidates by polygon: a counting sort.  kCandGroups blocks each own a
// contiguous range of the candidates: per-polygon counts of the range in LDS -> row b of a
// [kCandGroups][npoly] matrix and, one atomic per nonzero count, the polygons' totals
// (ppoly_cand_hist); one block scans the totals into the polygons' runs, their cursors and the
// work items (ppoly_cand_plan); the same ranges reserve their slice of each run from its cursor
// (one atomic per nonzero count) and scatter into it (ppoly_cand_scatter).  (The plan block
// summing the matrix's columns and scanning them per range took 21 us for C4's 1000 polygons;
// the order of the ranges inside a run is free: the pairs are unordered.)
constexpr unsigned kCandGroups = 128;
constexpr unsigned kCandThreads = 1024;
constexpr unsigned kCandPer = 4;  // candidates per thread per round (loads in flight together)
struct CandGroup {
    const unsigned long long* ccount;  // candidate total (StreamOut::ctotal, or the refined count)
    const unsigned long long* cstream; // the stream's candidate total (the capacity check)
    uint64_t ccap;
    unsigned* fault;                   // async calls: the ctx's fault word (kFaultCandNeed), else null
    unsigned long long* need;          // async calls: the candidate count an overflowing call needed
    const unsigned* cpoly;
    const double4* crec;
    unsigned* mat;          // [kCandGroups][npoly]: each range's counts
    unsigned* ptot;         // [npoly] candidates per polygon (zeroed with the step's totals)
    unsigned* pcur;         // [npoly] run cursors: each range reserves its slice of a run
    uint32_t npoly;         // <= kCandLdsPolys
    uint4* items;           // (poly, begin, end, -)
    unsigned* nitems;
    unsigned* eticket;      // the evaluation's item ticket (zeroed with the step's totals)
    unsigned* sidx;         // sorted runs: slots of the unsorted candidate arrays
};

__device__ __forceinline__ uint64_t cand_n(const CandGroup& c) {
    const unsigned long long n = *c.ccount;
    return n < c.ccap ? n : c.ccap;
}
__device__ __forceinline__ void cand_range(const CandGroup& c, uint64_t& b0, uint64_t& b1) {
    const uint64_t n = cand_n(c);
    const uint64_t per = (n + kCandGroups - 1) / kCandGroups;
    b0 = (uint64_t)blockIdx.x * per < n ? (uint64_t)blockIdx.x * per : n;
    b1 = b0 + per < n ? b0 + per : n;
}

__global__ __launch_bounds__(kCandThreads) void ppoly_cand_hist(CandGroup c) {
    __shared__ unsigned h[kCandLdsPolys];
    uint64_t b0, b1;
    cand_range(c, b0, b1);
    for (unsigned t = threadIdx.x; t < c.npoly; t += kCandThreads) h[t] = 0;
    __syncthreads();
    for (uint64_t i0 = b0 + threadIdx.x; i0 < b1; i0 += (uint64_t)kCandPer * kCandThreads) {
        unsigned p[kCandPer];
#pragma unroll
        for (unsigned u = 0; u < kCandPer; u++) {
            const uint64_t i = i0 + (uint64_t)u * kCandThreads;
            p[u] = i < b1 ? c.cpoly[i] : kCandGone;
        }
#pragma unroll
        for (unsigned u = 0; u < kCandPer; u++)
            if (p[u] != kCandGone) atomicAdd(&h[p[u]], 1u);
    }
    __syncthreads();
    unsigned* row = c.mat + (size_t)blockIdx.x * c.npoly;
    for (unsigned t = threadIdx.x; t < c.npoly; t += kCandThreads) {
        const unsigned v = h[t];
        row[t] = v;
        if (v) atomicAdd(&c.ptot[t], v);
    }
}

// one block: the polygons' totals scanned into run starts (their cursors) and the kCandItem
// work items -- every polygon's full items first, then the partial ones (the evaluation claims
// items in order, so the long items start first and the short ones fill in behind them)
__global__ __launch_bounds__(kCandThreads) void ppoly_cand_plan(CandGroup c) {
    __shared__ unsigned sc[kCandThreads], sf[kCandThreads], sp[kCandThreads];
    __shared__ unsigned carry_c, carry_f, carry_p, nfull;
    if (threadIdx.x == 0) {
        carry_c = 0;
        carry_f = 0;
        carry_p = 0;
        nfull = 0;
    }
    __syncthreads();
    {  // the full items' count (the partial items follow them)
        unsigned f = 0;
        for (unsigned p = threadIdx.x; p < c.npoly; p += kCandThreads) f += c.ptot[p] / kCandItem;
        f = wave_incl_scan(f);
        if (lane_id() == kWave - 1 && f) atomicAdd(&nfull, f);
    }
    __syncthreads();
    const unsigned F = nfull;
    for (unsigned p0 = 0; p0 < c.npoly; p0 += kCandThreads) {
        const unsigned p = p0 + threadIdx.x;
        const unsigned tot = p < c.npoly ? c.ptot[p] : 0u;
        const unsigned nf = tot / kCandItem, np = tot % kCandItem ? 1u : 0u;
        sc[threadIdx.x] = tot;
        sf[threadIdx.x] = nf;
        sp[threadIdx.x] = np;
        __syncthreads();
        for (unsigned o = 1; o < kCandThreads; o <<= 1) {
            const unsigned a = threadIdx.x >= o ? sc[threadIdx.x - o] : 0u;
            const unsigned b = threadIdx.x >= o ? sf[threadIdx.x - o] : 0u;
            const unsigned d = threadIdx.x >= o ? sp[threadIdx.x - o] : 0u;
            __syncthreads();
            sc[threadIdx.x] += a;
            sf[threadIdx.x] += b;
            sp[threadIdx.x] += d;
            __syncthreads();
        }
        const unsigned start = carry_c + sc[threadIdx.x] - tot;
        const unsigned f0 = carry_f + sf[threadIdx.x] - nf, p0i = F + carry_p + sp[threadIdx.x] - np;
        if (p < c.npoly) {
            c.pcur[p] = start;
            for (unsigned k = 0; k < nf; k++) {
                const unsigned lo = start + k * kCandItem;
                c.items[f0 + k] = make_uint4(p, lo, lo + kCandItem, 0u);
            }
            if (np) c.items[p0i] = make_uint4(p, start + nf * kCandItem, start + tot, 0u);
        }
        __syncthreads();
        if (threadIdx.x == kCandThreads - 1) {
            carry_c += sc[kCandThreads - 1];
            carry_f += sf[kCandThreads - 1];
            carry_p += sp[kCandThreads - 1];
        }
        __syncthreads();
    }
    const unsigned carry_i = F + carry_p;
    if (threadIdx.x == 0) {
        *c.nitems = carry_i;
        // a short candidate buffer (the chunks past it went to the redo pass): the size it needed
        // goes to the ctx's fault block as a hint, so the next async call sizes it
        const unsigned long long nc = *c.cstream;
        if (c.fault && nc > c.ccap) {
            atomicOr(c.fault, kFaultCandNeed);
            atomicMax(c.need, nc);
        }
    }
}

// Only the 4-byte slot of each candidate moves (a random scatter of its 20 bytes cost 3x the
// time); the evaluation gathers the coordinates from the unsorted arrays.
__global__ __launch_bounds__(kCandThreads) void ppoly_cand_scatter(CandGroup c) {
    __shared__ unsigned h[kCandLdsPolys];
    uint64_t b0, b1;
    cand_range(c, b0, b1);
    const unsigned* row = c.mat + (size_t)blockIdx.x * c.npoly;
    for (unsigned t = threadIdx.x; t < c.npoly; t += kCandThreads) {
        const unsigned v = row[t];
        h[t] = v ? atomicAdd(&c.pcur[t], v) : 0u;  // this range's slice of the run
    }
    __syncthreads();
    for (uint64_t i0 = b0 + threadIdx.x; i0 < b1; i0 += (uint64_t)kCandPer * kCandThreads) {
        unsigned p[kCandPer];
#pragma unroll
        for (unsigned u = 0; u < kCandPer; u++) {
            const uint64_t i = i0 + (uint64_t)u * kCandThreads;
            p[u] = i < b1 ? c.cpoly[i] : kCandGone;
        }
#pragma unroll
        for (unsigned u = 0; u < kCandPer; u++)
            if (p[u] != kCandGone) c.sidx[atomicAdd(&h[p[u]], 1u)] = (unsigned)(i0 + (uint64_t)u * kCandThreads);
    }
}

// Exact test of each grouped candidate: one work item = one polygon's run slice, its rings,
// ring ids, fp32 segment boxes and slab lists staged in LDS as in ppoly_eval.  The slice is
// ordered by y slab in LDS first (counting sort, 64 bins), so the lanes of a wave mostly walk
// the same crossing and distance lists (equal trip counts, broadcast LDS reads).
// Refinement of the stream's candidates (round 5): a candidate's point lies in a mixed subcell of
// its polygon's cell; the subcell's 4 x 4 parts were classified on the host (classify_cells), so
// its part decides it as a pair (HIT), nothing (MISS) or still a candidate (MIXED, or NaN
// coordinates, or no refinement).  A decided candidate's polygon slot becomes kCandGone, which
// the grouping skips (its range-end sentinel): no compaction, no counter -- the survivors, about
// a quarter for C4, go on to the grouping and the exact tests.  (Compacting survivors with a
// per-wave reservation on one counter serialised ~44k atomics: 568 us for C4; in place per
// grouping range, 128 blocks: 176 us; both measured.)  Pairs through per-wave LDS stages.
struct CandRefine {
    const unsigned long long* ccount;  // the stream's candidates (ctotal)
    uint64_t ccap;
    unsigned* cpoly;                   // decided candidates -> kCandGone
    const double4* crec;
    const PolyDev* polys;
    const uint2* rf;                   // per walk-region cell (PolyDev.cls indexing): (refinement base, class word)
    const uint2* rfw;                  // per mixed subcell: (part word, first second-level word)
    const uint32_t* rfw2;              // per mixed part: sub-part word
    double mnx, mny, l;                // the point grid (cells as the stream computed them)
};
// Pairs go to a block-wide LDS stage (kRefineStage) reserved with one global atomic per flush --
// about one per block (per-wave stages flushed every ~128 pairs cost 83 of the kernel's 148 us
// for C4: same-address atomics); kRefinePer candidates per thread per round keep their gather
// chains (slot -> polygon -> refinement base -> word) in flight together.
// (2 / 8 candidates per thread: 72.5 / 84.4 against 70.9 us at 4, round 5)
constexpr unsigned kRefineBlocks = 1024, kRefinePer = 4, kRefineStage = 4096;
__global__ __launch_bounds__(kTB) void ppoly_cand_refine(CandRefine c, StreamOut o) {
    __shared__ uint2 stage[kRefineStage];
    __shared__ unsigned s_n;
    __shared__ unsigned long long s_base;
    const int lane = lane_id();
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    auto flush = [&]() {  // block-uniform
        __syncthreads();
        const unsigned n = s_n;
        if (threadIdx.x == 0) s_base = atomicAdd(o.ptotal, (unsigned long long)n);
        __syncthreads();
        const unsigned long long base = s_base;
        for (unsigned t = threadIdx.x; t < n; t += kTB) stream_emit_pair(o, base + t, stage[t].x, stage[t].y);
        __syncthreads();
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
    };
    const unsigned long long nt = *c.ccount;
    const uint64_t n = nt < c.ccap ? nt : c.ccap;
    constexpr unsigned kRound = kTB * kRefinePer;
    for (uint64_t i0 = (uint64_t)blockIdx.x * kRound; i0 < n; i0 += (uint64_t)gridDim.x * kRound) {  // block-uniform
        // the chain slot -> polygon region -> refinement base -> part word, each level's loads for
        // the kRefinePer candidates issued together and unconditionally (clamped indices; the
        // branchy form waited for each candidate's chain in turn: 4 x 4 round trips per round)
        unsigned poly[kRefinePer], idx[kRefinePer];
        double2 xy[kRefinePer];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) {
            const uint64_t i = i0 + u * kTB + threadIdx.x;
            const uint64_t ii = i < n ? i : 0;
            poly[u] = c.cpoly[ii];
            xy[u] = *reinterpret_cast<const double2*>(&c.crec[ii]);
            idx[u] = reinterpret_cast<const unsigned*>(&c.crec[ii])[4];  // low word of the point bits
            if (i >= n) poly[u] = kCandGone;
        }
        uint32_t cls[kRefinePer];
        int32_t wx0[kRefinePer], wx1[kRefinePer], wy0[kRefinePer], wy1[kRefinePer];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) {
            const PolyDev& P = c.polys[poly[u] != kCandGone ? poly[u] : 0u];
            cls[u] = P.cls;
            wx0[u] = P.wx0;
            wx1[u] = P.wx1;
            wy0[u] = P.wy0;
            wy1[u] = P.wy1;
        }
        size_t ri[kRefinePer];
        bool go[kRefinePer];
        int32_t cx[kRefinePer], cy[kRefinePer];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) {
            cx[u] = d_axis_cell(xy[u].x, c.mnx, c.l);
            cy[u] = d_axis_cell(xy[u].y, c.mny, c.l);
            go[u] = poly[u] != kCandGone && xy[u].x == xy[u].x && xy[u].y == xy[u].y && cls[u] != kNoCls &&
                    cx[u] >= wx0[u] && cx[u] <= wx1[u] && cy[u] >= wy0[u] && cy[u] <= wy1[u];
            ri[u] = go[u] ? cls[u] + (size_t)(cx[u] - wx0[u]) * (uint32_t)(wy1[u] - wy0[u] + 1) + (uint32_t)(cy[u] - wy0[u]) : 0;
        }
        uint2 rb[kRefinePer];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) rb[u] = c.rf[ri[u]];
        uint32_t wi[kRefinePer], pt[kRefinePer], sh2[kRefinePer];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) {
            const int sx = sub_of(xy[u].x, c.mnx, c.l, cx[u]), sy = sub_of(xy[u].y, c.mny, c.l, cy[u]);
            const int tx = sub16_of(xy[u].x, c.mnx, c.l, cx[u], sx), ty = sub16_of(xy[u].y, c.mny, c.l, cy[u], sy);
            const int vx2 = sub64_of(xy[u].x, c.mnx, c.l, cx[u], 4 * sx + tx), vy2 = sub64_of(xy[u].y, c.mny, c.l, cy[u], 4 * sy + ty);
            const int sub = 4 * sx + sy;
            // the candidate's subcell is mixed (the stream emitted it for that); if not, it stays
            go[u] = go[u] && rb[u].x != kNoRefine && ((refine_mixed(rb[u].y) >> (2 * sub)) & 1u);
            wi[u] = go[u] ? rb[u].x + refine_rank(rb[u].y, sub) : 0u;
            pt[u] = 4 * tx + ty;
            sh2[u] = 2 * (4 * vx2 + vy2);
        }
        uint2 wd[kRefinePer];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) wd[u] = c.rfw[wi[u]];
        uint32_t code1[kRefinePer], w2i[kRefinePer];
        bool go2[kRefinePer];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) {
            code1[u] = go[u] ? (wd[u].x >> (2 * pt[u])) & 3u : kClsMixed;
            go2[u] = go[u] && code1[u] == kClsMixed && wd[u].y != kNoRefine;
            w2i[u] = go2[u] ? wd[u].y + refine_rank(wd[u].x, (int)pt[u]) : 0u;
        }
        uint32_t wd2[kRefinePer];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) wd2[u] = c.rfw2[w2i[u]];
#pragma unroll
        for (unsigned u = 0; u < kRefinePer; u++) {
            const uint64_t i = i0 + u * kTB + threadIdx.x;
            const uint32_t code = go2[u] ? (wd2[u] >> sh2[u]) & 3u : code1[u];
            const bool hit = code == kClsHit;
            const unsigned long long m = __ballot(hit);
            if (m) {  // this wave's hits: one LDS reservation
                unsigned wb = 0;
                if (lane == 0) wb = atomicAdd(&s_n, (unsigned)__popcll(m));
                wb = (unsigned)__shfl(wb, 0);
                if (hit) stage[wb + lanes_below(m)] = make_uint2(poly[u], idx[u]);
            }
            if (code != kClsMixed) c.cpoly[i] = kCandGone;
        }
        __syncthreads();
        if (s_n > kRefineStage - kRound) flush();
    }
    __syncthreads();
    if (s_n) flush();
}

// LDS of the candidate evaluation, sized for 4 blocks per CU (<= 40 KB: 4 waves per SIMD; the
// round-4 sizes -- 512 vertices, 2048 slab entries, 512 staged pairs per wave, 58.6 KB -- left 2
// blocks per CU and this latency-bound pass at 2 waves per SIMD).  Larger rings and slab lists
// are read from global memory (as ppoly_eval does past its limits).
constexpr int kEvalLdsVerts = 256;
constexpr int kEvalLdsSlab = 1024;
constexpr unsigned kEvalPairs = 256;
__global__ __launch_bounds__(kTB) void ppoly_cand_eval(CandGroup c, const PolyDev* __restrict__ polys,
                                                       const double* __restrict__ vx, const double* __restrict__ vy,
                                                       const ring_id_t* __restrict__ vring,
                                                       const double* __restrict__ renv,
                                                       const uint16_t* __restrict__ slabs, double r, StreamOut o) {
    __shared__ double lvx[kEvalLdsVerts];
    __shared__ double lvy[kEvalLdsVerts];
    __shared__ ring_id_t lvr[kEvalLdsVerts];
    __shared__ float4 lsb[kEvalLdsVerts];
    __shared__ uint16_t lsl[kEvalLdsSlab];
    __shared__ uint2 pbuf[kTB / kWave][kEvalPairs];
    __shared__ double lqx[kCandItem], lqy[kCandItem];
    __shared__ unsigned lqi[kCandItem];
    __shared__ unsigned scnt[64];
    constexpr unsigned kPer = kCandItem / kTB;
    const int wid = threadIdx.x / kWave, lane = lane_id();
    uint2* pb = pbuf[wid];
    unsigned pc = 0;
    const unsigned ni = *c.nitems;
    __shared__ unsigned s_it;
    for (bool first = true;; first = false) {
        // items claimed in order: block b's first is item b, the rest from a ticket -- a block
        // done with a short item takes the next (a static stride gave the blocks with two long
        // items the whole pass's tail; a ticket for the first items too queued every block's
        // start behind one counter)
        __syncthreads();  // the previous item's LDS reads are done
        if (threadIdx.x == 0) s_it = first ? blockIdx.x : gridDim.x + atomicAdd(c.eticket, 1u);
        __syncthreads();
        const unsigned it = (unsigned)__builtin_amdgcn_readfirstlane((int)s_it);
        if (it >= ni) break;
        const uint4 w = c.items[it];
        const unsigned poly = w.x, m = w.z - w.y;
        const PolyDev P = polys[poly];
        const bool v_lds = P.nv <= (uint32_t)kEvalLdsVerts;
        const bool s_lds = P.llen <= (uint32_t)kEvalLdsSlab;
        const bool holes = P.nring > 1;
        if (v_lds)
            for (uint32_t t = threadIdx.x; t < P.nv; t += kTB) {
                lvx[t] = vx[P.voff + t];
                lvy[t] = vy[P.voff + t];
                if (holes) lvr[t] = vring[P.voff + t];
                else lsb[t] = seg_box32(vx + P.voff, vy + P.voff, t, P.nv, P.gb[0], P.gb[1]);
            }
        if (s_lds)
            for (uint32_t t = threadIdx.x; t < P.llen; t += kTB) lsl[t] = slabs[P.loff + t];
        if (threadIdx.x < 64) scnt[threadIdx.x] = 0;
        // the slice (<= kCandItem) in registers, its slab histogram in LDS
        double qx[kPer], qy[kPer];
        unsigned qi[kPer], qs[kPer];
        // slot indices for every u first, then every record, then the slabs: two global round
        // trips per item instead of two per u (a load under a branch made the compiler wait for it
        // before issuing the next); lanes past the slice read the item's first slot
        unsigned sid[kPer];
#pragma unroll
        for (unsigned u = 0; u < kPer; u++) {
            const unsigned t = threadIdx.x + u * kTB;
            sid[u] = c.sidx[w.y + (t < m ? t : 0u)];
        }
        double4 rcs[kPer];
#pragma unroll
        for (unsigned u = 0; u < kPer; u++) rcs[u] = c.crec[sid[u]];
#pragma unroll
        for (unsigned u = 0; u < kPer; u++) {
            const unsigned t = threadIdx.x + u * kTB;
            qs[u] = 0;
            qx[u] = rcs[u].x;
            qy[u] = rcs[u].y;
            qi[u] = (unsigned)__double_as_longlong(rcs[u].z);
            if (t < m && P.ns) qs[u] = slab_of(qy[u], P.sy0, P.sinv, P.ns);
        }
        __syncthreads();
#pragma unroll
        for (unsigned u = 0; u < kPer; u++)
            if (threadIdx.x + u * kTB < m) atomicAdd(&scnt[qs[u]], 1u);
        __syncthreads();
        if (threadIdx.x < kWave) {  // exclusive scan of the 64 bins: slab starts
            const unsigned v = scnt[threadIdx.x];
            scnt[threadIdx.x] = wave_incl_scan(v) - v;
        }
        __syncthreads();
#pragma unroll
        for (unsigned u = 0; u < kPer; u++)
            if (threadIdx.x + u * kTB < m) {
                const unsigned at = atomicAdd(&scnt[qs[u]], 1u);
                lqx[at] = qx[u];
                lqy[at] = qy[u];
                lqi[at] = qi[u];
            }
        __syncthreads();
        const double* rvx = v_lds ? lvx : vx + P.voff;
        const double* rvy = v_lds ? lvy : vy + P.voff;
        const ring_id_t* rvr = v_lds ? lvr : vring + P.voff;
        const double* rre = renv + 4 * (size_t)P.eoff;
        const SlabView sv{s_lds ? lsl : slabs + P.loff, P.ns};
        for (unsigned b = (unsigned)wid * kWave; b < m; b += kTB) {
            const unsigned i = b + (unsigned)lane;
            bool in = false;
            unsigned pid = 0;
            if (i < m) {
                const double px = lqx[i], py = lqy[i];
                pid = lqi[i];
                in = holes ? point_polygon_within_rings(px, py, rvx, rvy, rvr, rre, P, sv, r)
                           : point_polygon_within(px, py, rvx, rvy, P, sv, r, v_lds ? lsb : nullptr);
            }
            spairs_push<kEvalPairs>(pb, pc, in, poly, pid, o);
        }
    }
    if (pc) spairs_flush(pb, pc, o);
}

// ============================================================ point-polygon kNN ===========
// PointPolygonKNNQuery window body (PointPolygonKNNQuery.java:162-236): candidates = points of
// the polygon's G u C cells; key = (distance bits, window index), distance = JTS
// point.distance(polygon) (DistanceFunctions.java:33-36) or the bbox distance when approximate
// (DistanceFunctions.java:150-200); result = the k smallest keys, ascending (the deterministic
// form of the per-cell heaps + windowAll merge, KNNQuery.java:204-272).
//   ppknn_scan    one pass over x/y: cell (HelperClass.java:104-116) vs the G/C rects; candidate
//                 window indices compacted per wave (one atomic per wave)
//   ppknn_dist    full waves over the compact list: ring in LDS, exact distance, key
//   rsel_hist/_pick  radix select of the k-th smallest 96-bit key (dist bits | idx), 12-bit
//                 digits, 9 rounds; device-resident state, no host round trip
//   rsel_gather   keys <= the k-th key (exactly min(k, M) of them)
//   rsel_sort     one block: bitonic sort of <= 256 keys, emit idx / dist / count
constexpr int kRselBins = 4096;
constexpr int kRselRounds = 9;
struct RselState {
    unsigned long long pd, md;  // decided distance bits and their mask
    unsigned pi, mi;            // decided index bits and their mask
    unsigned kk;                // rank still to find among the matching keys (1-based)
    unsigned nsel;              // gather cursor
    unsigned ncand;             // candidates (scan counter)
    unsigned small_max;         // rsel_small handles ncand <= small_max
    unsigned hist[kRselBins];
    unsigned hist0[kRselBins];  // round-0 digits (distance bits 63..52) of every key, by ppknn_dist
};
// digit (field, shift, width) of round t: distance bits 63..0, then index bits 31..0
__host__ __device__ __forceinline__ void rsel_round(int t, int& field, int& shift, int& width) {
    const int sh[kRselRounds] = {52, 40, 28, 16, 4, 0, 20, 8, 0};
    const int wd[kRselRounds] = {12, 12, 12, 12, 12, 4, 12, 12, 8};
    field = t < 6 ? 0 : 1;
    shift = sh[t];
    width = wd[t];
}

// Distance.pointToSegment (JTS), fp64 in Java source order
__device__ __forceinline__ double point_segment(double px, double py, double ax, double ay, double bx, double by) {
    if (ax == bx && ay == by) return coord_distance(px, py, ax, ay);
    const double len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay);
    const double rr = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2;
    if (rr <= 0.0) return coord_distance(px, py, ax, ay);
    if (rr >= 1.0) return coord_distance(px, py, bx, by);
    const double s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2;
    return __builtin_fabs(s) * __builtin_sqrt(len2);
}

// JTS DistanceOp(point, polygon).distance(): 0 unless EXTERIOR (PointLocator: envelope test, then
// RayCrossingCounter over the ring), else min over segments (start Double.MAX_VALUE, replaced
// only by a strictly smaller value -- a NaN segment distance never is).
__device__ double point_polygon_distance(double px, double py, const double* __restrict__ vx,
                                         const double* __restrict__ vy, int nv, const double bb[4]) {
    const bool in_env = !(px > bb[2] || px < bb[0] || py > bb[3] || py < bb[1]);
    if (in_env) {
        bool boundary = false;
        int crossings = 0;
        for (int i = 1; i < nv; i++) count_segment(px, py, vx[i], vy[i], vx[i - 1], vy[i - 1], boundary, crossings);
        if (boundary || (crossings & 1)) return 0.0;
    }
    double md = 1.7976931348623157e308;
    for (int i = 0; i < nv - 1; i++) {
        const double d = point_segment(px, py, vx[i], vy[i], vx[i + 1], vy[i + 1]);
        md = d < md ? d : md;
    }
    return md;
}

// LDS histogram increment; the lanes holding the first active lane's digit add with one atomic
// (digits concentrate: distance 0 inside the polygon, shared exponents)
__device__ __forceinline__ void hist_add(unsigned* h, unsigned dg) {
    const unsigned first = __builtin_amdgcn_readfirstlane(dg);
    const unsigned long long same = __ballot(dg == first);
    if (dg != first) atomicAdd(&h[dg], 1u);
    else if (lanes_below(same) == 0) atomicAdd(&h[first], (unsigned)__popcll(same));
}

struct PpknnPoly {
    double bb[4];
    uint32_t nv, nrect;  // closed rings' total length; G rects then C rects (cell space)
    uint32_t nring, pad;  // rings (shell first); > 1: ring ids per vertex + ring envelopes
};

__global__ __launch_bounds__(1024) void rsel_init(RselState* __restrict__ st, unsigned k, unsigned small_max) {
    for (int t = threadIdx.x; t < kRselBins; t += 1024) {
        st->hist[t] = 0;
        st->hist0[t] = 0;
    }
    if (threadIdx.x == 0) {
        st->pd = 0; st->md = 0; st->pi = 0; st->mi = 0;
        st->kk = k; st->nsel = 0; st->ncand = 0; st->small_max = small_max;
    }
}

__global__ __launch_bounds__(kTB) void ppknn_scan(const double* __restrict__ x, const double* __restrict__ y,
                                                  uint64_t n, double mnx, double mny, double l,
                                                  const int32_t* __restrict__ rects, uint32_t nrect,
                                                  unsigned* __restrict__ cand, RselState* __restrict__ st) {
    __shared__ int32_t lr[4 * 64];
    const uint32_t nr = nrect < 64 ? nrect : 64;
    for (uint32_t t = threadIdx.x; t < 4 * nr; t += kTB) lr[t] = rects[t];
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kTB;
    for (uint64_t b = (uint64_t)blockIdx.x * kTB; b < n; b += stride) {
        const uint64_t i = b + threadIdx.x;
        bool c = false;
        if (i < n) {
            const int32_t cx = d_axis_cell(x[i], mnx, l), cy = d_axis_cell(y[i], mny, l);
            c = in_rects(lr, nr, cx, cy) || (nrect > nr && in_rects(rects + 4 * nr, nrect - nr, cx, cy));
        }
        const unsigned long long m = __ballot(c);
        if (m == 0) continue;
        unsigned base = 0;
        if (lane_id() == 0) base = atomicAdd(&st->ncand, (unsigned)__popcll(m));
        base = __shfl(base, 0);
        if (c) cand[base + lanes_below(m)] = (unsigned)i;
    }
}

// G u C rects as exact coordinate boxes (planner: rect_to_box), classification by compares
constexpr int kPpBoxes = kMaxPointBoxes + 1;  // a point plan's G u C boxes fit too
constexpr unsigned kPpBuf = 1024;  // wave-private candidate buffer (u32 window indices)
struct PpknnBoxes {
    Box b[kPpBoxes];
    int32_t nb, pad;
};

// 4 points per lane per 256-point wave iteration (double2 loads of x and y, the next full
// iteration's loads in flight while the current one is classified; the partial last iteration
// is handled after the loop so the main loop has one load path and the compiler's vmcnt
// accounting keeps the prefetch in flight).  NB > 0: the boxes are wave-uniform registers;
// NB == 0: any count, read from LDS.  One atomic per wave-iteration with candidates.
// Candidate order in `cand` is irrelevant (the select keys carry the window index).
template <int NB>
__global__ __launch_bounds__(kTB) void ppknn_scan_boxes(const double* __restrict__ x, const double* __restrict__ y,
                                                        uint64_t n, PpknnBoxes B, unsigned* __restrict__ cand,
                                                        RselState* __restrict__ st) {
    __shared__ Box lb[NB == 0 ? kPpBoxes : 1];
    __shared__ unsigned wbuf[kTB / kWave][kPpBuf];
    const int lane = lane_id();
    Box rb[NB > 0 ? NB : 1];
    if (NB > 0) {
#pragma unroll
        for (int b = 0; b < (NB > 0 ? NB : 1); b++) rb[b] = B.b[b];
    } else {
        if (threadIdx.x < (unsigned)B.nb) lb[threadIdx.x] = B.b[threadIdx.x];
        __syncthreads();
    }
    auto cls = [&](double px, double py) {
        bool c = false;
        if (NB > 0) {
#pragma unroll
            for (int b = 0; b < (NB > 0 ? NB : 1); b++) c = c || in_box(rb[b], px, py);
        } else {
            for (int b = 0; b < B.nb; b++) c = c || in_box(lb[b], px, py);
        }
        return c;
    };
    // block b streams iterations [b per, (b + 1) per); its 4 waves interleave inside the chunk
    const uint64_t all_iters = (n + 255) / 256, full_iters = n / 256;
    const uint64_t per = (all_iters + gridDim.x - 1) / gridDim.x;
    const uint64_t blk_end = (uint64_t)(blockIdx.x + 1) * per;
    const uint64_t end = blk_end < all_iters ? blk_end : all_iters;
    const uint64_t fend = end < full_iters ? end : full_iters;
    const unsigned wid = threadIdx.x / kWave;
    // candidates gather in a wave-private LDS buffer and leave with one global atomic per
    // kPpBuf entries (the candidate points are scattered over the window: one atomic per
    // wave-iteration serialises ~10^5 atomics on one address, ~400 us for the C4 window)
    const int wslot = threadIdx.x / kWave;
    unsigned* buf = wbuf[wslot];
    unsigned cnt = 0;
    auto flush = [&]() {
        wave_lds_sync();
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(&st->ncand, cnt);
        base = __shfl(base, 0);
        for (unsigned q = lane; q < cnt; q += kWave) cand[base + q] = buf[q];
        wave_lds_sync();
        cnt = 0;
    };
    auto emit = [&](uint64_t it, const bool c[4]) {
        const uint64_t b0 = it * 256;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const unsigned long long m = __ballot(c[s]);
            if ((m >> lane) & 1ull) buf[cnt + lanes_below(m)] = (unsigned)(b0 + (s >> 1) * 128 + 2 * lane + (s & 1));
            cnt += (unsigned)__popcll(m);
        }
        if (cnt > kPpBuf - 256) flush();
    };
    auto load_full = [&](uint64_t it, double2 v[4]) {
        const uint64_t i0 = it * 256 + 2 * (uint64_t)lane;
        // read once here (ppknn_dist gathers only the candidates): past the caches (same box, 3
        // reps: scan 184 -> 170 us against plain loads)
        typedef double d2v __attribute__((ext_vector_type(2)));
        const uint64_t io[4] = {i0, i0 + 128, i0, i0 + 128};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const d2v w = __builtin_nontemporal_load(reinterpret_cast<const d2v*>((u < 2 ? x : y) + io[u]));
            v[u] = make_double2(w.x, w.y);
        }
    };
    uint64_t it = (uint64_t)blockIdx.x * per + wid;
    double2 cur[4], nxt[4];
    if (it < fend) load_full(it, cur);
    for (; it < fend; it += kTB / kWave) {
        const uint64_t nit = it + kTB / kWave;
        if (nit < fend) load_full(nit, nxt);
        const bool c[4] = {cls(cur[0].x, cur[2].x), cls(cur[0].y, cur[2].y), cls(cur[1].x, cur[3].x),
                           cls(cur[1].y, cur[3].y)};
        emit(it, c);
#pragma unroll
        for (int q = 0; q < 4; q++) cur[q] = nxt[q];
    }
    // the partial last iteration of the window (at most one, in the last chunk)
    if (it < end && it == full_iters) {
        const uint64_t i0 = it * 256 + 2 * (uint64_t)lane;
        const bool v0 = i0 < n, v1 = i0 + 1 < n, v2 = i0 + 128 < n, v3 = i0 + 129 < n;
        const double x0 = v0 ? x[i0] : 0.0, y0 = v0 ? y[i0] : 0.0;
        const double x1 = v1 ? x[i0 + 1] : 0.0, y1 = v1 ? y[i0 + 1] : 0.0;
        const double x2 = v2 ? x[i0 + 128] : 0.0, y2 = v2 ? y[i0 + 128] : 0.0;
        const double x3 = v3 ? x[i0 + 129] : 0.0, y3 = v3 ? y[i0 + 129] : 0.0;
        const bool c0 = cls(x0, y0), c1 = cls(x1, y1), c2 = cls(x2, y2), c3 = cls(x3, y3);
        const bool c[4] = {v0 && c0, v1 && c1, v2 && c2, v3 && c3};
        emit(it, c);
    }
    if (cnt) flush();
}

template <bool APPROX>
__global__ __launch_bounds__(kTB) void ppknn_dist(const double* __restrict__ x, const double* __restrict__ y,
                                                  const unsigned* __restrict__ cand, RselState* __restrict__ st,
                                                  const double* __restrict__ vx, const double* __restrict__ vy,
                                                  const ring_id_t* __restrict__ vring, const double* __restrict__ renv,
                                                  PpknnPoly P, unsigned long long* __restrict__ key) {
    __shared__ double lvx[kMaxLdsVerts];
    __shared__ double lvy[kMaxLdsVerts];
    __shared__ ring_id_t lvr[kMaxLdsVerts];
    __shared__ unsigned lh[kRselBins];  // round-0 digits of this block's keys (-> st->hist0)
    for (int t = threadIdx.x; t < kRselBins; t += kTB) lh[t] = 0;
    const bool v_lds = P.nv <= (uint32_t)kMaxLdsVerts;
    const bool holes = P.nring > 1;
    if (!APPROX && v_lds)
        for (uint32_t t = threadIdx.x; t < P.nv; t += kTB) {
            lvx[t] = vx[t];
            lvy[t] = vy[t];
            if (holes) lvr[t] = vring[t];
        }
    __syncthreads();
    const double* rvx = v_lds ? lvx : vx;
    const double* rvy = v_lds ? lvy : vy;
    const ring_id_t* rvr = v_lds ? lvr : vring;
    const unsigned m = st->ncand;
    if (APPROX) {
        for (unsigned t = blockIdx.x * kTB + threadIdx.x; t < m; t += gridDim.x * kTB) {
            const unsigned i = cand[t];
            const double d = bbox_distance(x[i], y[i], P.bb);
            unsigned long long bits = (unsigned long long)__double_as_longlong(d);
            if (d != d) bits = 0x7ff8000000000000ull;
            key[t] = bits;
            hist_add(lh, (unsigned)(bits >> 52));
        }
        __syncthreads();
        for (int b = threadIdx.x; b < kRselBins; b += kTB)
            if (lh[b]) atomicAdd(&st->hist0[b], lh[b]);
        return;
    }
    // exact (point_polygon_distance split over 8 lanes per candidate, each taking every 8th
    // segment): crossings summed, boundary OR-ed, segment minima combined -- min is
    // order-independent here, as no partial minimum is NaN (each starts at Double.MAX_VALUE and
    // takes only strictly smaller values)
    constexpr unsigned kG = 8;
    const unsigned sub = threadIdx.x % kG;
    const int nv = (int)P.nv;
    for (unsigned t0 = (blockIdx.x * kTB + threadIdx.x) / kG; t0 < m; t0 += gridDim.x * (kTB / kG)) {
        const unsigned i = cand[t0];
        const double px = x[i], py = y[i];
        const bool in_env = !(px > P.bb[2] || px < P.bb[0] || py > P.bb[3] || py < P.bb[1]);
        bool boundary = false;
        int crossings = 0;
        double md = 1.7976931348623157e308;
        double d;
        if (!holes) {
            for (int e = (int)sub; e < nv - 1; e += (int)kG) {
                const double ax = rvx[e], ay = rvy[e], bx = rvx[e + 1], by = rvy[e + 1];
                if (in_env) count_segment(px, py, bx, by, ax, ay, boundary, crossings);
                const double sd = point_segment(px, py, ax, ay, bx, by);
                md = sd < md ? sd : md;
            }
#pragma unroll
            for (unsigned o = 1; o < kG; o <<= 1) {
                crossings += __shfl_xor(crossings, (int)o);
                boundary = (__shfl_xor((int)boundary, (int)o) != 0) || boundary;
                const double od = __shfl_xor(md, (int)o);
                md = od < md ? od : md;
            }
            d = (in_env && (boundary || (crossings & 1))) ? 0.0 : md;
        } else {
            // per-ring boundary / parity masks (rings_locate_chunk); the minimum covers every
            // ring's segments (DistanceOp's envelope skip drops only rings farther than the
            // running minimum)
            for (int e = (int)sub; e < nv - 1; e += (int)kG) {
                if (rvr[e] != rvr[e + 1]) continue;  // junction between two rings
                const double sd = point_segment(px, py, rvx[e], rvy[e], rvx[e + 1], rvy[e + 1]);
                md = sd < md ? sd : md;
            }
#pragma unroll
            for (unsigned o = 1; o < kG; o <<= 1) {
                const double od = __shfl_xor(md, (int)o);
                md = od < md ? od : md;
            }
            int loc = in_env ? -1 : 0;  // the 8 lanes of a candidate decide together
            const uint32_t nch = (P.nring + 63) / 64;
            for (uint32_t c = 0; c < nch && loc < 0; c++) {
                unsigned long long bnd = 0, par = 0;
                for (int e = (int)sub; e < nv - 1; e += (int)kG) {
                    const unsigned rid = rvr[e];
                    if (rid != rvr[e + 1] || (rid >> 6) != c) continue;
                    bool b = false;
                    int cr = 0;
                    count_segment(px, py, rvx[e + 1], rvy[e + 1], rvx[e], rvy[e], b, cr);
                    bnd |= b ? 1ull << (rid & 63) : 0ull;
                    par ^= (cr & 1) ? 1ull << (rid & 63) : 0ull;
                }
#pragma unroll
                for (unsigned o = 1; o < kG; o <<= 1) {
                    bnd |= __shfl_xor(bnd, (int)o);
                    par ^= __shfl_xor(par, (int)o);
                }
                loc = rings_locate_chunk(px, py, bnd, par, renv, c);
            }
            d = loc != 0 ? 0.0 : md;
        }
        if (sub == 0) {
            const unsigned long long bits = (unsigned long long)__double_as_longlong(d);
            key[t0] = bits;
            hist_add(lh, (unsigned)(bits >> 52));
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kRselBins; b += kTB)
        if (lh[b]) atomicAdd(&st->hist0[b], lh[b]);
}

__device__ __forceinline__ bool rsel_match(const RselState& s, unsigned long long d, unsigned i) {
    return (d & s.md) == s.pd && (i & s.mi) == s.pi;
}

// candidate counts up to this are selected by one workgroup (rsel_small); the multi-block
// rounds below are no-ops then
constexpr unsigned kRselSmall = 1u << 17;

__global__ __launch_bounds__(kTB) void rsel_hist(const unsigned long long* __restrict__ key,
                                                 const unsigned* __restrict__ cand, RselState* __restrict__ st,
                                                 int round, unsigned k) {
    __shared__ unsigned h[kRselBins];
    const unsigned m = st->ncand;
    if (m <= k || m <= st->small_max) return;  // every candidate is selected / rsel_small did it
    for (int t = threadIdx.x; t < kRselBins; t += kTB) h[t] = 0;
    __syncthreads();
    int field, shift, width;
    rsel_round(round, field, shift, width);
    const unsigned long long md = st->md, pd = st->pd;
    const unsigned mi = st->mi, pi = st->pi;
    const unsigned dm = (1u << width) - 1u;
    for (unsigned t = blockIdx.x * kTB + threadIdx.x; t < m; t += gridDim.x * kTB) {
        const unsigned long long d = key[t];
        const unsigned i = cand[t];
        if ((d & md) != pd || (i & mi) != pi) continue;
        const unsigned dg = field == 0 ? (unsigned)(d >> shift) & dm : (i >> shift) & dm;
        atomicAdd(&h[dg], 1u);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < kRselBins; t += kTB)
        if (h[t]) atomicAdd(&st->hist[t], h[t]);
}

__global__ __launch_bounds__(1024) void rsel_pick(RselState* __restrict__ st, int round, unsigned k) {
    __shared__ unsigned part[1024];
    const unsigned m = st->ncand;
    if (m <= st->small_max) return;
    if (m <= k) {  // select all: the k-th key is the maximum
        if (threadIdx.x == 0) {
            st->md = 0; st->pd = 0; st->mi = 0; st->pi = 0;
        }
        return;
    }
    int field, shift, width;
    rsel_round(round, field, shift, width);
    // 4 bins per thread, inclusive scan of the per-thread sums
    unsigned v[4], sum = 0;
    for (int j = 0; j < 4; j++) {
        v[j] = st->hist[4 * threadIdx.x + j];
        sum += v[j];
    }
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const unsigned a = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += a;
        __syncthreads();
    }
    const unsigned kk = st->kk;
    const unsigned incl = part[threadIdx.x], excl = incl - sum;
    __syncthreads();  // every thread has read kk before it changes
    if (excl < kk && incl >= kk) {  // exactly one thread holds the k-th
        unsigned c = excl;
        int j = 0;
        while (c + v[j] < kk) c += v[j++];
        const unsigned dg = 4 * threadIdx.x + j;
        st->kk = kk - c;
        const unsigned dm = (1u << width) - 1u;
        if (field == 0) {
            st->pd |= (unsigned long long)dg << shift;
            st->md |= (unsigned long long)dm << shift;
        } else {
            st->pi |= dg << shift;
            st->mi |= dm << shift;
        }
    }
    for (int j = 0; j < 4; j++) st->hist[4 * threadIdx.x + j] = 0;
}

__global__ __launch_bounds__(kTB) void rsel_gather(const unsigned long long* __restrict__ key,
                                                   const unsigned* __restrict__ cand, RselState* __restrict__ st,
                                                   unsigned k, unsigned long long* __restrict__ sel_d,
                                                   unsigned* __restrict__ sel_i) {
    const unsigned m = st->ncand;
    if (m <= st->small_max) return;
    const bool all = m <= k;
    const unsigned long long kd = st->pd;
    const unsigned ki = st->pi;
    for (unsigned t = blockIdx.x * kTB + threadIdx.x; t < m; t += gridDim.x * kTB) {
        const unsigned long long d = key[t];
        const unsigned i = cand[t];
        if (all || d < kd || (d == kd && i <= ki)) {
            const unsigned s = atomicAdd(&st->nsel, 1u);
            if (s < k) {
                sel_d[s] = d;
                sel_i[s] = i;
            }
        }
    }
}

// slot of this lane among the wave's active lanes in a counter (one atomic per wave)
__device__ __forceinline__ unsigned wave_reserve(unsigned* ctr) {
    const unsigned long long m = __ballot(1);
    const int lead = __builtin_ctzll(m);
    unsigned b = 0;
    if (lane_id() == lead) b = atomicAdd(ctr, (unsigned)__popcll(m));
    b = __shfl(b, lead);
    return b + lanes_below(m);
}

// One workgroup, M <= kRselSmall candidates (L2-resident keys): the 9 radix rounds with an LDS
// histogram, the gather and the sort, in one launch.  Once the keys still matching the decided
// prefix fit kCompact, they are copied into LDS and the later rounds no longer read L2 (one CU
// streams ~64 B/clk: each full pass over 10^5 keys costs ~5 us).
constexpr unsigned kCompact = 10240;
__global__ __launch_bounds__(1024) void rsel_small(const unsigned long long* __restrict__ key,
                                                   const unsigned* __restrict__ cand, const RselState* __restrict__ st,
                                                   unsigned k, double* __restrict__ out_d, unsigned* __restrict__ out_i,
                                                   unsigned* __restrict__ out_count) {
    __shared__ unsigned h[kRselBins];
    __shared__ unsigned part[64];
    __shared__ unsigned long long sd[256];
    __shared__ unsigned si[256];
    __shared__ unsigned long long cd[kCompact];
    __shared__ unsigned ci[kCompact];
    __shared__ unsigned long long s_pd, s_md;
    __shared__ unsigned s_pi, s_mi, s_kk, s_nsel, s_cnt, s_lds, s_lcnt;
    __shared__ unsigned long long s_and_d, s_or_d;  // over the LDS keys matching the prefix
    __shared__ unsigned s_and_i, s_or_i;
    const unsigned m = st->ncand;
    if (m > st->small_max) return;
    const unsigned t = threadIdx.x;
    if (t == 0) {
        s_pd = 0; s_md = 0; s_pi = 0; s_mi = 0; s_kk = k; s_nsel = 0; s_cnt = m; s_lds = 0; s_lcnt = 0;
    }
    __syncthreads();
    const bool all = m <= k;
    // visit every key of the current source (global list or the LDS copy) matching the prefix
    auto for_matching = [&](auto&& fn) {
        const unsigned long long md = s_md, pd = s_pd;
        const unsigned mi = s_mi, pi = s_pi;
        if (s_lds) {
            const unsigned cnt = s_lcnt;  // entries of the LDS copy
            for (unsigned c = t; c < cnt; c += 1024) {
                const unsigned long long d = cd[c];
                const unsigned i = ci[c];
                if ((d & md) == pd && (i & mi) == pi) fn(d, i);
            }
            return;
        }
        for (unsigned c0 = t; c0 < m; c0 += 4 * 1024) {  // 4 independent loads per thread in flight
            unsigned long long d[4];
            unsigned i[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const unsigned c = c0 + u * 1024;
                d[u] = c < m ? key[c] : ~0ull;
                i[u] = c < m ? cand[c] : ~0u;
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (c0 + u * 1024 < m && (d[u] & md) == pd && (i[u] & mi) == pi) fn(d[u], i[u]);
        }
    };
    bool pre = false;  // keys below the round-0 digit were selected outright (LDS-only rounds)
    bool andor_ok = false;  // s_and_* / s_or_* hold the current matching set's AND / OR (block-uniform)
    for (int round = 0; round < kRselRounds && !all; round++) {
        int field, shift, width;
        rsel_round(round, field, shift, width);
        const unsigned dm = (1u << width) - 1u;
        if (round > 0 && s_lds && andor_ok) {
            // the matching set is unchanged since the last AND/OR pass: its digits of this round
            // are already known (uniform -> taken below without a pass)
        } else if (round > 0 && s_lds) {
            // a round whose digit every matching key shares decides nothing: take it without a
            // histogram (keys at distance 0 inside the polygon skip all the distance rounds)
            if (t == 0) {
                s_and_d = ~0ull; s_or_d = 0; s_and_i = ~0u; s_or_i = 0;
            }
            __syncthreads();
            const unsigned long long md = s_md, pd = s_pd;
            const unsigned mi = s_mi, pi = s_pi, cnt = s_lcnt;
            unsigned long long ad = ~0ull, od = 0;
            unsigned ai = ~0u, oi = 0;
            for (unsigned c = t; c < cnt; c += 1024) {
                const unsigned long long d = cd[c];
                const unsigned i = ci[c];
                if ((d & md) == pd && (i & mi) == pi) {
                    ad &= d; od |= d; ai &= i; oi |= i;
                }
            }
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                ad &= xor_lane64(ad, o);
                od |= xor_lane64(od, o);
                ai &= xor_lane(ai, o);
                oi |= xor_lane(oi, o);
            }
            if (lane_id() == 0) {
                atomicAnd(&s_and_d, ad);
                atomicOr(&s_or_d, od);
                atomicAnd(&s_and_i, ai);
                atomicOr(&s_or_i, oi);
            }
            __syncthreads();
            andor_ok = true;
        }
        if (round > 0 && s_lds) {
            const unsigned a = field == 0 ? (unsigned)(s_and_d >> shift) & dm : (s_and_i >> shift) & dm;
            const unsigned b = field == 0 ? (unsigned)(s_or_d >> shift) & dm : (s_or_i >> shift) & dm;
            __syncthreads();
            if (a == b) {  // uniform: every thread read the same shared words
                if (t == 0) {
                    if (field == 0) {
                        s_pd |= (unsigned long long)a << shift;
                        s_md |= (unsigned long long)dm << shift;
                    } else {
                        s_pi |= a << shift;
                        s_mi |= dm << shift;
                    }
                }
                __syncthreads();
                continue;
            }
        }
        andor_ok = false;  // a histogram round narrows the matching set
        if (round == 0) {  // the producers' histogram (ppknn_dist) of the round-0 digits
            for (int b = t; b < kRselBins; b += 1024) h[b] = st->hist0[b];
        } else {
            for (int b = t; b < kRselBins; b += 1024) h[b] = 0;
            __syncthreads();
            for_matching([&](unsigned long long d, unsigned i) {
                hist_add(h, field == 0 ? (unsigned)(d >> shift) & dm : (i >> shift) & dm);
            });
        }
        __syncthreads();
        unsigned v[4], sum = 0;
        for (int j = 0; j < 4; j++) {
            v[j] = h[4 * t + j];
            sum += v[j];
        }
        // block inclusive scan of the per-thread sums: DPP within waves, then 16 wave totals
        const unsigned winc = wave_incl_scan(sum);
        if (lane_id() == kWave - 1) part[t / kWave] = winc;
        __syncthreads();
        unsigned wbase = 0;
        for (unsigned w = 0; w < t / kWave; w++) wbase += part[w];
        const unsigned kk = s_kk;
        const unsigned incl = wbase + winc, excl = incl - sum;
        __syncthreads();
        if (excl < kk && incl >= kk) {
            unsigned c = excl;
            int j = 0;
            while (c + v[j] < kk) c += v[j++];
            const unsigned dg = 4 * t + j;
            s_kk = kk - c;
            s_cnt = v[j];  // keys matching the extended prefix
            if (field == 0) {
                s_pd |= (unsigned long long)dg << shift;
                s_md |= (unsigned long long)dm << shift;
            } else {
                s_pi |= dg << shift;
                s_mi |= dm << shift;
            }
        }
        __syncthreads();
        if (round == 0 && s_cnt <= kCompact) {
            // one pass over the list: keys below the chosen digit are among the k smallest
            // (fewer than k of them), the digit's keys move into LDS for the later rounds
            const unsigned d0 = (unsigned)(s_pd >> 52);
            for (unsigned c0 = t; c0 < m; c0 += 4 * 1024) {
                unsigned long long d[4];
                unsigned i[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const unsigned c = c0 + u * 1024;
                    d[u] = c < m ? key[c] : ~0ull;
                    i[u] = c < m ? cand[c] : ~0u;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (c0 + u * 1024 >= m) continue;
                    const unsigned dg = (unsigned)(d[u] >> 52);
                    if (dg < d0) {
                        const unsigned sl = wave_reserve(&s_nsel);
                        sd[sl] = d[u];
                        si[sl] = i[u];
                    } else if (dg == d0) {
                        const unsigned sl = wave_reserve(&s_lcnt);
                        cd[sl] = d[u];
                        ci[sl] = i[u];
                    }
                }
            }
            __syncthreads();
            if (t == 0) s_lds = 1;
            pre = true;
            __syncthreads();
        }
        if (!s_lds && s_cnt <= kCompact && round + 1 < kRselRounds) {  // move the survivors into LDS
            if (t == 0) s_nsel = 0;
            __syncthreads();
            for_matching([&](unsigned long long d, unsigned i) {
                const unsigned sl = wave_reserve(&s_nsel);
                cd[sl] = d;
                ci[sl] = i;
            });
            __syncthreads();
            if (t == 0) {
                s_lds = 1;
                s_lcnt = s_nsel;
                s_nsel = 0;
            }
            __syncthreads();
        }
    }
    // keys <= the k-th key: all of the global list (M <= k), else the gather of the rounds'
    // prefix plus every key below it -- taken from the full global list
    const unsigned long long kd = s_pd;
    const unsigned ki = s_pi;
    if (pre) {  // the rest of the k smallest: the LDS copy's keys up to the k-th
        const unsigned cnt = s_lcnt;
        for (unsigned c = t; c < cnt; c += 1024) {
            const unsigned long long d = cd[c];
            const unsigned i = ci[c];
            if (d < kd || (d == kd && i <= ki)) {
                const unsigned sl = wave_reserve(&s_nsel);
                if (sl < 256) {
                    sd[sl] = d;
                    si[sl] = i;
                }
            }
        }
    } else {
        for (unsigned c = t; c < m; c += 1024) {
            const unsigned long long d = key[c];
            const unsigned i = cand[c];
            if (all || d < kd || (d == kd && i <= ki)) {
                const unsigned sl = wave_reserve(&s_nsel);
                if (sl < 256) {
                    sd[sl] = d;
                    si[sl] = i;
                }
            }
        }
    }
    __syncthreads();
    const unsigned ns = s_nsel < k ? s_nsel : k;
    if (t < 256 && t >= ns) {
        sd[t] = ~0ull;
        si[t] = ~0u;
    }
    __syncthreads();
    for (unsigned size = 2; size <= 256; size <<= 1) {
        for (unsigned j = size >> 1; j > 0; j >>= 1) {
            const unsigned p = t ^ j;
            if (t < 256 && p > t) {
                const bool up = (t & size) == 0;
                const bool gt = sd[t] > sd[p] || (sd[t] == sd[p] && si[t] > si[p]);
                if (gt == up) {
                    const unsigned long long td = sd[t]; sd[t] = sd[p]; sd[p] = td;
                    const unsigned ti = si[t]; si[t] = si[p]; si[p] = ti;
                }
            }
            __syncthreads();
        }
    }
    if (t < ns) {
        out_d[t] = __longlong_as_double((long long)sd[t]);
        out_i[t] = si[t];
    }
    if (t == 0) out_count[0] = ns;
}

__global__ __launch_bounds__(256) void rsel_sort(const unsigned long long* __restrict__ sel_d,
                                                 const unsigned* __restrict__ sel_i, const RselState* __restrict__ st,
                                                 unsigned k, double* __restrict__ out_d, unsigned* __restrict__ out_i,
                                                 unsigned* __restrict__ out_count) {
    __shared__ unsigned long long d[256];
    __shared__ unsigned id[256];
    if (st->ncand <= st->small_max) return;
    const unsigned m = st->nsel < k ? st->nsel : k;
    const unsigned t = threadIdx.x;
    d[t] = t < m ? sel_d[t] : ~0ull;
    id[t] = t < m ? sel_i[t] : ~0u;
    __syncthreads();
    for (unsigned size = 2; size <= 256; size <<= 1) {
        for (unsigned j = size >> 1; j > 0; j >>= 1) {
            const unsigned p = t ^ j;
            if (p > t) {
                const bool up = (t & size) == 0;
                const bool gt = d[t] > d[p] || (d[t] == d[p] && id[t] > id[p]);
                if (gt == up) {
                    const unsigned long long td = d[t]; d[t] = d[p]; d[p] = td;
                    const unsigned ti = id[t]; id[t] = id[p]; id[p] = ti;
                }
            }
            __syncthreads();
        }
    }
    if (t < m) {
        out_d[t] = __longlong_as_double((long long)d[t]);
        out_i[t] = id[t];
    }
    if (t == 0) out_count[0] = m;
}

// ---- large-k forms (k above what the one-workgroup selections rank in LDS) ----------------
// Point kNN keys: JTS point.distance of every candidate as raw bits, the order the one-pass kNN
// (knn_pass) ranks them in.
__global__ __launch_bounds__(kTB) void ppknn_pp_keys(const double* __restrict__ x, const double* __restrict__ y,
                                                     const unsigned* __restrict__ cand,
                                                     const RselState* __restrict__ st, double qx, double qy,
                                                     unsigned long long* __restrict__ key) {
    const unsigned m = st->ncand;
    for (unsigned t = blockIdx.x * kTB + threadIdx.x; t < m; t += gridDim.x * kTB) {
        const unsigned i = cand[t];
        key[t] = (unsigned long long)__double_as_longlong(jts_pp_distance(qx, qy, x[i], y[i]));
    }
}

// result count of a large-k selection: min(candidates, k)
__global__ void rsel_count(const RselState* __restrict__ st, unsigned k, unsigned* __restrict__ out_count) {
    if (threadIdx.x == 0) {
        const unsigned m = st->ncand;
        out_count[0] = m < k ? m : k;
    }
}

// the first k of m sorted (dist, idx) entries (sentinels sort last), the rest sentinels; count =
// real entries among them
__global__ __launch_bounds__(1024) void topk_take(const unsigned long long* __restrict__ sd,
                                                  const unsigned* __restrict__ si, unsigned m, unsigned k,
                                                  double* __restrict__ out_d, unsigned* __restrict__ out_i,
                                                  unsigned* __restrict__ out_count) {
    __shared__ unsigned cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    unsigned mine = 0;
    for (unsigned t = threadIdx.x; t < k; t += 1024) {
        const unsigned long long d = t < m ? sd[t] : kSentinelD;
        out_d[t] = __longlong_as_double((long long)d);
        out_i[t] = t < m ? si[t] : kSentinelI;
        mine += d != kSentinelD ? 1u : 0u;
    }
    if (mine) atomicAdd(&cnt, mine);
    __syncthreads();
    if (threadIdx.x == 0) out_count[0] = cnt;
}

// ================================================================== host side =============
namespace {

enum JSlot {
    J_HIST, J_TTOT, J_TSTART, J_SEG, J_SX, J_SY, J_SIDX, J_SKEY, J_MISC, J_AUX, J_POLY, J_OUT, J_RECT, J_QSTART,
    J_QLIST, J_GLIST, J_QCNT, J_BCNT, J_BOFF, J_PMASK, J_MWORDS, J_MOFF, J_TCUR,
    J_KCAND, J_KTEMP, J_KBLOB,  // point kNN (large k) and point-polygon kNN scratch
    J_COVF                      // point-polygon stream: per-wave overflow candidate lists
};
static_assert(J_COVF <= 27, "scratch slots (abi.cpp S_J0 .. S_J27)");

// J_MISC words: [0] outside count, [1] outside cursor, [2] scan grand total, [3] global
// query count, [8..9] pair total (u64)
constexpr int kMiscWords = 16;

struct Scratch {
    geohip_ctx* ctx;
    int rc = GEOHIP_OK;
    template <typename T>
    T* get(JSlot slot, size_t bytes) {
        void* p = nullptr;
        if (rc) return nullptr;
        rc = ctx_ensure(ctx, slot, bytes, &p);
        return reinterpret_cast<T*>(p);
    }
};

int check_grid_basic(geohip_ctx* ctx, const geohip_grid* g, const char* what) {
    if (!g) return ctx_fail(ctx, GEOHIP_ERR_ARG, std::string(what) + ": null grid");
    if (!(g->n > 0) || !(g->cell_len > 0) || !std::isfinite(g->cell_len) || !std::isfinite(g->min_x) ||
        !std::isfinite(g->min_y))
        return ctx_fail(ctx, GEOHIP_ERR_ARG, std::string(what) + ": invalid grid");
    if (g->n > 99999) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, std::string(what) + ": more than 99999 cells per side");
    return GEOHIP_OK;
}

TileGeom tile_geom(const geohip_grid& g, int32_t nb) {
    TileGeom t;
    t.mnx = g.min_x;
    t.mny = g.min_y;
    t.l = g.cell_len;
    t.il = 1.0 / g.cell_len;
    t.nb = nb;
    t.ts = (nb + 127) / 128;
    if (t.ts < 1) t.ts = 1;
    t.nt = (nb + t.ts - 1) / t.ts;
    t.ntiles = (uint32_t)t.nt * (uint32_t)t.nt;
    t.dts = make_fastdiv((unsigned)t.ts);
    t.dnb = make_fastdiv((unsigned)(nb > 0 ? nb : 1));
    return t;
}

// exclusive scan of in[0..n) into out[0..n] (out[n] = total) on the stream
template <typename T>
void scan_launch(hipStream_t st, const T* in, uint64_t n, T* seg, T* grand, T* out) {
    const uint64_t nseg = (n + kScanSeg - 1) / kScanSeg;
    const unsigned g = (unsigned)(nseg ? nseg : 1);
    scan_seg_totals<T><<<g, kTB, 0, st>>>(in, n, seg);
    scan_totals<T><<<1, kTB, 0, st>>>(seg, g, grand);
    scan_apply<T><<<g, kTB, 0, st>>>(in, n, seg, grand, out);
}

SoA carve_soa(void* base, uint64_t n) {
    char* p = reinterpret_cast<char*>(base);
    SoA o;
    o.x = reinterpret_cast<double*>(p);
    o.y = reinterpret_cast<double*>(p + 8 * n);
    o.idx = reinterpret_cast<unsigned*>(p + 16 * n);
    o.key = reinterpret_cast<unsigned*>(p + 20 * n);
    return o;
}

// Bin the window's points into tiles of `geo` (two local-sort levels, SoA copies in scratch).
// keep_outside: return the out-of-grid points' window indices (*outside_idx, count read back
// into *n_outside_host).
int bin_tiles(geohip_ctx* ctx, Scratch& S, const double* dx, const double* dy, uint64_t n, const TileGeom& geo,
              bool keep_outside, TileBins* tb, unsigned** outside_idx, unsigned* n_outside_host,
              const unsigned* keep = nullptr) {
    hipStream_t st = ctx_stream(ctx);
    uint64_t nblk = (n + 16383) / 16384;
    if (nblk > 256) nblk = 256;
    if (nblk < 1) nblk = 1;
    const uint64_t chunk = (n + nblk - 1) / nblk;
    const uint64_t nt = geo.ntiles;
    const unsigned nbands = (unsigned)((nt + kBandTiles - 1) / kBandTiles);
    const uint64_t maxitems = (n + kL2Items - 1) / kL2Items + nbands;
    unsigned* hist1 = S.get<unsigned>(J_HIST, nblk * (nbands + 2) * 4);
    unsigned* hist2 = S.get<unsigned>(J_SIDX, maxitems * kBandTiles * 4 + 16);
    uint4* items = S.get<uint4>(J_SKEY, maxitems * sizeof(uint4) + 16);
    unsigned* aux = S.get<unsigned>(J_AUX, (2 * (uint64_t)nbands + 8) * 4);  // start1 (nbands + 3) | wfirst
    unsigned* tot = S.get<unsigned>(J_TTOT, (nt + 1) * 4);
    unsigned* start = S.get<unsigned>(J_TSTART, (nt + 1) * 4);
    unsigned* seg = S.get<unsigned>(J_SEG, ((nt + kScanSeg - 1) / kScanSeg + 1) * 8 + 64);
    void* l1 = S.get<void>(J_SY, n * 24 + 64);
    void* l2 = S.get<void>(J_SX, n * 24 + 64);
    unsigned* misc = S.get<unsigned>(J_MISC, kMiscWords * 4);
    if (S.rc) return S.rc;
    if (hipMemsetAsync(misc, 0, kMiscWords * 4, st) != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    unsigned* start1 = aux;
    unsigned* wfirst = aux + nbands + 3;
    BinPass a;
    memset(&a, 0, sizeof a);
    a.x = dx;
    a.y = dy;
    a.src = carve_soa(l1, n);
    a.dst = a.src;
    a.n = n;
    a.chunk = chunk;
    a.g = geo;
    a.nbands = nbands;
    a.hist = hist1;
    a.nitems = misc + 4;
    a.keep = keep;
    a.keep_words = keep ? (unsigned)(((uint64_t)geo.nb * (uint64_t)geo.nb + 31) / 32) : 0u;
    // level 1: bands
    // (the keep bitmap in LDS when it fits: its per-point word reads are random gathers)
    if (keep && a.keep_words <= kKeepLds) {
        bin_count<1, true><<<(unsigned)nblk, kBinThreads, 0, st>>>(a);
        bin1_offsets<<<1, kTB, 0, st>>>(hist1, (unsigned)nblk, nbands + 2, start1);
        bin_scatter<1, true><<<(unsigned)nblk, kBinThreads, 0, st>>>(a);
    } else {
        bin_count<1><<<(unsigned)nblk, kBinThreads, 0, st>>>(a);
        bin1_offsets<<<1, kTB, 0, st>>>(hist1, (unsigned)nblk, nbands + 2, start1);
        bin_scatter<1><<<(unsigned)nblk, kBinThreads, 0, st>>>(a);
    }
    // level 2: tiles within each band
    bin2_plan<<<1, kTB, 0, st>>>(start1, nbands, items, wfirst, misc + 4);
    a.dst = carve_soa(l2, n);
    a.hist = hist2;
    a.items = items;
    bin_count<2><<<(unsigned)maxitems, kBinThreads, 0, st>>>(a);
    const unsigned tg = (unsigned)((nt + kTB - 1) / kTB);
    bin2_tiles<false><<<tg, kTB, 0, st>>>(hist2, wfirst, geo.ntiles, tot, nullptr);
    scan_launch<unsigned>(st, tot, nt, seg, misc + 2, start);
    bin2_tiles<true><<<tg, kTB, 0, st>>>(hist2, wfirst, geo.ntiles, nullptr, start);
    bin_scatter<2><<<(unsigned)maxitems, kBinThreads, 0, st>>>(a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("tile binning: ") + hipGetErrorString(e));
    if (keep_outside && n_outside_host) {
        uint64_t* pin = ctx_pinned(ctx);
        if (hipMemcpyAsync(pin, start1 + nbands, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "outside count readback failed");
        const unsigned valid = (unsigned)(pin[0] & 0xffffffffu);          // start of the out-of-grid bin
        const unsigned dropped = (unsigned)(pin[0] >> 32);               // start of the dropped bin
        *n_outside_host = dropped - valid;
        if (outside_idx) *outside_idx = a.src.idx + valid;
    } else if (outside_idx) {
        *outside_idx = nullptr;
    }
    tb->sx = a.dst.x;
    tb->sy = a.dst.y;
    tb->sidx = a.dst.idx;
    tb->skey = a.dst.key;
    tb->start = start;
    tb->nb = geo.nb;
    tb->dnb = geo.dnb;
    tb->ts = geo.ts;
    tb->nt = geo.nt;
    tb->mnx = geo.mnx;
    tb->mny = geo.mny;
    tb->l = geo.l;
    return GEOHIP_OK;
}

// Join binning (jb_bands / jb_scan / jb_segs / jb_tiles): the window's in-grid points as
// tile-sorted 16-B records; *recs and *tstart (ntiles + 1) on the device.
int join_bin(geohip_ctx* ctx, Scratch& S, const double* dx, const double* dy, uint64_t n, const TileGeom& geo,
             unsigned* tcnt, const unsigned* qstart, const unsigned* gcnt, unsigned* istart, uint2* items,
             const uint4** recs, const unsigned** tstart) {
    hipStream_t st = ctx_stream(ctx);
    uint64_t nblk = (n + 16383) / 16384;
    if (nblk > kJbBlocks) nblk = kJbBlocks;
    if (nblk < 1) nblk = 1;
    JBin a;
    memset(&a, 0, sizeof a);
    a.x = dx;
    a.y = dy;
    a.n = n;
    a.chunk = (n + nblk - 1) / nblk;
    a.g = geo;
    a.nbands = (unsigned)((geo.ntiles + kBandTiles - 1) / kBandTiles);
    a.nsub = (unsigned)((a.chunk + kJbSub - 1) / kJbSub);
    if (a.nsub < 1) a.nsub = 1;
    a.nblk = (unsigned)nblk;
    const uint64_t nt = geo.ntiles;
    const uint64_t nseg = (uint64_t)a.nblk * a.nsub;
    const uint64_t maxround = n / kJbRound + a.nbands + 1;
    a.l1 = S.get<uint4>(J_SY, n * 16 + 64);
    a.recs = S.get<uint4>(J_SX, n * 16 + 64);
    a.soff = S.get<unsigned>(J_HIST, (size_t)nblk * a.nsub * (a.nbands + 1) * 4 + 16);
    a.tstart = S.get<unsigned>(J_TSTART, (nt + 1) * 4);
    a.tcur = S.get<unsigned>(J_TCUR, (nt + 1) * 4);
    char* seg = S.get<char>(J_SEG, (size_t)a.nbands * (2 * nseg + 1) * 4 + a.nbands * 4 + 16 + maxround * 16 + 64);
    if (S.rc) return S.rc;
    a.rinfo = reinterpret_cast<uint4*>(seg);
    a.spre = reinterpret_cast<unsigned*>(seg + maxround * 16);
    a.sst = a.spre + (size_t)a.nbands * (nseg + 1);
    a.nne = a.sst + (size_t)a.nbands * nseg;
    a.nround = a.nne + a.nbands;
    a.tcnt = tcnt;  // zero on entry: part of the step's zero block, no state carried between calls
    a.qstart = qstart;
    a.gcnt = gcnt;
    a.istart = istart;
    a.items = items;
    if (n) tlaunch(ctx, jb_bands, (unsigned)nblk, kBinThreads, 0, st, a);
    tlaunch(ctx, jb_scan, 1, kBinThreads, 0, st, a);
    if (n) {
        tlaunch(ctx, jb_segs, a.nbands, kBinThreads, 0, st, a);
        tlaunch(ctx, jb_tiles, (unsigned)std::min<uint64_t>(kJbL2Blocks, maxround), kJbL2Threads, 0, st, a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("join binning: ") + hipGetErrorString(e));
    *recs = a.recs;
    *tstart = a.tstart;
    return GEOHIP_OK;
}

int read_total(geohip_ctx* ctx, unsigned long long* dev_total, uint64_t* out) {
    hipStream_t st = ctx_stream(ctx);
    uint64_t* pin = ctx_pinned(ctx);
    if (hipMemcpyAsync(pin, dev_total, 8, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "count readback failed");
    *out = pin[0];
    return GEOHIP_OK;
}

// Squared-distance screen bounds for "dist <= r" (device_common.h kSqLo/kSqHi), disabled
// (r2lo < 0, r2hi = inf: every candidate takes the exact path) where r*r leaves the normal
// range and the 2^-40 relative margin would not hold.
void screen_bounds(double r, double* r2lo, double* r2hi) {
    const double r2 = r * r;
    if (r >= 0.0 && r2 >= 0x1.0p-960 && r2 <= 0x1.0p960) {
        *r2lo = r2 * kSqLo;
        *r2hi = r2 * kSqHi;
    } else if (r > 0.0 && r2 > 0x1.0p960) {  // every finite square is below the bound
        *r2lo = r2 * kSqLo;
        *r2hi = __builtin_inf();
    } else {
        *r2lo = -1.0;
        *r2hi = __builtin_inf();
    }
}

}  // namespace

void pp_screen_bounds(double r, double* r2lo, double* r2hi) { screen_bounds(r, r2lo, r2hi); }

int join_pp_impl(geohip_ctx* ctx, const geohip_grid* gd, const geohip_grid* gq, const double* dx, const double* dy,
                 uint64_t nd, const double* qx, const double* qy, uint64_t nq, double r, int approximate,
                 uint32_t* out_pairs, uint64_t cap, uint64_t* out_count, bool count_only, uint64_t* count_dev) {
    const bool async = count_dev != nullptr;
    if (!out_count && !async) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out_count");
    if (out_count) *out_count = 0;
    int rc = check_grid_basic(ctx, gd, "data grid");
    if (!rc) rc = check_grid_basic(ctx, gq, "query grid");
    if (rc) return rc;
    if (nd >= 0xffffffffull || nq >= 0xffffffffull) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "stream larger than 2^32-1");
    if (!count_only && cap && !out_pairs) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out_pairs");
    const bool all_cells = (r == 0);  // UniformGrid.java:264-266
    const int32_t lc = layers_candidate(*gq, r);
    if (!all_cells && lc <= 0)
        return ctx_fail(ctx, GEOHIP_ERR_ARG, "candidateNeighboringLayers cannot be 0 or less (UniformGrid.java:272-276)");
    hipStream_t st = ctx_stream(ctx);
    const bool dev = ctx_mem(ctx) == GEOHIP_MEM_DEVICE;
    const int32_t nb = gq->n;
    const TileGeom geo = tile_geom(*gd, nb);
    // per-query tile span bound (the block is 2 Lc + 1 cells before clipping): per-tile query
    // lists when small, otherwise every tile checks every query
    const uint64_t span_cells = all_cells ? (uint64_t)nb : std::min<uint64_t>(2ull * (uint64_t)lc + 1ull, (uint64_t)nb);
    const uint64_t span_tiles = std::min<uint64_t>((span_cells + geo.ts - 1) / geo.ts + 1, (uint64_t)geo.nt);
    const uint64_t per_query = span_tiles * span_tiles;
    const bool global_mode = all_cells || per_query > kGlobalTiles;
    const uint64_t list_cap = global_mode ? 0 : per_query * nq;
    Scratch S{ctx};
    const double *ddx, *ddy, *dqx, *dqy;
    rc = ctx_stage_xy(ctx, dx, dy, nd, 0, &ddx, &ddy);
    if (!rc) rc = ctx_stage_xy(ctx, qx, qy, nq, 1, &dqx, &dqy);
    if (rc) return rc;
    const uint64_t ntl = geo.ntiles;
    // item bound: per tile ceil(points / kJP) * ceil(queries / kJQ)
    const uint64_t qpt = global_mode ? nq : std::min<uint64_t>(nq, list_cap);
    const uint64_t item_cap = ((nd + kJP - 1) / kJP + ntl) * ((qpt + kJQ - 1) / kJQ) + 1;
    QRect* drect = S.get<QRect>(J_RECT, nq * sizeof(QRect) + 16);
    // per-call counters, zeroed by one launch (fill_words): query counts | query cursors | misc words
    // ([0] jq_rect error, [4] ticket, [5] global query count) | the pair total (u64) | tile counts
    const uint64_t ztot = (2 * (ntl + 1) + kMiscWords + 1) & ~(uint64_t)1;  // word offset of the total
    const unsigned nzero = (unsigned)(ztot + 2 + ntl + 1);
    unsigned* zero = S.get<unsigned>(J_QCNT, (size_t)nzero * 4 + 16);
    unsigned* qstart = S.get<unsigned>(J_QSTART, (ntl + 1) * 4);
    unsigned* qlist = S.get<unsigned>(J_QLIST, list_cap * 4 + 16);
    unsigned* glist = S.get<unsigned>(J_GLIST, nq * 4 + 16);
    unsigned* istart = S.get<unsigned>(J_BOFF, (ntl + 1) * 4);
    uint2* items = S.get<uint2>(J_MWORDS, item_cap * 8);
    if (S.rc) return S.rc;
    unsigned* qcnt = zero;
    unsigned* qcur = zero + (ntl + 1);
    unsigned* misc = zero + 2 * (ntl + 1);
    unsigned long long* total = reinterpret_cast<unsigned long long*>(zero + ztot);
    unsigned* tcnt = zero + ztot + 2;
    unsigned* fault = nullptr;  // async: query-key errors surface at geohip_ctx_sync
    if (async) {
        rc = ctx_fault_block(ctx, &fault);
        if (rc) return rc;
        total = reinterpret_cast<unsigned long long*>(count_dev);  // the caller's device count word
    }
    hipEvent_t e0, e1;
    ctx_timing_events(ctx, &e0, &e1);
    if (e0) hipEventRecord(e0, st);  // the whole device step: binning, replication, join
    // every kernel of the step is timed on its own (tlaunch: the dispatch's begin / end stamps)
    tlaunch(ctx, zero_step, (nzero + kTB - 1) / kTB, kTB, 0, st, zero, nzero,
            async ? reinterpret_cast<unsigned long long*>(count_dev) : (unsigned long long*)nullptr, (unsigned*)nullptr, 0u);
    const unsigned qb = (unsigned)((nq + kTB - 1) / kTB);
    if (nq) {
        JqGeom jg{gq->min_x, gq->min_y, gq->cell_len, nb, lc, all_cells ? 1 : 0};
        tlaunch(ctx, jq_rect, qb, kTB, 0, st, dqx, dqy, nq, jg, drect, misc, fault);
    }
    if (global_mode) {
        if (nq) tlaunch(ctx, jq_global, qb, kTB, 0, st, nq, glist, misc + 5);
        tlaunch(ctx, jq_starts, 1, kBinThreads, 0, st, (const unsigned*)qcnt, geo.ntiles, qstart);  // all zero
    } else {
        const unsigned qg = (unsigned)((nq + kTB / kWave - 1) / (kTB / kWave));  // one wave per query
        if (nq) tlaunch(ctx, jq_build<false>, qg, kTB, 0, st, (const QRect*)drect, nq, geo, qcnt, (const unsigned*)nullptr,
                        (unsigned*)nullptr);
        tlaunch(ctx, jq_starts, 1, kBinThreads, 0, st, (const unsigned*)qcnt, geo.ntiles, qstart);
        if (nq) tlaunch(ctx, jq_build<true>, qg, kTB, 0, st, (const QRect*)drect, nq, geo, qcur, (const unsigned*)qstart,
                        qlist);
    }
    const uint4* recs = nullptr;
    const unsigned* tstart = nullptr;
    rc = join_bin(ctx, S, ddx, ddy, nd, geo, tcnt, qstart, misc + 5, istart, items, &recs, &tstart);
    if (rc) return rc;
    // output: device pointer directly, or a device staging buffer for host output
    unsigned* out = nullptr;
    if (!count_only && cap) {
        if (dev) {
            out = out_pairs;
        } else {
            void* p = nullptr;
            rc = ctx_ensure(ctx, J_OUT, cap * 8, &p);
            if (rc) return rc;
            out = reinterpret_cast<unsigned*>(p);
        }
    }
    double r2lo, r2hi;
    screen_bounds(r, &r2lo, &r2hi);
    const bool write = !count_only;
    JoinRun jr{recs, tstart, ddx, ddy, geo, qstart, qlist, glist, misc + 5, dqx, dqy, drect, r, r2lo, r2hi, istart, items, geo.ntiles,
               misc + 4, total, out, out ? cap : 0, ((uintptr_t)out & 7u) == 0};
    if (nq && nd) {
        if (approximate) {
            if (write) tlaunch(ctx, join_fused<true, true>, kJBlocksW, kTB, 0, st, jr);
            else tlaunch(ctx, join_fused<true, false>, kJBlocksC, kTB, 0, st, jr);
        } else {
            if (write) tlaunch(ctx, join_fused<false, true>, kJBlocksW, kTB, 0, st, jr);
            else tlaunch(ctx, join_fused<false, false>, kJBlocksC, kTB, 0, st, jr);
        }
    }
    if (e1) hipEventRecord(e1, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("join launch: ") + hipGetErrorString(e));
    if (async) return GEOHIP_OK;  // the total is in *count_dev; errors at geohip_ctx_sync
    // one readback: the pair total and the query-block error word
    uint64_t* pin = ctx_pinned(ctx);
    if (hipMemcpyAsync(pin, total, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(pin + 1, misc, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "count readback failed");
    const uint64_t tot = pin[0];
    const unsigned qerr = (unsigned)(pin[1] & 0xffffffffu);
    if (qerr == 1) return ctx_fail(ctx, GEOHIP_ERR_ARG, "NumberFormatException in getIntCellIndices (query point key)");
    if (qerr == 2) return ctx_fail(ctx, GEOHIP_ERR_ARG, "reference neighbour loop does not terminate");
    *out_count = tot;
    if (!count_only && !dev && cap) {
        const uint64_t m = std::min<uint64_t>(tot, cap);
        if (m && hipMemcpy(out_pairs, out, m * 8, hipMemcpyDeviceToHost) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "pair readback failed");
    }
    if (!count_only && tot > cap) return ctx_fail(ctx, GEOHIP_ERR_CAPACITY, "output capacity too small; *out_count = required");
    return GEOHIP_OK;
}

// y-slab lists of one polygon (SlabView), appended to blob; P.ns = 0 when they cannot be built
// (few or very many segments, non-finite extent): the device then visits every segment.
// rid (nullable): ring id per vertex; a ring junction (rid[e] != rid[e+1]) is no segment.
void plan_slabs(PolyDev& P, const double* ry, const ring_id_t* rid, double r, double cell_len,
                std::vector<uint16_t>& blob) {
    P.ns = 0;
    P.sy0 = 0.0;
    P.sinv = 0.0;
    P.E = 0.0;
    P.loff = (uint32_t)blob.size();
    P.llen = 0;
    const uint32_t nseg = P.nv >= 2 ? P.nv - 1 : 0;
    if (nseg < 8 || nseg > 30000) return;
    const double ext = (P.gb[2] - P.gb[0]) + (P.gb[3] - P.gb[1]);
    // E bounds the screen radius of every point a work item evaluates (C cells lie within
    // r + 2 cells of the envelope); a point with a larger screen radius takes the full loop
    const double E = r + 0x1.0p-40 * 4.0 * (ext + std::fabs(r) + cell_len);
    if (!(E >= 0.0) || !std::isfinite(E) || !std::isfinite(ext)) return;
    const double y0 = P.gb[1] - E, y1 = P.gb[3] + E;
    const uint32_t ns = std::min<uint32_t>(64, nseg);
    const double span = y1 - y0;
    if (!(span > 0.0) || !std::isfinite(span)) return;
    const double sinv = (double)ns / span;
    if (!(sinv > 0.0) || !std::isfinite(sinv)) return;
    const double pad = 1e-6 * span / ns;
    // slab ranges of segment e: crossing [c0, c1], distance [d0, d1] (empty for a NaN y: such a
    // segment never counts, flags or comes within r); computed in both passes, nothing stored
    auto ranges = [&](uint32_t e, uint32_t& c0, uint32_t& c1, uint32_t& d0, uint32_t& d1) -> bool {
        const double a = ry[e], b = ry[e + 1];
        if (a != a || b != b) return false;
        if (rid && rid[e] != rid[e + 1]) return false;
        const double lo = std::min(a, b), hi = std::max(a, b);
        c0 = slab_of(lo - pad, y0, sinv, ns);
        c1 = slab_of(hi + pad, y0, sinv, ns);
        d0 = slab_of((lo - E) - pad, y0, sinv, ns);
        d1 = slab_of((hi + E) + pad, y0, sinv, ns);
        return true;
    };
    uint32_t cn[65] = {0}, dn[65] = {0};
    for (uint32_t e = 0; e < nseg; e++) {
        uint32_t c0, c1, d0, d1;
        if (!ranges(e, c0, c1, d0, d1)) continue;
        for (uint32_t t = c0; t <= c1; t++) cn[t]++;
        for (uint32_t t = d0; t <= d1; t++) dn[t]++;
    }
    uint64_t total = 0;
    for (uint32_t t = 0; t < ns; t++) total += cn[t] + dn[t];
    if (total + 2ull * (ns + 1) > 65535ull) return;
    const size_t h = blob.size();
    blob.resize(h + 2 * (ns + 1) + total);
    uint16_t* B = blob.data() + h;
    uint32_t k = 0;
    for (uint32_t t = 0; t < ns; t++) { B[t] = (uint16_t)k; k += cn[t]; }
    B[ns] = (uint16_t)k;
    for (uint32_t t = 0; t < ns; t++) { B[ns + 1 + t] = (uint16_t)k; k += dn[t]; }
    B[2 * ns + 1] = (uint16_t)k;
    uint32_t cf[64] = {0}, df[64] = {0};
    uint16_t* ids = B + 2 * (ns + 1);
    for (uint32_t e = 0; e < nseg; e++) {
        uint32_t c0, c1, d0, d1;
        if (!ranges(e, c0, c1, d0, d1)) continue;
        for (uint32_t t = c0; t <= c1; t++) ids[B[t] + cf[t]++] = (uint16_t)e;
        for (uint32_t t = d0; t <= d1; t++) ids[B[ns + 1 + t] + df[t]++] = (uint16_t)e;
    }
    P.ns = ns;
    P.sy0 = y0;
    P.sinv = sinv;
    P.E = E;
    P.llen = (uint32_t)(2 * (ns + 1) + total);
}

// ---------------------------------------------------------------- cell classes ------------
// Host geometry for classify_cells.  Every decision below is conservative: a computed quantity
// only decides when it clears its rounding by a wide relative margin; otherwise the cell stays
// kClsMixed and its points take the exact per-point path on the device.
namespace cls {
struct Seg {
    double ax, ay, bx, by;
    uint32_t ring;
};
// distance from p to segment s in plain fp64 (error << the margins used)
inline double pt_seg(double px, double py, const Seg& s) {
    const double ex = s.bx - s.ax, ey = s.by - s.ay;
    const double l2 = ex * ex + ey * ey;
    double t = l2 > 0.0 ? ((px - s.ax) * ex + (py - s.ay) * ey) / l2 : 0.0;
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    const double dx = px - (s.ax + t * ex), dy = py - (s.ay + t * ey);
    return std::sqrt(dx * dx + dy * dy);
}
// does the segment meet the box [x0, x1] x [y0, y1] (Liang-Barsky clip; the caller inflates the
// box, so a computed "no" is a true "no")
inline bool seg_meets_box(const Seg& s, double x0, double x1, double y0, double y1) {
    double t0 = 0.0, t1 = 1.0;
    const double dx = s.bx - s.ax, dy = s.by - s.ay;
    const double pv[4] = {-dx, dx, -dy, dy};
    const double qv[4] = {s.ax - x0, x1 - s.ax, s.ay - y0, y1 - s.ay};
    for (int i = 0; i < 4; i++) {
        if (pv[i] == 0.0) {
            if (qv[i] < 0.0) return false;
        } else {
            const double t = qv[i] / pv[i];
            if (pv[i] < 0.0) { if (t > t1) return false; if (t > t0) t0 = t; }
            else { if (t < t0) return false; if (t < t1) t1 = t; }
        }
    }
    return true;
}
// distance from the box to a segment that does not meet it: attained at a box corner or a
// segment end (two disjoint convex sets)
inline double box_seg(double x0, double x1, double y0, double y1, const Seg& s) {
    double d = std::min(std::min(pt_seg(x0, y0, s), pt_seg(x0, y1, s)), std::min(pt_seg(x1, y0, s), pt_seg(x1, y1, s)));
    auto pb = [&](double px, double py) {
        const double ex = std::max(std::max(x0 - px, px - x1), 0.0), ey = std::max(std::max(y0 - py, py - y1), 0.0);
        return std::sqrt(ex * ex + ey * ey);
    };
    return std::min(d, std::min(pb(s.ax, s.ay), pb(s.bx, s.by)));
}
}  // namespace cls

// Classes of the cells of P's walk region that the device evaluates exactly (C cells; the join's
// G u C in exact mode).  For a box B of doubles (a cell's exact coordinate box from plan.cpp's
// axis bounds -- every non-NaN point of the cell lies in it -- or a subcell's):
//  * HIT when one segment s has all four corners of B within r - m of it (distance to a segment
//    is convex, so every p in B is within r - m of s and the JTS distance, 0 inside or the
//    minimum over segments outside, is <= r), or when no segment meets B and B's centre is
//    inside the polygon (no point of B is then on a ring, the crossing parities are the same
//    for all of B: every point is interior, distance 0);
//  * MISS when no segment meets B, the centre is outside (so all of B is) and every segment is
//    farther than r + m from B;
//  * MIXED otherwise.  m = 2^-36 (scale + r) covers JTS's rounding (<= 2^-49 of the magnitudes,
//    segment_within) and this code's own.
// A cell that stays MIXED is split into 4 x 4 subcells (sub_edge) classified the same way.
struct BoxClassifier {
    std::vector<cls::Seg> segs;
    double scale = 0.0, r = 0.0;
    uint32_t nring = 1;
    std::vector<uint8_t> par;
    uint8_t operator()(double x0, double x1, double y0, double y1) {
        using cls::Seg;
        if (!(x0 <= x1) || !(y0 <= y1)) return kClsMiss;  // an empty box holds no point
        const double sc = std::max(scale, std::max(std::max(std::fabs(x0), std::fabs(x1)), std::max(std::fabs(y0), std::fabs(y1))));
        const double m = 0x1.0p-36 * (sc + r);
        for (const Seg& s : segs) {
            // (only a segment whose box, grown by r, holds B can cover it)
            if (std::min(s.ax, s.bx) - r > x0 || std::max(s.ax, s.bx) + r < x1 || std::min(s.ay, s.by) - r > y0 ||
                std::max(s.ay, s.by) + r < y1)
                continue;
            if (std::max(std::max(cls::pt_seg(x0, y0, s), cls::pt_seg(x0, y1, s)),
                         std::max(cls::pt_seg(x1, y0, s), cls::pt_seg(x1, y1, s))) <= r - m)
                return kClsHit;
        }
        const double d = 0x1.0p-30 * (sc + (x1 - x0) + (y1 - y0));  // inflation
        for (const Seg& s : segs)
            if (cls::seg_meets_box(s, x0 - d, x1 + d, y0 - d, y1 + d)) return kClsMixed;
        // location of the centre: crossing parity per ring to the +x side (the device's
        // RayCrossingCounter direction); no segment is near the centre, so the determinant signs
        // are far from their rounding -- checked, else mixed
        const double px = 0.5 * x0 + 0.5 * x1, py = 0.5 * y0 + 0.5 * y1;
        std::fill(par.begin(), par.end(), (uint8_t)0);
        for (const Seg& s : segs) {
            const double p1x = s.bx, p1y = s.by, p2x = s.ax, p2y = s.ay;  // count_segment(p, v[e+1], v[e])
            if (p1x < px && p2x < px) continue;
            if (!((p1y > py && p2y <= py) || (p2y > py && p1y <= py))) continue;
            const double x1r = p1x - px, y1r = p1y - py, x2r = p2x - px, y2r = p2y - py;
            const double tl = x1r * y2r, tr = y1r * x2r, det = tl - tr;
            if (!(std::fabs(det) > 1e-9 * (std::fabs(tl) + std::fabs(tr)))) return kClsMixed;
            int sg = det > 0.0 ? 1 : -1;
            if (y2r < y1r) sg = -sg;
            if (sg > 0) par[s.ring] ^= 1;
        }
        bool inside = par[0] != 0;
        for (uint32_t j = 1; j < nring && inside; j++) inside = par[j] == 0;
        if (inside) return kClsHit;
        const double rm = r + 2.0 * m;
        double dmin = INFINITY;
        for (const Seg& s : segs) {
            // a segment whose box is farther than r + 2m from B is farther still
            if (std::min(s.ax, s.bx) > x1 + rm || std::max(s.ax, s.bx) < x0 - rm || std::min(s.ay, s.by) > y1 + rm ||
                std::max(s.ay, s.by) < y0 - rm)
                continue;
            dmin = std::min(dmin, cls::box_seg(x0, x1, y0, y1, s));
        }
        return dmin > r + m ? kClsMiss : kClsMixed;
    }
};

// Returns false (no classes) for r < 0 / NaN / inf, non-finite vertices or too large a region.
// rf / rfw (may be null): the refinement table of the mixed subcells (kNoRefine entries otherwise),
// rf parallel to blob.
bool classify_cells(const PolyDev& P, const std::vector<double>& hvx, const std::vector<double>& hvy,
                    const ring_id_t* rid, const geohip_grid& pg, const int32_t* rects, uint32_t first_c,
                    uint32_t nrect_c, uint32_t nring, double r, std::vector<uint32_t>& blob, uint32_t* off,
                    std::vector<uint32_t>* rf = nullptr, std::vector<uint32_t>* rfw = nullptr,
                    std::vector<uint32_t>* rfw2 = nullptr) {
    *off = kNoCls;
    if (!(r >= 0.0) || !std::isfinite(r) || P.wx0 > P.wx1 || P.wy0 > P.wy1 || nrect_c == 0) return false;
    BoxClassifier bc;
    bc.r = r;
    bc.scale = std::fabs(r);
    bc.nring = nring;
    bc.par.assign(nring, 0);
    for (uint32_t i = 0; i + 1 < P.nv; i++) {
        const double ax = hvx[P.voff + i], ay = hvy[P.voff + i], bx = hvx[P.voff + i + 1], by = hvy[P.voff + i + 1];
        if (!std::isfinite(ax) || !std::isfinite(ay) || !std::isfinite(bx) || !std::isfinite(by)) return false;
        bc.scale = std::max(bc.scale, std::max(std::max(std::fabs(ax), std::fabs(ay)), std::max(std::fabs(bx), std::fabs(by))));
        if (rid && rid[i] != rid[i + 1]) continue;  // ring junction: no segment
        bc.segs.push_back(cls::Seg{ax, ay, bx, by, rid ? (uint32_t)rid[i] : 0u});
    }
    if (bc.segs.empty()) return false;
    const int32_t w = P.wx1 - P.wx0 + 1, h = P.wy1 - P.wy0 + 1;
    if ((uint64_t)w * (uint64_t)h * bc.segs.size() > 8000000ull) return false;
    std::vector<double> xl(w), xh(w), yl(h), yh(h);
    std::vector<uint8_t> okx(w), oky(h);
    for (int32_t a = 0; a < w; a++)
        okx[a] = axis_lower(pg.min_x, pg.cell_len, P.wx0 + a, &xl[a]) && axis_upper(pg.min_x, pg.cell_len, P.wx0 + a, &xh[a]) &&
                 std::isfinite(xl[a]) && std::isfinite(xh[a]) && xl[a] <= xh[a];
    for (int32_t c = 0; c < h; c++)
        oky[c] = axis_lower(pg.min_y, pg.cell_len, P.wy0 + c, &yl[c]) && axis_upper(pg.min_y, pg.cell_len, P.wy0 + c, &yh[c]) &&
                 std::isfinite(yl[c]) && std::isfinite(yh[c]) && yl[c] <= yh[c];
    const size_t base = blob.size();
    blob.resize(base + (size_t)w * h, 0u);  // all mixed
    uint32_t* out = blob.data() + base;
    if (rf) rf->resize(2 * (base + (size_t)w * h), kNoRefine);
    // subcell i of an axis: the doubles v of the cell box [bl, bh] with sub_of(v) == i
    auto sub_iv = [](double mn, double l, int32_t c, double bl, double bh, int i, double& lo, double& hi) {
        lo = i == 0 ? bl : std::max(bl, sub_edge(mn, l, c, i));
        hi = i == 3 ? bh : std::min(bh, std::nextafter(sub_edge(mn, l, c, i + 1), -INFINITY));
    };
    for (int32_t a = 0; a < w; a++) {
        if (!okx[a]) continue;
        for (int32_t c = 0; c < h; c++) {
            if (!oky[c]) continue;
            const int32_t cx = P.wx0 + a, cy = P.wy0 + c;
            bool in_c = false;
            for (uint32_t q = 0; q < nrect_c && !in_c; q++) {
                const int32_t* R = rects + 4 * (first_c + q);
                in_c = cx >= R[0] && cx <= R[1] && cy >= R[2] && cy <= R[3];
            }
            if (!in_c) continue;
            const uint8_t k = bc(xl[a], xh[a], yl[c], yh[c]);
            if (k == kClsHit) { out[(size_t)a * h + c] = kWordHit; continue; }
            if (k == kClsMiss) { out[(size_t)a * h + c] = kWordMiss; continue; }
            uint32_t word = 0;
            uint32_t rw[16];
            uint32_t qw[16][16];  // [subcell][part]: second-level words of the mixed parts
            bool refined = false;
            for (int sx = 0; sx < 4; sx++) {
                double sx0, sx1;
                sub_iv(pg.min_x, pg.cell_len, cx, xl[a], xh[a], sx, sx0, sx1);
                for (int sy = 0; sy < 4; sy++) {
                    double sy0, sy1;
                    sub_iv(pg.min_y, pg.cell_len, cy, yl[c], yh[c], sy, sy0, sy1);
                    const uint8_t ks = bc(sx0, sx1, sy0, sy1);
                    word |= (uint32_t)ks << (2 * (4 * sx + sy));
                    rw[4 * sx + sy] = 0u;
                    if (ks != kClsMixed || !rf) continue;
                    // the subcell's 4 x 4 parts: [sub16 edge, next edge) clipped to the subcell; a
                    // mixed part's 4 x 4 sub-parts likewise on the sub64 edges
                    uint32_t pw = 0;
                    for (int tx = 0; tx < 4; tx++) {
                        const int qx = 4 * sx + tx;
                        const double px0 = tx == 0 ? sx0 : std::max(sx0, sub16_edge(pg.min_x, pg.cell_len, cx, qx));
                        const double px1 = tx == 3 ? sx1 : std::min(sx1, std::nextafter(sub16_edge(pg.min_x, pg.cell_len, cx, qx + 1), -INFINITY));
                        for (int ty = 0; ty < 4; ty++) {
                            const int qy = 4 * sy + ty;
                            const double py0 = ty == 0 ? sy0 : std::max(sy0, sub16_edge(pg.min_y, pg.cell_len, cy, qy));
                            const double py1 = ty == 3 ? sy1 : std::min(sy1, std::nextafter(sub16_edge(pg.min_y, pg.cell_len, cy, qy + 1), -INFINITY));
                            const uint8_t kp = bc(px0, px1, py0, py1);
                            pw |= (uint32_t)kp << (2 * (4 * tx + ty));
                            uint32_t w2 = 0;
                            if (kp == kClsMixed)
                                for (int ux = 0; ux < 4; ux++) {
                                    const double qx0 = ux == 0 ? px0 : std::max(px0, sub64_edge(pg.min_x, pg.cell_len, cx, 4 * qx + ux));
                                    const double qx1 = ux == 3 ? px1 : std::min(px1, std::nextafter(sub64_edge(pg.min_x, pg.cell_len, cx, 4 * qx + ux + 1), -INFINITY));
                                    for (int uy = 0; uy < 4; uy++) {
                                        const double qy0 = uy == 0 ? py0 : std::max(py0, sub64_edge(pg.min_y, pg.cell_len, cy, 4 * qy + uy));
                                        const double qy1 = uy == 3 ? py1 : std::min(py1, std::nextafter(sub64_edge(pg.min_y, pg.cell_len, cy, 4 * qy + uy + 1), -INFINITY));
                                        w2 |= (uint32_t)bc(qx0, qx1, qy0, qy1) << (2 * (4 * ux + uy));
                                    }
                                }
                            qw[4 * sx + sy][4 * tx + ty] = w2;
                            refined = refined || w2 != 0u;  // some sub-part decided
                        }
                    }
                    rw[4 * sx + sy] = pw;
                    refined = refined || pw != 0u;  // some part decided
                }
            }
            out[(size_t)a * h + c] = word;
            if (refined) {
                const size_t at = 2 * (base + (size_t)a * h + c);
                (*rf)[at] = (uint32_t)(rfw->size() / 2);
                (*rf)[at + 1] = word;
                for (int q = 0; q < 16; q++) {
                    if (!((refine_mixed(word) >> (2 * q)) & 1u)) continue;
                    const uint32_t pw = rw[q];
                    rfw->push_back(pw);
                    rfw->push_back(refine_mixed(pw) ? (uint32_t)rfw2->size() : kNoRefine);
                    for (int t = 0; t < 16; t++)
                        if ((refine_mixed(pw) >> (2 * t)) & 1u) rfw2->push_back(qw[q][t]);
                }
            }
        }
    }
    *off = (uint32_t)base;
    return true;
}

// The work item of polygon P on tile (a, c): kNoWork when no point of the tile can be a hit
// (every cell of the tile is outside P's rectangles or a kClsMiss C cell), kWorkAllHit when
// every point is (every cell of the tile is in a G rectangle, or a C cell of class kClsHit or
// with r = MAX_VALUE -- but NaN coordinates land in cell 0 of their axis, so a cell of row or
// column 0 must be guaranteed), else 0.
constexpr uint32_t kNoWork = 0xffffffffu;
uint32_t tile_work(const PolyDev& P, const int32_t* rects, const std::vector<uint32_t>& hcls, const TileGeom& geo,
                   int32_t a, int32_t c, bool r_is_max) {
    auto in_list = [&](uint32_t off, uint32_t n, int32_t cx, int32_t cy) {
        for (uint32_t q = 0; q < n; q++) {
            const int32_t* R = rects + 4 * (off + q);
            if (cx >= R[0] && cx <= R[1] && cy >= R[2] && cy <= R[3]) return true;
        }
        return false;
    };
    const int32_t ch = P.wy1 - P.wy0 + 1;
    bool any = false, all = true;
    for (int32_t cx = a * geo.ts; cx < std::min((a + 1) * geo.ts, geo.nb); cx++)
        for (int32_t cy = c * geo.ts; cy < std::min((c + 1) * geo.ts, geo.nb); cy++) {
            const bool g = in_list(P.goff, P.ng, cx, cy);
            const bool cc = !g && in_list(P.coff, P.nc, cx, cy);
            uint32_t k = 0;
            if (cc && P.cls != kNoCls) k = hcls[P.cls + (size_t)(cx - P.wx0) * ch + (cy - P.wy0)];
            any = any || g || (cc && k != kWordMiss);
            const bool hit = g || (cc && (r_is_max || k == kWordHit) && cx > 0 && cy > 0);
            all = all && hit;
        }
    if (!any) return kNoWork;
    return all ? kWorkAllHit : 0u;
}

// Polygon plan cache, one entry per ctx: a continuous point-polygon query evaluates the same
// polygons on every window, so the host planning (rings, envelopes, G/C rectangles, work items,
// slab lists: ~2 ms for 1000 polygons) and the device upload are done once; later calls compare
// their inputs bitwise with the cached copies (the inputs decide everything the plan holds).
struct PolyCache {
    geohip_grid grid{}, gq{};
    int jmode = 0;
    int approx = 0;  // the cell classes and the keep filter hold for exact distances only
    double r = 0.0;
    std::vector<uint32_t> poly_rings;  // as given, or the identity when the caller passed none
    std::vector<uint32_t> ring_off;    // ring_off[R0 .. R1] (absolute vertex offsets)
    std::vector<double> vx, vy;        // vx/vy[ring_off[R0] .. ring_off[R1])
    std::vector<PolyDev> pd;
    std::vector<double> hvx, hvy, henv;
    std::vector<ring_id_t> hvr;
    std::vector<int32_t> hrects;
    std::vector<PolyWork> hwork;
    std::vector<uint16_t> hslab;
    std::vector<uint32_t> hcls;  // per-cell class words (classify_cells), PolyDev.cls offsets into it
    std::vector<uint32_t> hrf;   // 2 per hcls cell: first refinement word (or kNoRefine), class word
    std::vector<uint32_t> hrfw;  // 2 per mixed subcell of a refined cell: part word, first second-level word
    std::vector<uint32_t> hrfw2; // second-level words (one per mixed part of those subcells)
    std::vector<uint32_t> keep;  // cells of any polygon's G or C rectangles (empty: no filter)
    bool any_outside = false;
    // streaming path (ppoly_stream): per key cell its polygon entries, the cells holding any
    // (bitmap), the polygons whose rectangles reach outside the grid; stream_ok = false when the
    // key space or the table is too large (the tile-binned path runs instead)
    bool stream_ok = false;
    std::vector<uint32_t> cell_off;   // nb * nb + 1 (host only)
    std::vector<uint32_t> cell_ent;   // 2 per entry: poly | kEntC, class word
    std::vector<uint32_t> cell_head;  // 2 per cell (see kMulti)
    uint32_t max_cell_ent = 0;        // the most entries of one cell (sizes the overflow lists)
    std::vector<uint32_t> skeep;
    std::vector<uint32_t> opoly;
    uint64_t last_cand = 0;           // candidates of the previous step (sizes the buffer)
    void* dev_blob = nullptr;  // J_POLY buffer holding the uploaded tables
    size_t blob_bytes = 0;
};
// the cache lives in the ctx (one ctx per calling thread: no lock)
PolyCache* ctx_pcache(geohip_ctx* ctx) {
    void** slot = ctx_pcache_slot(ctx);
    if (!*slot) *slot = new PolyCache();
    return static_cast<PolyCache*>(*slot);
}

// ring range of polygon p: [poly_rings[p], poly_rings[p+1]) (poly_rings null: ring p)
inline uint32_t ring_of(const uint32_t* poly_rings, uint32_t p) { return poly_rings ? poly_rings[p] : p; }

bool same_inputs(const PolyCache& c, const geohip_grid& g, double r, const uint32_t* poly_rings,
                 const uint32_t* ring_off, uint32_t npoly, const double* vx, const double* vy) {
    if (c.grid.min_x != g.min_x || c.grid.min_y != g.min_y || c.grid.cell_len != g.cell_len || c.grid.n != g.n) return false;
    if (memcmp(&c.r, &r, sizeof r) != 0 || c.poly_rings.size() != (size_t)npoly + 1) return false;
    for (uint32_t p = 0; p <= npoly; p++)
        if (c.poly_rings[p] != ring_of(poly_rings, p)) return false;
    const uint32_t R0 = c.poly_rings[0], R1 = c.poly_rings[npoly];
    if (c.ring_off.size() != (size_t)(R1 - R0) + 1) return false;
    if (memcmp(c.ring_off.data(), ring_off + R0, ((size_t)(R1 - R0) + 1) * 4) != 0) return false;
    const size_t v0 = ring_off[R0], v1 = ring_off[R1];
    if (v1 < v0 || c.vx.size() != v1 - v0) return false;
    return memcmp(c.vx.data(), vx + v0, (v1 - v0) * 8) == 0 && memcmp(c.vy.data(), vy + v0, (v1 - v0) * 8) == 0;
}

void ppoly_note_cand_need(geohip_ctx* ctx, uint64_t need) {
    PolyCache* pc = ctx_pcache(ctx);
    if (need > pc->last_cand) pc->last_cand = need;
}

void ppoly_cache_drop(geohip_ctx* ctx) {
    void** slot = ctx_pcache_slot(ctx);
    delete static_cast<PolyCache*>(*slot);
    *slot = nullptr;
}

// Ring ids, ring envelopes and the box of every ring of a planned polygon (PolyPlan rings).
// Envelopes as JTS computes them (Envelope.expandToInclude: NaN coordinates never enter).
static void ring_tables(const PolyPlan& pl, std::vector<ring_id_t>& vr, std::vector<double>& env, double gb[4]) {
    const size_t nring = pl.ring_start.size() - 1;
    for (size_t j = 0; j < nring; j++) {
        const uint32_t a = pl.ring_start[j], b = pl.ring_start[j + 1];
        double mnx = pl.rx[a], mxx = pl.rx[a], mny = pl.ry[a], mxy = pl.ry[a];
        for (uint32_t i = a; i < b; i++) {
            vr.push_back((ring_id_t)j);
            const double x = pl.rx[i], y = pl.ry[i];
            if (x < mnx) mnx = x;
            if (x > mxx) mxx = x;
            if (y < mny) mny = y;
            if (y > mxy) mxy = y;
        }
        if (nring > 1) env.insert(env.end(), {mnx, mny, mxx, mxy});
        if (j == 0) { gb[0] = mnx; gb[1] = mny; gb[2] = mxx; gb[3] = mxy; }
        else {
            gb[0] = std::min(gb[0], mnx); gb[1] = std::min(gb[1], mny);
            gb[2] = std::max(gb[2], mxx); gb[3] = std::max(gb[3], mxy);
        }
    }
}

// The streaming path's cell table (see ppoly_stream): for every polygon and every cell of its
// walk region in one of its rectangles, one entry -- G (its G list, or r = MAX_VALUE) or C with
// the cell's class word (0 = every subcell mixed when the polygon has no classes); C cells of
// class kClsMiss hold no point within r and get no entry.
void build_stream_table(PolyCache& c, uint32_t npoly, int32_t nb, bool r_is_max) {
    c.stream_ok = false;
    c.cell_off.clear();
    c.cell_ent.clear();
    c.cell_head.clear();
    c.skeep.clear();
    c.opoly.clear();
    if (nb <= 0 || (uint64_t)nb * (uint64_t)nb > (1ull << 24)) return;
    const size_t ncell = (size_t)nb * (size_t)nb;
    auto in_list = [&](uint32_t off, uint32_t n, int32_t cx, int32_t cy) {
        for (uint32_t q = 0; q < n; q++) {
            const int32_t* R = &c.hrects[4 * (size_t)(off + q)];
            if (cx >= R[0] && cx <= R[1] && cy >= R[2] && cy <= R[3]) return true;
        }
        return false;
    };
    // pass 0 counts per cell, pass 1 fills
    std::vector<uint32_t> cur;
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 0) c.cell_off.assign(ncell + 1, 0u);
        for (uint32_t p = 0; p < npoly; p++) {
            const PolyDev& P = c.pd[p];
            if (P.wx0 > P.wx1 || P.wy0 > P.wy1) continue;
            const int32_t ch = P.wy1 - P.wy0 + 1;
            for (int32_t cx = P.wx0; cx <= P.wx1; cx++)
                for (int32_t cy = P.wy0; cy <= P.wy1; cy++) {
                    const bool g = in_list(P.goff, P.ng, cx, cy);
                    const bool cc = !g && in_list(P.coff, P.nc, cx, cy);
                    if (!g && !cc) continue;
                    uint32_t ex = p, word = 0;
                    if (cc && !r_is_max) {
                        if (P.cls != kNoCls) word = c.hcls[P.cls + (size_t)(cx - P.wx0) * ch + (cy - P.wy0)];
                        if (word == kWordMiss) continue;
                        ex |= kEntC;
                    }
                    const size_t k = (size_t)cx * nb + cy;
                    if (pass == 0) {
                        c.cell_off[k + 1]++;
                    } else {
                        const uint32_t at = cur[k]++;
                        c.cell_ent[2 * (size_t)at] = ex;
                        c.cell_ent[2 * (size_t)at + 1] = word;
                    }
                }
        }
        if (pass == 0) {
            for (size_t k = 0; k < ncell; k++) c.cell_off[k + 1] += c.cell_off[k];
            if (c.cell_off[ncell] >= (1u << 28)) {
                c.cell_off.clear();
                return;
            }
            c.cell_ent.assign(2 * (size_t)c.cell_off[ncell], 0u);
            cur.assign(c.cell_off.begin(), c.cell_off.end() - 1);
        }
    }
    // packed stage words; LDS per-polygon counts; entry words (bits 30, 31 are flags)
    if (npoly >= kStreamMaxPolys || npoly > kCandLdsPolys || c.cell_off[ncell] >= kMulti) return;
    c.skeep.assign((ncell + 31) / 32, 0u);
    c.cell_head.assign(2 * ncell, 0u);
    c.max_cell_ent = 0;
    for (size_t k = 0; k < ncell; k++) {
        const uint32_t b = c.cell_off[k], e = c.cell_off[k + 1];
        c.cell_head[2 * k] = kNoEntry;
        if (e == b) continue;
        c.max_cell_ent = std::max(c.max_cell_ent, e - b);
        c.skeep[k >> 5] |= 1u << (k & 31);
        if (e - b == 1) {
            c.cell_head[2 * k] = c.cell_ent[2 * (size_t)b];
            c.cell_head[2 * k + 1] = c.cell_ent[2 * (size_t)b + 1];
        } else {
            c.cell_head[2 * k] = kMulti | (e - b);
            c.cell_head[2 * k + 1] = b;
        }
    }
    for (uint32_t p = 0; p < npoly; p++)
        if (c.pd[p].outside) c.opoly.push_back(p);
    c.stream_ok = true;
}

int ppoly_impl(geohip_ctx* ctx, const geohip_grid* grid, const geohip_grid* gq, int join, const double* x,
               const double* y, uint64_t n, const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
               const double* vy, uint64_t nv, uint32_t npoly, double r, int approximate, uint32_t* out_pairs,
               uint64_t cap, uint64_t* out_count, uint32_t point_base, uint64_t* count_dev) {
    const bool async = count_dev != nullptr;
    uint64_t count_local = 0;
    if (!out_count && !async) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out_count");
    if (!out_count) out_count = &count_local;
    *out_count = 0;
    int rc = check_grid_basic(ctx, grid, join ? "point grid" : "grid");
    if (!rc && join) rc = check_grid_basic(ctx, gq, "query grid");
    if (rc) return rc;
    if (!join) gq = grid;
    // join (PointPolygonJoinQuery.java:162-201): every point of G u C is distance-checked
    // (exact) or emitted (approximate); the range query's guaranteed shortcut does not apply
    const int jmode = join ? (approximate ? 2 : 1) : 0;
    if (n >= 0xffffffffull) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "window larger than 2^32-1 points");
    if (cap && !out_pairs) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out_pairs");
    if (npoly == 0) {  // no polygon: no pair (the polygon arrays may be null)
        if (async) {
            set_u64<<<1, 1, 0, ctx_stream(ctx)>>>(reinterpret_cast<unsigned long long*>(count_dev), 0ull);
            if (hipGetLastError() != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "count launch failed");
        }
        return GEOHIP_OK;
    }
    if (!ring_off || !vx || !vy) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null polygon arrays");
    hipStream_t st = ctx_stream(ctx);
    const bool dev = ctx_mem(ctx) == GEOHIP_MEM_DEVICE;
    const int32_t nb = gq->n;  // key space: the polygons' (query) grid; point cells on `grid`
    const TileGeom geo = tile_geom(*grid, nb);
    static const bool prof = getenv("GEOHIP_HOST_PROFILE") != nullptr;  // measurement only
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto t_start = now();
    for (uint32_t p = 0; p < npoly; p++)
        if (ring_of(poly_rings, p + 1) <= ring_of(poly_rings, p))
            return ctx_fail(ctx, GEOHIP_ERR_ARG, "poly_rings not strictly ascending (a polygon needs a ring)");
    const uint32_t R0 = ring_of(poly_rings, 0), R1 = ring_of(poly_rings, npoly);
    for (uint32_t j = R0; j < R1; j++)
        if (ring_off[j + 1] < ring_off[j]) return ctx_fail(ctx, GEOHIP_ERR_ARG, "ring_off not ascending");
    if (ring_off[R1] > nv) return ctx_fail(ctx, GEOHIP_ERR_ARG, "ring_off refers past the nv vertices of vx / vy");
    // polygon planning (host): rings (createPolygon), envelope, G / C rectangles (plan.cpp), the
    // (polygon, tile) work items of each polygon's walk region and the slab lists -- or the
    // cached plan of the same inputs
    PolyCache* pc = ctx_pcache(ctx);
    bool cached = same_inputs(*pc, *grid, r, poly_rings, ring_off, npoly, vx, vy) && pc->jmode == jmode &&
                  pc->approx == (approximate ? 1 : 0) && memcmp(&pc->gq, gq, sizeof *gq) == 0;
    if (!cached) {
        PolyCache fresh;
        std::vector<PolyDev>& pd = fresh.pd;
        std::vector<double>& hvx = fresh.hvx;
        std::vector<double>& hvy = fresh.hvy;
        std::vector<int32_t>& hrects = fresh.hrects;
        std::vector<PolyWork>& hwork = fresh.hwork;
        std::vector<uint16_t>& hslab = fresh.hslab;
        bool& any_outside = fresh.any_outside;
        pd.resize(npoly);
        for (uint32_t p = 0; p < npoly; p++) {
            PolyPlan pl;
            std::string err;
            const uint32_t r0 = ring_of(poly_rings, p), r1 = ring_of(poly_rings, p + 1);
            if (r1 - r0 > kMaxRings) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "polygon with more than 65535 rings");
            rc = plan_polygon_rings(*gq, ring_off + r0, r1 - r0, vx, vy, r, &pl, &err);
            if (rc) return ctx_fail(ctx, rc, err);
            PolyDev& P = pd[p];
            memset(&P, 0, sizeof P);
            P.voff = (uint32_t)hvx.size();
            P.nv = (uint32_t)pl.rx.size();
            P.nring = (uint32_t)pl.ring_start.size() - 1;
            P.eoff = (uint32_t)(fresh.henv.size() / 4);
            hvx.insert(hvx.end(), pl.rx.begin(), pl.rx.end());
            hvy.insert(hvy.end(), pl.ry.begin(), pl.ry.end());
            ring_tables(pl, fresh.hvr, fresh.henv, P.gb);
            for (int i = 0; i < 4; i++) P.bb[i] = pl.bbox[i];
            P.goff = (uint32_t)(hrects.size() / 4);
            P.ng = (uint32_t)pl.g.size();
            int32_t wx0 = INT32_MAX, wx1 = INT32_MIN, wy0 = INT32_MAX, wy1 = INT32_MIN;
            auto acc = [&](const geohip_rect& q) {
                const int32_t a0 = std::max(q.x0, 0), a1 = std::min(q.x1, nb - 1);
                const int32_t c0 = std::max(q.y0, 0), c1 = std::min(q.y1, nb - 1);
                if (q.x0 < 0 || q.y0 < 0 || q.x1 > nb - 1 || q.y1 > nb - 1) P.outside = 1;
                if (a0 > a1 || c0 > c1) return;
                wx0 = std::min(wx0, a0); wx1 = std::max(wx1, a1);
                wy0 = std::min(wy0, c0); wy1 = std::max(wy1, c1);
            };
            for (auto& q : pl.g) { hrects.insert(hrects.end(), {q.x0, q.x1, q.y0, q.y1}); acc(q); }
            P.coff = (uint32_t)(hrects.size() / 4);
            P.nc = (uint32_t)pl.c.size();
            for (auto& q : pl.c) { hrects.insert(hrects.end(), {q.x0, q.x1, q.y0, q.y1}); acc(q); }
            P.wx0 = wx0; P.wx1 = wx1; P.wy0 = wy0; P.wy1 = wy1;
            any_outside = any_outside || P.outside;
            // the C rects follow the G rects: the join sees one list, all checked or all emitted
            if (jmode == 1) { P.coff = P.goff; P.nc += P.ng; P.ng = 0; }
            if (jmode == 2) { P.ng += P.nc; P.nc = 0; }
            plan_slabs(P, pl.ry.data(), P.nring > 1 ? fresh.hvr.data() + P.voff : nullptr, r, gq->cell_len, hslab);
            P.cls = kNoCls;
        }
        // the cell classes (exact modes): polygons in parallel on the host's cores (the refined
        // parts of a mixed subcell cost 16 box classifications each: 0.6 s on one core for C4's
        // 3000 polygons), each into its own tables, then concatenated in polygon order
        if (!approximate && npoly) {
            struct Cls {
                std::vector<uint32_t> blob, rf, rfw, rfw2;
                uint32_t off = kNoCls;
            };
            std::vector<Cls> part(npoly);
            std::atomic<uint32_t> next{0};
            auto work = [&]() {
                for (uint32_t p; (p = next.fetch_add(1)) < npoly;) {
                    const PolyDev& P = pd[p];
                    classify_cells(P, hvx, hvy, P.nring > 1 ? fresh.hvr.data() + P.voff : nullptr, *grid, hrects.data(),
                                   P.coff, P.nc, P.nring, r, part[p].blob, &part[p].off, &part[p].rf, &part[p].rfw, &part[p].rfw2);
                }
            };
            const unsigned nth = std::min<unsigned>(std::max(1u, std::min(std::thread::hardware_concurrency(), 16u)),
                                                    std::max<uint32_t>(1u, npoly / 8));
            std::vector<std::thread> th;
            for (unsigned t = 1; t < nth; t++) try {
                th.emplace_back(work);
            } catch (...) {  // no more threads (RLIMIT_NPROC, a container): this one does the rest
                break;
            }
            work();
            for (auto& t : th) t.join();
            for (uint32_t p = 0; p < npoly; p++) {
                Cls& q = part[p];
                if (q.off == kNoCls) continue;
                const uint32_t wbase = (uint32_t)(fresh.hrfw.size() / 2), w2base = (uint32_t)fresh.hrfw2.size();
                pd[p].cls = (uint32_t)fresh.hcls.size();
                fresh.hcls.insert(fresh.hcls.end(), q.blob.begin(), q.blob.end());
                for (size_t k = 0; k < q.rf.size(); k += 2) {  // (first word, class word) pairs
                    fresh.hrf.push_back(q.rf[k] == kNoRefine ? kNoRefine : q.rf[k] + wbase);
                    fresh.hrf.push_back(q.rf[k + 1]);
                }
                for (size_t k = 0; k < q.rfw.size(); k += 2) {  // (part word, first second-level word) pairs
                    fresh.hrfw.push_back(q.rfw[k]);
                    fresh.hrfw.push_back(q.rfw[k + 1] == kNoRefine ? kNoRefine : q.rfw[k + 1] + w2base);
                }
                fresh.hrfw2.insert(fresh.hrfw2.end(), q.rfw2.begin(), q.rfw2.end());
                std::vector<uint32_t>().swap(q.blob);
            }
        }
        for (uint32_t p = 0; p < npoly; p++) {
            const PolyDev& P = pd[p];
            if (P.wx0 <= P.wx1 && P.wy0 <= P.wy1)
                for (int32_t a = P.wx0 / geo.ts; a <= P.wx1 / geo.ts; a++)
                    for (int32_t c = P.wy0 / geo.ts; c <= P.wy1 / geo.ts; c++) {
                        const uint32_t t = tile_work(P, hrects.data(), fresh.hcls, geo, a, c, r >= 1.7976931348623157e308);
                        if (t != kNoWork) hwork.push_back(PolyWork{p, (uint32_t)a * (uint32_t)geo.nt + (uint32_t)c | t});
                    }
        }

        if (fresh.hwork.size() >= 0x7fffffffull) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "too many polygon work items");
        // the cells any polygon can emit from: points elsewhere are dropped while binning
        if ((uint64_t)nb * (uint64_t)nb <= (1ull << 24)) {
            fresh.keep.assign(((uint64_t)nb * nb + 31) / 32, 0u);
            for (uint32_t p = 0; p < npoly; p++) {
                const PolyDev& P = pd[p];
                const int32_t ch = P.wy1 - P.wy0 + 1;
                for (uint32_t q = 0; q < P.ng + P.nc; q++) {
                    const int32_t* R = &hrects[4 * ((q < P.ng ? P.goff : P.coff) + (q < P.ng ? q : q - P.ng))];
                    const int32_t a0 = std::max(R[0], 0), a1 = std::min(R[1], nb - 1);
                    const int32_t c0 = std::max(R[2], 0), c1 = std::min(R[3], nb - 1);
                    for (int32_t a = a0; a <= a1; a++)
                        for (int32_t c = c0; c <= c1; c++) {
                            // a C cell none of whose points can be within r is not needed by P
                            // (a cell in P's G as well is kept by the G rectangle's own pass)
                            if (q >= P.ng && P.cls != kNoCls &&
                                fresh.hcls[P.cls + (size_t)(a - P.wx0) * ch + (c - P.wy0)] == kWordMiss)
                                continue;
                            const uint64_t k = (uint64_t)a * nb + c;
                            fresh.keep[k >> 5] |= 1u << (k & 31);
                        }
                }
            }
        }
        build_stream_table(fresh, npoly, nb, r >= 1.7976931348623157e308);
        fresh.grid = *grid;
        fresh.gq = *gq;
        fresh.jmode = jmode;
        fresh.approx = approximate ? 1 : 0;
        fresh.r = r;
        fresh.poly_rings.resize((size_t)npoly + 1);
        for (uint32_t p = 0; p <= npoly; p++) fresh.poly_rings[p] = ring_of(poly_rings, p);
        fresh.ring_off.assign(ring_off + R0, ring_off + R1 + 1);
        fresh.vx.assign(vx + ring_off[R0], vx + ring_off[R1]);
        fresh.vy.assign(vy + ring_off[R0], vy + ring_off[R1]);
        *pc = std::move(fresh);
    }
    const std::vector<PolyDev>& pd = pc->pd;
    const std::vector<double>& hvx = pc->hvx;
    const std::vector<double>& hvy = pc->hvy;
    const std::vector<int32_t>& hrects = pc->hrects;
    const std::vector<PolyWork>& hwork = pc->hwork;
    const std::vector<uint16_t>& hslab = pc->hslab;
    const std::vector<ring_id_t>& hvr = pc->hvr;
    const std::vector<double>& henv = pc->henv;
    const bool any_outside = pc->any_outside;
    const std::vector<uint32_t>& keep = pc->keep;
    const std::vector<uint32_t>& hcls = pc->hcls;
    Scratch S{ctx};
    const double *dx, *dy;
    rc = ctx_stage_xy(ctx, x, y, n, 0, &dx, &dy);
    if (rc) return rc;
    const auto t_planned = now();
    // polygon tables in one device blob:
    //   PolyDev[] | vx | vy | ring envelopes | rects | work | slab lists | keep | ring ids | classes
    const size_t sz_p = npoly * sizeof(PolyDev), sz_v = hvx.size() * 8, sz_r = hrects.size() * 4;
    const size_t sz_w = hwork.size() * sizeof(PolyWork), sz_s = hslab.size() * 2, sz_k = keep.size() * 4;
    const size_t sz_e = henv.size() * 8, sz_vr = hvr.size() * sizeof(ring_id_t);
    const size_t off_v = (sz_p + 15) & ~(size_t)15;
    const size_t off_e = off_v + 2 * sz_v;
    const size_t off_r = off_e + sz_e;
    const size_t off_w = (off_r + sz_r + 15) & ~(size_t)15;
    const size_t off_s = (off_w + sz_w + 15) & ~(size_t)15;
    const size_t off_k = (off_s + sz_s + 15) & ~(size_t)15;
    const size_t off_vr = (off_k + sz_k + 15) & ~(size_t)15;
    const size_t off_cl = (off_vr + sz_vr + 15) & ~(size_t)15, sz_cl = hcls.size() * 4;
    // streaming-path tables (empty unless stream_ok)
    const size_t off_co = (off_cl + sz_cl + 15) & ~(size_t)15, sz_co = pc->cell_head.size() * 4;
    const size_t off_ce = (off_co + sz_co + 15) & ~(size_t)15, sz_ce = pc->cell_ent.size() * 4;
    const size_t off_sk = (off_ce + sz_ce + 15) & ~(size_t)15, sz_sk = pc->skeep.size() * 4;
    const size_t off_op = (off_sk + sz_sk + 15) & ~(size_t)15, sz_op = pc->opoly.size() * 4;
    const size_t off_rf = (off_op + sz_op + 15) & ~(size_t)15, sz_rf = pc->hrf.size() * 4;
    const size_t off_rw = (off_rf + sz_rf + 15) & ~(size_t)15, sz_rw = pc->hrfw.size() * 4;
    const size_t off_r2 = (off_rw + sz_rw + 15) & ~(size_t)15, sz_r2 = pc->hrfw2.size() * 4;
    const size_t blob_end = off_r2 + (sz_r2 ? sz_r2 : 16);  // >= one readable word (unconditional gathers)
    void* pblob = nullptr;
    rc = ctx_ensure(ctx, J_POLY, blob_end + 64, &pblob);
    if (rc) return rc;
    const bool upload = !(cached && pc->dev_blob == pblob && pc->blob_bytes == blob_end);
    char* bp = reinterpret_cast<char*>(pblob);
    PolyDev* dpoly = reinterpret_cast<PolyDev*>(bp);
    double* dvx = reinterpret_cast<double*>(bp + off_v);
    double* dvy = dvx + hvx.size();
    int32_t* drects = reinterpret_cast<int32_t*>(bp + off_r);
    PolyWork* dwork = reinterpret_cast<PolyWork*>(bp + off_w);
    uint16_t* dslab = reinterpret_cast<uint16_t*>(bp + off_s);
    unsigned* dkeep = sz_k ? reinterpret_cast<unsigned*>(bp + off_k) : nullptr;
    double* denv = reinterpret_cast<double*>(bp + off_e);
    ring_id_t* dvr = reinterpret_cast<ring_id_t*>(bp + off_vr);
    uint32_t* dcls = reinterpret_cast<uint32_t*>(bp + off_cl);
    uint2* dchead = reinterpret_cast<uint2*>(bp + off_co);
    uint2* dcent = reinterpret_cast<uint2*>(bp + off_ce);
    unsigned* dskeep = reinterpret_cast<unsigned*>(bp + off_sk);
    uint32_t* dopoly = reinterpret_cast<uint32_t*>(bp + off_op);
    uint2* drf = reinterpret_cast<uint2*>(bp + off_rf);
    uint2* drfw = reinterpret_cast<uint2*>(bp + off_rw);
    uint32_t* drfw2 = reinterpret_cast<uint32_t*>(bp + off_r2);
    if (upload) {
        pc->dev_blob = nullptr;  // until the copies are issued
        if ((sz_p && hipMemcpyAsync(dpoly, pd.data(), sz_p, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_v && hipMemcpyAsync(dvx, hvx.data(), sz_v, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_v && hipMemcpyAsync(dvy, hvy.data(), sz_v, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_r && hipMemcpyAsync(drects, hrects.data(), sz_r, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_w && hipMemcpyAsync(dwork, hwork.data(), sz_w, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_s && hipMemcpyAsync(dslab, hslab.data(), sz_s, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_k && hipMemcpyAsync(dkeep, keep.data(), sz_k, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_e && hipMemcpyAsync(denv, henv.data(), sz_e, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_vr && hipMemcpyAsync(dvr, hvr.data(), sz_vr, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_cl && hipMemcpyAsync(dcls, hcls.data(), sz_cl, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_co && hipMemcpyAsync(dchead, pc->cell_head.data(), sz_co, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_ce && hipMemcpyAsync(dcent, pc->cell_ent.data(), sz_ce, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_sk && hipMemcpyAsync(dskeep, pc->skeep.data(), sz_sk, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_op && hipMemcpyAsync(dopoly, pc->opoly.data(), sz_op, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_rf && hipMemcpyAsync(drf, pc->hrf.data(), sz_rf, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_rw && hipMemcpyAsync(drfw, pc->hrfw.data(), sz_rw, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (sz_r2 && hipMemcpyAsync(drfw2, pc->hrfw2.data(), sz_r2, hipMemcpyHostToDevice, st) != hipSuccess))
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "polygon upload failed");
        pc->dev_blob = pblob;
        pc->blob_bytes = blob_end;
    }
    static const int force_tiles = getenv("GEOHIP_PPOLY_TILES") ? atoi(getenv("GEOHIP_PPOLY_TILES")) : 0;  // A/B only
    if (pc->stream_ok && !force_tiles) {
        unsigned* out = nullptr;
        if (cap) {
            if (dev) {
                out = out_pairs;
            } else {
                void* p = nullptr;
                rc = ctx_ensure(ctx, J_OUT, cap * 8, &p);
                if (rc) return rc;
                out = reinterpret_cast<unsigned*>(p);
            }
        }
        const bool cands = !approximate && jmode != 2;
        uint64_t ccap = std::max<uint64_t>(std::max<uint64_t>(65536, n / 16), pc->last_cand + pc->last_cand / 4);
        uint64_t tot = 0;
        const uint64_t nchunks = (n + kStreamChunk - 1) / kStreamChunk;
        unsigned* fault = nullptr;  // async: a candidate overflow surfaces at geohip_ctx_sync
        if (async) {
            rc = ctx_fault_block(ctx, &fault);
            if (rc) return rc;
        }
        {
            // one pass: the chunks whose candidates pass ccap (or fill a wave's spill list) are
            // decided by ppoly_stream_redo; the count they needed sizes the next call's buffer
            // J_MISC: [0..1] pair total, [2..3] candidate total, [4] work items, [5] early wave
            // flushes, [6] eval ticket, [7] chunks queued for the redo pass
            unsigned* misc = S.get<unsigned>(J_MISC, kMiscWords * 4);
            unsigned* mat = cands ? S.get<unsigned>(J_HIST, ((size_t)kCandGroups + 2) * npoly * 4 + 16) : nullptr;
            void* cbuf = cands ? S.get<void>(J_SY, ccap * 36 + 64) : nullptr;
            const bool refine = cands && !pc->hrfw.empty();
            void* sbuf = cands ? S.get<void>(J_SX, ccap * 4 + 64) : nullptr;
            uint4* items = cands ? S.get<uint4>(J_SKEY, (ccap / kCandItem + npoly + 1) * sizeof(uint4)) : nullptr;
            if (S.rc) return S.rc;
            hipEvent_t e0, e1;
            ctx_timing_events(ctx, &e0, &e1);
            if (e0) hipEventRecord(e0, st);  // the whole device step
            // totals and the item count (async: the pair total is the caller's device word)
            unsigned* ptot = cands ? mat + (size_t)kCandGroups * npoly : nullptr;  // then pcur
            tlaunch(ctx, zero_step, 1, kTB, 0, st, misc, 8u,
                    async ? reinterpret_cast<unsigned long long*>(count_dev) : (unsigned long long*)nullptr, ptot,
                    cands ? npoly : 0u);
            StreamOut so;
            so.out = out;
            so.cap = out ? cap : 0;
            so.aligned8 = ((uintptr_t)out & 7u) == 0;
            so.swap = join ? 1 : 0;
            so.point_base = point_base;
            so.flushes = misc + 5;  // zeroed with the totals
            so.ptotal = async ? reinterpret_cast<unsigned long long*>(count_dev) : reinterpret_cast<unsigned long long*>(misc);
            so.ctotal = reinterpret_cast<unsigned long long*>(misc) + 1;
            so.ccap = cands ? ccap : 0;
            char* cb = reinterpret_cast<char*>(cbuf);
            so.cpoly = cands ? reinterpret_cast<unsigned*>(cb) : nullptr;
            so.crec = cands ? reinterpret_cast<double4*>(cb + ((ccap * 4 + 31) & ~(uint64_t)31)) : nullptr;
            // per wave, the spill list holds its chunk points x the most entries a point meets (a
            // cell's, or the polygons reaching outside the grid), up to kSpillEnt entries per point
            // (<= 128 MB in all); a wave whose candidates exceed it sends its chunk to the redo pass
            const unsigned stream_blocks =
                (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nchunks, (uint64_t)ctx_cus(ctx) * kStreamBlocksPerCU));
            const uint32_t ment = std::max<uint32_t>(1u, std::max<uint32_t>(pc->max_cell_ent, (uint32_t)pc->opoly.size()));
            so.covf_wave = cands ? (kStreamChunk / kStreamNW) * std::min<uint32_t>(ment, kSpillEnt) : 0u;
            const size_t covf_words = (size_t)stream_blocks * kStreamNW * so.covf_wave;
            unsigned* cov = cands ? S.get<unsigned>(J_COVF, (covf_words + nchunks + 64) * 4) : nullptr;
            if (S.rc) return S.rc;
            so.covf = cov;
            so.redo = cands ? cov + covf_words : nullptr;
            so.nredo = misc + 7;  // zeroed with the totals
            StreamArgs sa;
            sa.x = dx;
            sa.y = dy;
            sa.n = n;
            sa.g = geo;
            sa.keep = sz_sk ? dskeep : nullptr;
            sa.keep_words = (unsigned)pc->skeep.size();
            sa.head = dchead;
            sa.ent = dcent;
            sa.polys = dpoly;
            sa.opoly = dopoly;
            sa.nopoly = (uint32_t)pc->opoly.size();
            sa.rects = drects;
            sa.jmode = jmode;
            sa.r = r;
            sa.o = so;
            sa.vx = dvx;
            sa.vy = dvy;
            sa.vring = dvr;
            sa.renv = denv;
            sa.slabs = dslab;
            if (nchunks) {
                const unsigned nblk = stream_blocks;
                // the cell bitmap staged in LDS (from global memory: 516 against 460 us; none: 487)
                const bool kl = sa.keep && sa.keep_words <= kKeepLds;
                if (approximate) {
                    if (kl) tlaunch(ctx, ppoly_stream<true, true>, nblk, kStreamNW * kWave, 0, st, sa);
                    else tlaunch(ctx, ppoly_stream<true, false>, nblk, kStreamNW * kWave, 0, st, sa);
                } else {
                    if (kl) tlaunch(ctx, ppoly_stream<false, true>, nblk, kStreamNW * kWave, 0, st, sa);
                    else tlaunch(ctx, ppoly_stream<false, false>, nblk, kStreamNW * kWave, 0, st, sa);
                }
                if (cands) {  // the chunks whose candidates did not fit (an empty list: blocks exit at once)
                    if (kl) tlaunch(ctx, ppoly_stream_redo<true>, nblk, kStreamNW * kWave, 0, st, sa);
                    else tlaunch(ctx, ppoly_stream_redo<false>, nblk, kStreamNW * kWave, 0, st, sa);
                }
            }
            if (cands) {
                char* sb = reinterpret_cast<char*>(sbuf);
                CandGroup cg;
                cg.ccount = so.ctotal;
                cg.cstream = so.ctotal;
                cg.cpoly = so.cpoly;
                cg.crec = so.crec;
                if (refine) {  // the candidates' refined parts first: decided ones leave the grouping
                    CandRefine cr;
                    cr.ccount = so.ctotal;
                    cr.ccap = ccap;
                    cr.cpoly = so.cpoly;
                    cr.crec = so.crec;
                    cr.polys = dpoly;
                    cr.rf = drf;
                    cr.rfw = drfw;
                    cr.rfw2 = drfw2;
                    cr.mnx = grid->min_x;
                    cr.mny = grid->min_y;
                    cr.l = grid->cell_len;
                    tlaunch(ctx, ppoly_cand_refine, kRefineBlocks, kTB, 0, st, cr, so);
                }
                cg.ccap = ccap;
                cg.fault = fault;
                cg.need = fault ? reinterpret_cast<unsigned long long*>(fault + 2) : nullptr;
                cg.mat = mat;
                cg.ptot = ptot;
                cg.pcur = ptot + npoly;
                cg.npoly = npoly;
                cg.items = items;
                cg.nitems = misc + 4;
                cg.eticket = misc + 6;
                cg.sidx = reinterpret_cast<unsigned*>(sb);
                tlaunch(ctx, ppoly_cand_hist, kCandGroups, kCandThreads, 0, st, cg);
                tlaunch(ctx, ppoly_cand_plan, 1, kCandThreads, 0, st, cg);
                tlaunch(ctx, ppoly_cand_scatter, kCandGroups, kCandThreads, 0, st, cg);
                tlaunch(ctx, ppoly_cand_eval, kEvalBlocks, kTB, 0, st, cg, dpoly, dvx, dvy, dvr, denv, dslab, r, so);
            }
            if (e1) hipEventRecord(e1, st);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("ppoly stream launch: ") + hipGetErrorString(e));
            if (async) return GEOHIP_OK;  // pairs counted into *count_dev; an overflow at geohip_ctx_sync
            uint64_t* pin = ctx_pinned(ctx);
            if (hipMemcpyAsync(pin, misc, 32, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
                return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "count readback failed");
            tot = pin[0];
            const uint64_t ncand = pin[1];
            pc->last_cand = ncand;
            if (prof)
                fprintf(stderr, "ppoly host: plan %.1f us (cached %d), %zu refined cells, class table %zu cells\n",
                        std::chrono::duration<double, std::micro>(t_planned - t_start).count(), (int)cached,
                        (size_t)std::count_if(pc->hrf.begin(), pc->hrf.end(), [](uint32_t v) { return v != kNoRefine; }) / 2,
                        pc->hcls.size());
            if (prof)
                fprintf(stderr, "ppoly host: refinement words %zu (parts) + %zu (sub-parts)\n", pc->hrfw.size() / 2,
                        pc->hrfw2.size());
            if (prof) fprintf(stderr, "ppoly stream: %llu pairs, %llu candidates (capacity %llu: %llu past it), "
                              "%u early wave flushes, %u of %llu chunks decided by the redo pass, one pass\n",
                              (unsigned long long)tot, (unsigned long long)ncand, (unsigned long long)ccap,
                              (unsigned long long)(ncand > ccap ? ncand - ccap : 0), (unsigned)(pin[2] >> 32),
                              (unsigned)(pin[3] >> 32), (unsigned long long)nchunks);
        }
        *out_count = tot;
        if (!dev && cap) {
            const uint64_t m = std::min<uint64_t>(tot, cap);
            if (m && hipMemcpy(out_pairs, out, m * 8, hipMemcpyDeviceToHost) != hipSuccess)
                return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "pair readback failed");
        }
        if (tot > cap) return ctx_fail(ctx, GEOHIP_ERR_CAPACITY, "output capacity too small; *out_count = required");
        return GEOHIP_OK;
    }
    hipEvent_t e0, e1;
    ctx_timing_events(ctx, &e0, &e1);
    if (e0) hipEventRecord(e0, st);  // the whole device step: binning, mask sizing, count and write passes
    TileBins tb;
    unsigned* oidx = nullptr;
    unsigned n_out = 0;
    rc = bin_tiles(ctx, S, dx, dy, n, geo, any_outside, &tb, &oidx, any_outside ? &n_out : nullptr, dkeep);
    if (rc) return rc;
    const auto t_binned = now();
    const unsigned nwork = (unsigned)hwork.size();
    const unsigned nob = (any_outside && n_out) ? (npoly < 4096u ? npoly : 4096u) : 0u;
    const uint64_t nslots = (uint64_t)nwork + nob;
    const uint64_t nscan = std::max<uint64_t>(nslots, nwork);
    unsigned* misc = S.get<unsigned>(J_MISC, kMiscWords * 4);
    unsigned* seg = S.get<unsigned>(J_SEG, ((nscan + kScanSeg - 1) / kScanSeg + 1) * 8 + 64);
    unsigned long long* bcount = S.get<unsigned long long>(J_BCNT, (nslots + 1) * 8);
    unsigned long long* boff = S.get<unsigned long long>(J_BOFF, (nslots + 1) * 8);
    unsigned long long* words = S.get<unsigned long long>(J_QLIST, ((uint64_t)nwork + 1) * 8);
    unsigned long long* wofs = S.get<unsigned long long>(J_QSTART, ((uint64_t)nwork + 1) * 8);
    if (S.rc) return S.rc;
    // hit-mask layout: words per work item, scanned; the total sizes the mask (one readback)
    uint64_t nmask = 0;
    if (nwork) {
        if (prof) {
            size_t nc[3] = {0, 0, 0};
            for (uint32_t v : hcls) nc[v == kWordHit ? 1 : v == kWordMiss ? 2 : 0]++;
            fprintf(stderr, "ppoly host: cell classes mixed %zu hit %zu miss %zu (region cells incl. non-C)\n", nc[0], nc[1], nc[2]);
        }
        if (prof) fprintf(stderr, "ppoly host: plan %.1f us (cached %d), bin launch %.1f us, upload %.1f us\n",
                          std::chrono::duration<double, std::micro>(t_planned - t_start).count(), (int)cached,
                          std::chrono::duration<double, std::micro>(t_binned - t_planned).count(),
                          std::chrono::duration<double, std::micro>(now() - t_binned).count());
        ppoly_words<<<(nwork + kTB - 1) / kTB, kTB, 0, st>>>(dwork, nwork, tb.start, words);
        scan_launch<unsigned long long>(st, words, nwork, reinterpret_cast<unsigned long long*>(seg),
                                        reinterpret_cast<unsigned long long*>(misc + 8), wofs);
        rc = read_total(ctx, wofs + nwork, &nmask);
        if (rc) return rc;
    }
    unsigned long long* mask = S.get<unsigned long long>(J_PMASK, nmask * 8 + 8);
    if (S.rc) return S.rc;
    if (nmask && hipMemsetAsync(mask, 0, nmask * 8, st) != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    unsigned* out = nullptr;
    if (cap) {
        if (dev) {
            out = out_pairs;
        } else {
            void* p = nullptr;
            rc = ctx_ensure(ctx, J_OUT, cap * 8, &p);
            if (rc) return rc;
            out = reinterpret_cast<unsigned*>(p);
        }
    }
    PairSink sink{bcount, boff, 0u, out, out ? cap : 0, ((uintptr_t)out & 7u) == 0, join ? 1 : 0, point_base};
    PairSink osink = sink;
    osink.slot0 = nwork;
    const int r_is_max = r >= 1.7976931348623157e308;
    if (hipMemsetAsync(bcount, 0, (nslots + 1) * 8, st) != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    // count pass: hit masks + per-work-item counts; out-of-grid points counted separately
    if (nwork) {
        if (approximate)
            ppoly_eval<true><<<nwork, kTB, 0, st>>>(tb, dwork, dpoly, dvx, dvy, dvr, denv, drects, dslab, dcls, r, r_is_max, wofs, mask, bcount);
        else
            ppoly_eval<false><<<nwork, kTB, 0, st>>>(tb, dwork, dpoly, dvx, dvy, dvr, denv, drects, dslab, dcls, r, r_is_max, wofs, mask, bcount);
    }
    if (nob && jmode == 1)
        ppoly_outside<false, true><<<nob, kTB, 0, st>>>(dx, dy, oidx, n_out, grid->min_x, grid->min_y, grid->cell_len,
                                                        dpoly, npoly, drects, osink, dvx, dvy, dslab, r, dvr, denv);
    else if (nob)
        ppoly_outside<false><<<nob, kTB, 0, st>>>(dx, dy, oidx, n_out, grid->min_x, grid->min_y, grid->cell_len, dpoly,
                                                  npoly, drects, osink);
    scan_launch<unsigned long long>(st, bcount, nslots, reinterpret_cast<unsigned long long*>(seg),
                                    reinterpret_cast<unsigned long long*>(misc + 8), boff);
    // write pass: pairs from the masks
    if (out) {
        if (nwork) ppoly_emit<<<nwork, kTB, 0, st>>>(tb, dwork, wofs, mask, sink);
        if (nob && jmode == 1)
            ppoly_outside<true, true><<<nob, kTB, 0, st>>>(dx, dy, oidx, n_out, grid->min_x, grid->min_y,
                                                           grid->cell_len, dpoly, npoly, drects, osink, dvx, dvy, dslab, r,
                                                           dvr, denv);
        else if (nob)
            ppoly_outside<true><<<nob, kTB, 0, st>>>(dx, dy, oidx, n_out, grid->min_x, grid->min_y, grid->cell_len, dpoly,
                                                     npoly, drects, osink);
    }
    if (e1) hipEventRecord(e1, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("ppoly launch: ") + hipGetErrorString(e));
    unsigned long long* total = boff + nslots;
    if (async) {  // the tile-binned path read its mask size back already; the total stays on the device
        if (hipMemcpyAsync(count_dev, total, 8, hipMemcpyDeviceToDevice, st) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "count copy failed");
        return GEOHIP_OK;
    }
    uint64_t tot = 0;
    rc = read_total(ctx, total, &tot);
    if (rc) return rc;
    *out_count = tot;
    if (!dev && cap) {
        const uint64_t m = std::min<uint64_t>(tot, cap);
        if (m && hipMemcpy(out_pairs, out, m * 8, hipMemcpyDeviceToHost) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "pair readback failed");
    }
    if (tot > cap) return ctx_fail(ctx, GEOHIP_ERR_CAPACITY, "output capacity too small; *out_count = required");
    return GEOHIP_OK;
}

// Large-k selection tail shared by the point and point-polygon kNN: the 9 radix rounds over the
// candidate keys, the gather of exactly min(k, M) keys into sel (pre-filled with sentinels), the
// (dist, idx) sort of the k entries into od / oi, and the count.  The candidate scan and key
// kernels ran before on st.
int rsel_large_tail(hipStream_t st, const unsigned long long* key, const unsigned* cand, RselState* rs, unsigned k,
                    unsigned long long* sel_d, unsigned* sel_i, unsigned long long* tmp_d, unsigned* tmp_i, void* temp,
                    size_t temp_bytes, double* od, unsigned* oi, unsigned* ocnt) {
    for (int t = 0; t < kRselRounds; t++) {
        rsel_hist<<<512, kTB, 0, st>>>(key, cand, rs, t, k);
        rsel_pick<<<1, 1024, 0, st>>>(rs, t, k);
    }
    rsel_gather<<<512, kTB, 0, st>>>(key, cand, rs, k, sel_d, sel_i);
    hipError_t e = sort_dist_idx(temp, temp_bytes, sel_d, sel_i, tmp_d, tmp_i,
                                 reinterpret_cast<unsigned long long*>(od), oi, k, st);
    if (e != hipSuccess) return GEOHIP_ERR_DEVICE;
    rsel_count<<<1, 64, 0, st>>>(rs, k, ocnt);
    return hipGetLastError() == hipSuccess ? GEOHIP_OK : GEOHIP_ERR_DEVICE;
}

// Scratch of a large-k selection in slot 23: RselState | sel (k) | tmp (k) | sort temp.
struct LargeK {
    RselState* rs;
    unsigned long long *sel_d, *tmp_d;
    unsigned *sel_i, *tmp_i;
    void* temp;
    size_t temp_bytes;
    char* extra;  // caller's area after the sort temp (extra_bytes)
};
int large_k_scratch(geohip_ctx* ctx, unsigned k, size_t extra_bytes, LargeK* L) {
    const size_t a16 = 255;
    L->temp_bytes = sort_dist_idx_temp_bytes(k);
    if (!L->temp_bytes) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "sort temp size query failed");
    const size_t off_sel = (sizeof(RselState) + a16) & ~a16;
    const size_t off_tmp = (off_sel + (size_t)k * 12 + a16) & ~a16;
    const size_t off_temp = (off_tmp + (size_t)k * 12 + a16) & ~a16;
    const size_t off_extra = (off_temp + L->temp_bytes + a16) & ~a16;
    void* p = nullptr;
    int rc = ctx_ensure(ctx, J_KTEMP, off_extra + extra_bytes + 64, &p);
    if (rc) return rc;
    char* b = reinterpret_cast<char*>(p);
    L->rs = reinterpret_cast<RselState*>(b);
    L->sel_d = reinterpret_cast<unsigned long long*>(b + off_sel);
    L->sel_i = reinterpret_cast<unsigned*>(b + off_sel + (size_t)k * 8);
    L->tmp_d = reinterpret_cast<unsigned long long*>(b + off_tmp);
    L->tmp_i = reinterpret_cast<unsigned*>(b + off_tmp + (size_t)k * 8);
    L->temp = b + off_temp;
    L->extra = b + off_extra;
    return GEOHIP_OK;
}

// Point kNN with k > GEOHIP_KNN_MAX_K (PointPointKNNQuery.java:33 takes any Integer k): the
// candidates of G u C compacted by one box-classifying pass, their keys, then the radix-select
// tail.  Same result as the one-pass kNN: the min(k, M) smallest (dist bits, idx), ascending.
int knn_pp_large_impl(geohip_ctx* ctx, const PointPlan& plan, const double* dx, const double* dy, uint64_t n,
                      double qx, double qy, uint32_t k, double* od, unsigned* oi, unsigned* ocnt) {
    hipStream_t st = ctx_stream(ctx);
    const uint64_t ncap = n ? n : 1;
    void* pc = nullptr;
    int rc = ctx_ensure(ctx, J_KCAND, ncap * 12 + 64, &pc);
    LargeK L;
    if (!rc) rc = large_k_scratch(ctx, k, 0, &L);
    if (rc) return rc;
    unsigned long long* key = reinterpret_cast<unsigned long long*>(pc);
    unsigned* cand = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(pc) + ncap * 8);
    hipEvent_t e0, e1;
    ctx_timing_events(ctx, &e0, &e1);
    if (e0) hipEventRecord(e0, st);
    rsel_init<<<1, 1024, 0, st>>>(L.rs, k, 0u);
    if (hipMemsetAsync(L.sel_d, 0xff, (size_t)k * 12, st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    if (n && plan.nu) {
        PpknnBoxes PB;
        memset(&PB, 0, sizeof PB);
        for (int q = 0; q < plan.nu; q++) PB.b[q] = plan.u[q];
        PB.nb = plan.nu;
        const uint64_t nb = std::max<uint64_t>(1, std::min<uint64_t>(((n + 255) / 256 + 3) / 4, 2048));
        switch (PB.nb) {
            case 1: ppknn_scan_boxes<1><<<(unsigned)nb, kTB, 0, st>>>(dx, dy, n, PB, cand, L.rs); break;
            case 2: ppknn_scan_boxes<2><<<(unsigned)nb, kTB, 0, st>>>(dx, dy, n, PB, cand, L.rs); break;
            default: ppknn_scan_boxes<0><<<(unsigned)nb, kTB, 0, st>>>(dx, dy, n, PB, cand, L.rs); break;
        }
        ppknn_pp_keys<<<1024, kTB, 0, st>>>(dx, dy, cand, L.rs, qx, qy, key);
    }
    rc = rsel_large_tail(st, key, cand, L.rs, k, L.sel_d, L.sel_i, L.tmp_d, L.tmp_i, L.temp, L.temp_bytes, od, oi, ocnt);
    if (rc) return ctx_fail(ctx, rc, "large-k kNN launch failed");
    if (e1) hipEventRecord(e1, st);
    return GEOHIP_OK;
}

// Rank merge of nlists sorted lists when k > 256 and the lists hold more than one workgroup
// sorts in LDS (KNNQuery.java:204-272 over any number of per-cell or per-rank results): every
// entry sorted by (dist, idx), the first k taken.
int knn_merge_large_impl(geohip_ctx* ctx, const unsigned long long* d, const unsigned* i, unsigned nlists,
                         unsigned list_len, unsigned k, double* od, unsigned* oi, unsigned* ocnt) {
    const uint64_t m64 = (uint64_t)nlists * list_len;
    if (m64 >= 0xffffffffull) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "merge of 2^32 or more entries");
    const unsigned m = (unsigned)m64;
    hipStream_t st = ctx_stream(ctx);
    const size_t tb = sort_dist_idx_temp_bytes(m ? m : 1);
    if (!tb) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "sort temp size query failed");
    const size_t mcap = (size_t)(m ? m : 1);
    void* p = nullptr;
    int rc = ctx_ensure(ctx, J_KCAND, mcap * 24 + tb + 512, &p);
    if (rc) return rc;
    char* b = reinterpret_cast<char*>(p);
    unsigned long long* tmp_d = reinterpret_cast<unsigned long long*>(b);
    unsigned long long* srt_d = tmp_d + mcap;
    unsigned* tmp_i = reinterpret_cast<unsigned*>(srt_d + mcap);
    unsigned* srt_i = tmp_i + mcap;
    void* temp = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(srt_i + mcap) + 255) & ~(uintptr_t)255);
    if (sort_dist_idx(temp, tb, d, i, tmp_d, tmp_i, srt_d, srt_i, m, st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "merge sort launch failed");
    topk_take<<<1, 1024, 0, st>>>(srt_d, srt_i, m, k, od, oi, ocnt);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("merge launch: ") + hipGetErrorString(e));
    return GEOHIP_OK;
}

// Point-polygon kNN polygon cache (one per ctx): a continuous PointPolygonKNNQuery evaluates the
// same polygon on every window, so its plan (rings, envelopes, G/C rectangles, boxes) is built and
// uploaded to a dedicated ctx slot once; later calls compare their inputs bitwise.  It also keeps
// the previous window's candidate count, which picks the selection path of the next window without
// a host round trip (either path is exact for any count; the guess only decides which is fast).
struct KnnPolyCache {
    bool valid = false;
    geohip_grid grid{};
    double r = 0.0;
    std::vector<uint32_t> ring_off;  // ring offsets relative to ring_off[0]
    std::vector<double> vx, vy;      // the rings' vertices as given
    PpknnPoly P;
    PpknnBoxes PB;
    bool boxed = false;
    uint32_t nrect = 0;
    size_t off_vx = 0, off_env = 0, off_rect = 0, off_vr = 0, blob_bytes = 0;
    size_t n_env = 0, n_vr = 0;
    void* dev_blob = nullptr;
    uint32_t* pin = nullptr;    // pinned: the last window's candidate count
    hipEvent_t ev = nullptr;    // ... landed when this event completes
    bool ev_pending = false;
    uint32_t last_m = 0;
};

KnnPolyCache* ctx_kcache(geohip_ctx* ctx) {
    void** slot = ctx_kcache_slot(ctx);
    if (!*slot) *slot = new KnnPolyCache();
    return static_cast<KnnPolyCache*>(*slot);
}

void knn_poly_cache_drop(geohip_ctx* ctx) {
    void** slot = ctx_kcache_slot(ctx);
    KnnPolyCache* c = static_cast<KnnPolyCache*>(*slot);
    if (!c) return;
    if (c->ev) {
        hipEventSynchronize(c->ev);
        hipEventDestroy(c->ev);
    }
    if (c->pin) hipHostFree(c->pin);
    delete c;
    *slot = nullptr;
}

// Point-polygon kNN of one query polygon over one window (host side of the kernels above).
int knn_ppoly_impl(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                   const uint32_t* ring_off, uint32_t nring, const double* vx, const double* vy, uint64_t nv, double r,
                   uint32_t k, int approximate, uint32_t* out_idx, double* out_dist, uint32_t* out_count, bool async) {
    if (!out_idx || !out_dist || !out_count) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null output");
    if (!async) *out_count = 0;
    if (k == 0) return ctx_fail(ctx, GEOHIP_ERR_ARG, "k must be > 0");
    // k above one workgroup's LDS sort (GEOHIP_KNN_PPOLY_MAX_K): the radix rounds always run,
    // the k selected keys are gathered and sorted (PointPolygonKNNQuery.java:34 takes any k)
    const bool big_k = k > GEOHIP_KNN_PPOLY_MAX_K;
    int rc = check_grid_basic(ctx, grid, "grid");
    if (rc) return rc;
    if (n >= 0xffffffffull) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "window larger than 2^32-1 points");
    if (!ring_off || !vx || !vy) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null polygon arrays");
    if (nring > kMaxRings) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "polygon with more than 65535 rings");
    for (uint32_t j = 0; j < nring; j++)
        if (ring_off[j + 1] < ring_off[j]) return ctx_fail(ctx, GEOHIP_ERR_ARG, "ring_off not ascending");
    if (ring_off[nring] > nv) return ctx_fail(ctx, GEOHIP_ERR_ARG, "ring_off refers past the nv vertices of vx / vy");
    hipStream_t st = ctx_stream(ctx);
    const bool dev = ctx_mem(ctx) == GEOHIP_MEM_DEVICE;
    KnnPolyCache* kc = ctx_kcache(ctx);
    // ---- the polygon's plan: cached, or built and uploaded once
    const size_t v0 = nring ? ring_off[0] : 0, v1 = nring ? ring_off[nring] : 0;
    bool same = kc->valid && memcmp(&kc->grid, grid, sizeof *grid) == 0 && memcmp(&kc->r, &r, sizeof r) == 0 &&
                kc->ring_off.size() == (size_t)nring + 1 && kc->vx.size() == v1 - v0;
    if (same)
        for (uint32_t j = 0; j <= nring && same; j++) same = kc->ring_off[j] == ring_off[j] - ring_off[0];
    if (same && v1 > v0)
        same = memcmp(kc->vx.data(), vx + v0, (v1 - v0) * 8) == 0 && memcmp(kc->vy.data(), vy + v0, (v1 - v0) * 8) == 0;
    if (!same) {
        kc->valid = false;
        PolyPlan pl;
        std::string err;
        rc = plan_polygon_rings(*grid, ring_off, nring, vx, vy, r, &pl, &err);
        if (rc) return ctx_fail(ctx, rc, err);
        std::vector<ring_id_t> hvr;
        std::vector<double> henv;
        double gb[4];
        ring_tables(pl, hvr, henv, gb);
        std::vector<int32_t> hrect;
        for (auto& q : pl.g) hrect.insert(hrect.end(), {q.x0, q.x1, q.y0, q.y1});
        for (auto& q : pl.c) hrect.insert(hrect.end(), {q.x0, q.x1, q.y0, q.y1});
        const uint32_t nrect = (uint32_t)(hrect.size() / 4);
        // exact coordinate boxes of the rects (no division in the scan) when they fit the kernel args
        PpknnBoxes PB;
        memset(&PB, 0, sizeof PB);
        const bool boxed = nrect <= (uint32_t)kPpBoxes;
        if (boxed) {
            for (uint32_t q = 0; q < nrect; q++) {
                const geohip_rect rr{hrect[4 * q], hrect[4 * q + 1], hrect[4 * q + 2], hrect[4 * q + 3]};
                PB.b[q] = rect_to_box(*grid, rr);
            }
            PB.nb = (int32_t)nrect;
        }
        PpknnPoly P;
        memset(&P, 0, sizeof P);
        for (int i = 0; i < 4; i++) P.bb[i] = pl.bbox[i];
        P.nv = (uint32_t)pl.rx.size();
        P.nrect = nrect;
        P.nring = (uint32_t)pl.ring_start.size() - 1;
        // device tables in slot 24 (only this path writes it): vx | vy | ring envelopes | rects | ring ids
        const size_t off_vx = 0;
        const size_t off_env = off_vx + 2 * 8 * (size_t)P.nv;
        const size_t off_rect = off_env + 8 * henv.size();
        const size_t off_vr = off_rect + 16 * (size_t)nrect;
        const size_t blob = off_vr + hvr.size() * sizeof(ring_id_t);
        void* pb = nullptr;
        rc = ctx_ensure(ctx, J_KBLOB, blob + 64, &pb);
        if (rc) return rc;
        char* b = reinterpret_cast<char*>(pb);
        if ((P.nv && (hipMemcpyAsync(b + off_vx, pl.rx.data(), 8 * (size_t)P.nv, hipMemcpyHostToDevice, st) != hipSuccess ||
                      hipMemcpyAsync(b + off_vx + 8 * (size_t)P.nv, pl.ry.data(), 8 * (size_t)P.nv, hipMemcpyHostToDevice,
                                     st) != hipSuccess)) ||
            (nrect && hipMemcpyAsync(b + off_rect, hrect.data(), 16 * (size_t)nrect, hipMemcpyHostToDevice, st) != hipSuccess) ||
            (P.nring > 1 &&
             (hipMemcpyAsync(b + off_env, henv.data(), 8 * henv.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
              hipMemcpyAsync(b + off_vr, hvr.data(), hvr.size() * sizeof(ring_id_t), hipMemcpyHostToDevice, st) != hipSuccess)))
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "polygon upload failed");
        kc->grid = *grid;
        kc->r = r;
        kc->ring_off.resize((size_t)nring + 1);
        for (uint32_t j = 0; j <= nring; j++) kc->ring_off[j] = ring_off[j] - ring_off[0];
        kc->vx.assign(vx + v0, vx + v1);
        kc->vy.assign(vy + v0, vy + v1);
        kc->P = P;
        kc->PB = PB;
        kc->boxed = boxed;
        kc->nrect = nrect;
        kc->off_vx = off_vx;
        kc->off_env = off_env;
        kc->off_rect = off_rect;
        kc->off_vr = off_vr;
        kc->blob_bytes = blob;
        kc->dev_blob = pb;
        kc->valid = true;
    } else {
        void* pb = nullptr;  // the slot is this path's own: same pointer, same contents
        rc = ctx_ensure(ctx, J_KBLOB, kc->blob_bytes + 64, &pb);
        if (rc) return rc;
        if (pb != kc->dev_blob) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "polygon table slot moved");
    }
    const PpknnPoly& P = kc->P;
    const PpknnBoxes& PB = kc->PB;
    const uint32_t nrect = kc->nrect;
    char* tb = reinterpret_cast<char*>(kc->dev_blob);
    double* dvx = reinterpret_cast<double*>(tb + kc->off_vx);
    double* dvy = dvx + P.nv;
    int32_t* drect = reinterpret_cast<int32_t*>(tb + kc->off_rect);
    double* denv = reinterpret_cast<double*>(tb + kc->off_env);
    ring_id_t* dvr = reinterpret_cast<ring_id_t*>(tb + kc->off_vr);
    // ---- the last window's candidate count, if it has landed: picks the selection path
    if (!kc->pin) {
        if (hipHostMalloc((void**)&kc->pin, 16, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&kc->ev, hipEventDisableTiming) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "pinned count allocation failed");
        kc->pin[0] = 0;
    }
    if (kc->ev_pending && hipEventQuery(kc->ev) == hipSuccess) {
        kc->last_m = kc->pin[0];
        kc->ev_pending = false;
    }
    (void)hipGetLastError();  // a not-ready query is no error
    const double *dx, *dy;
    rc = ctx_stage_xy(ctx, x, y, n, 0, &dx, &dy);
    if (rc) return rc;
    Scratch S{ctx};
    const uint64_t ncap = n ? n : 1;
    char* cbuf = S.get<char>(J_KCAND, ncap * 12 + 64);
    if (S.rc) return S.rc;
    const size_t kout = std::max<size_t>(k, 256);
    LargeK L;
    rc = large_k_scratch(ctx, (unsigned)kout, kout * 12 + 64, &L);  // + output staging (host windows)
    if (rc) return rc;
    unsigned long long* key = reinterpret_cast<unsigned long long*>(cbuf);
    unsigned* cand = reinterpret_cast<unsigned*>(cbuf + ncap * 8);
    RselState* rs = L.rs;
    double* od = dev ? out_dist : reinterpret_cast<double*>(L.extra);
    unsigned* oi = dev ? out_idx : reinterpret_cast<unsigned*>(L.extra + kout * 8);
    unsigned* ocnt = async ? out_count : reinterpret_cast<unsigned*>(L.extra + kout * 12);
    hipEvent_t e0, e1;
    ctx_timing_events(ctx, &e0, &e1);
    if (e0) hipEventRecord(e0, st);
    // one workgroup selects (any candidate count, fast up to kRselSmall) unless the last window
    // had more candidates than that: then the multi-block rounds (GEOHIP_RSEL_SMALL: test hook
    // forcing them above the given count)
    static const char* env_small = getenv("GEOHIP_RSEL_SMALL");
    const bool multi = big_k || (env_small ? true : kc->last_m > kRselSmall);
    const unsigned small_max = big_k ? 0u : (env_small ? (unsigned)atol(env_small) : (multi ? 0u : 0xffffffffu));
    tlaunch(ctx, rsel_init, 1, 1024, 0, st, rs, k, small_max);
    if (big_k && hipMemsetAsync(L.sel_d, 0xff, (size_t)kout * 12, st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    if (n && nrect) {
        if (kc->boxed) {
            const uint64_t iters = (n + 255) / 256;
            static const uint64_t max_blocks = getenv("GEOHIP_PPKNN_BLOCKS") ? (uint64_t)atol(getenv("GEOHIP_PPKNN_BLOCKS")) : 2048;
            const uint64_t nb = std::max<uint64_t>(1, std::min<uint64_t>((iters + 3) / 4, max_blocks));  // 4 waves per block
            switch (PB.nb) {
                case 1: tlaunch(ctx, ppknn_scan_boxes<1>, (unsigned)nb, kTB, 0, st, dx, dy, n, PB, cand, rs); break;
                case 2: tlaunch(ctx, ppknn_scan_boxes<2>, (unsigned)nb, kTB, 0, st, dx, dy, n, PB, cand, rs); break;
                case 3: tlaunch(ctx, ppknn_scan_boxes<3>, (unsigned)nb, kTB, 0, st, dx, dy, n, PB, cand, rs); break;
                case 4: tlaunch(ctx, ppknn_scan_boxes<4>, (unsigned)nb, kTB, 0, st, dx, dy, n, PB, cand, rs); break;
                default: tlaunch(ctx, ppknn_scan_boxes<0>, (unsigned)nb, kTB, 0, st, dx, dy, n, PB, cand, rs); break;
            }
        } else {
            const uint64_t nb = std::min<uint64_t>((n + kTB - 1) / kTB, 4096);
            tlaunch(ctx, ppknn_scan, (unsigned)nb, kTB, 0, st, dx, dy, n, grid->min_x, grid->min_y, grid->cell_len, drect, nrect,
                                                     cand, rs);
        }
        if (approximate) tlaunch(ctx, ppknn_dist<true>, 1024, kTB, 0, st, dx, dy, cand, rs, dvx, dvy, dvr, denv, P, key);
        else tlaunch(ctx, ppknn_dist<false>, 1024, kTB, 0, st, dx, dy, cand, rs, dvx, dvy, dvr, denv, P, key);
    }
    if (big_k) {
        rc = rsel_large_tail(st, key, cand, rs, k, L.sel_d, L.sel_i, L.tmp_d, L.tmp_i, L.temp, L.temp_bytes, od, oi,
                             ocnt);
        if (rc) return ctx_fail(ctx, rc, "large-k kNN launch failed");
    } else {
        tlaunch(ctx, rsel_small, 1, 1024, 0, st, key, cand, rs, k, od, oi, ocnt);  // M <= small_max (and M = 0)
        if (multi) {
            for (int t = 0; t < kRselRounds; t++) {
                tlaunch(ctx, rsel_hist, 512, kTB, 0, st, key, cand, rs, t, k);
                tlaunch(ctx, rsel_pick, 1, 1024, 0, st, rs, t, k);
            }
            tlaunch(ctx, rsel_gather, 512, kTB, 0, st, key, cand, rs, k, L.sel_d, L.sel_i);
            tlaunch(ctx, rsel_sort, 1, 256, 0, st, L.sel_d, L.sel_i, rs, k, od, oi, ocnt);
        }
    }
    if (e1) hipEventRecord(e1, st);
    // this window's candidate count for the next call's choice (lands with the event)
    if (hipMemcpyAsync(kc->pin, &rs->ncand, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipEventRecord(kc->ev, st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "candidate count copy failed");
    kc->ev_pending = true;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("knn_ppoly launch: ") + hipGetErrorString(e));
    if (async) return GEOHIP_OK;
    uint32_t m = 0;
    if (hipMemcpyAsync(&m, ocnt, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "count readback failed");
    kc->last_m = kc->pin[0];
    kc->ev_pending = false;
    if (!dev && m &&
        (hipMemcpy(out_dist, od, 8 * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess ||
         hipMemcpy(out_idx, oi, 4 * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess))
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "kNN readback failed");
    *out_count = m;
    return GEOHIP_OK;
}

}  // namespace geohip
