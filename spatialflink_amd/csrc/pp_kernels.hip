// pp_kernels.hip -- point-query kernels of libgeohip for gfx950 (MI355X).
//
// kNN   (PointPointKNNQuery.java:125-191 + KNNQuery.java:204-272):
//   knn_scan   one HBM pass over SoA x/y: exact box classification (4 compares, no division),
//              candidates compacted per wave through LDS so fdlibm hypot runs on full waves,
//              distances pruned by a block-wide threshold (LDS min of the waves' k-th distance,
//              a valid upper bound of the block's k-th), survivors kept in a per-wave sorted
//              list (64*KPL entries across lanes, bitonic merge of 64-entry batches); the 4
//              wave lists of a block are merged into one sorted block list.
//   knn_final  one workgroup: T = k-th smallest block-list head (an upper bound of the global
//              k-th key; register sorts + LDS merge tree), gather every entry <= T (typically
//              ~k), one-wave register bitonic sort, emit top-k.
// range (PointPointRangeQuery.java:86-137):
//   range_scan   same pass; guaranteed boxes -> hit without distance, candidate boxes ->
//                compacted distance batches; hits kept as a bitmask per 1024-point unit.
//   scan_units   exclusive scan of per-unit hit counts.
//   range_emit   bitmask -> ascending window indices.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <type_traits>

#include "device_common.h"
#include "pp_kernels.h"

namespace geohip {

constexpr int kBlock = 256;            // 4 waves
constexpr int kPtsIter = 256;          // points per wave iteration (4 per lane)
constexpr int kCandCap = 64 + kPtsIter;
struct WaveStage {  // wave-private LDS
    double cx[kCandCap];
    double cy[kCandCap];
    unsigned ci[kCandCap];
};

__device__ __forceinline__ void load4(const double* __restrict__ x, const double* __restrict__ y,
                                      uint64_t base, uint64_t end, int lane, double px[4], double py[4],
                                      bool valid[4]) {
    const uint64_t i0 = base + 2 * (uint64_t)lane;
    const uint64_t i1 = base + 128 + 2 * (uint64_t)lane;
    if (base + kPtsIter <= end) {
        // plain loads: nontemporal ones measured no gain for the range passes (47.7-49.0 against
        // 47.4-47.7 us, round 5)
        const double2 a = *reinterpret_cast<const double2*>(x + i0);
        const double2 b = *reinterpret_cast<const double2*>(x + i1);
        const double2 c = *reinterpret_cast<const double2*>(y + i0);
        const double2 d = *reinterpret_cast<const double2*>(y + i1);
        px[0] = a.x; px[1] = a.y; px[2] = b.x; px[3] = b.y;
        py[0] = c.x; py[1] = c.y; py[2] = d.x; py[3] = d.y;
        valid[0] = valid[1] = valid[2] = valid[3] = true;
    } else {
        const uint64_t id[4] = {i0, i0 + 1, i1, i1 + 1};
#pragma unroll
        for (int s = 0; s < 4; s++) {
            valid[s] = id[s] < end;
            px[s] = valid[s] ? x[id[s]] : 0.0;
            py[s] = valid[s] ? y[id[s]] : 0.0;
        }
    }
}

__device__ __forceinline__ uint64_t slot_index(uint64_t base, int lane, int s) {
    return base + (uint64_t)((s >> 1) * 128 + 2 * lane + (s & 1));
}

__device__ __forceinline__ bool lds_kless(unsigned long long ad, unsigned ai, unsigned long long bd, unsigned bi) {
    return ad < bd || (ad == bd && ai < bi);
}

// bitonic sort of m (power of two) keys in LDS by the whole workgroup (fallback path)
__device__ void block_sort_lds(unsigned long long* d, unsigned* i, int m) {
    for (int size = 2; size <= m; size <<= 1) {
        for (int j = size >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < m / 2; t += blockDim.x) {
                const int lo = 2 * j * (t / j) + (t % j);
                const int hi = lo + j;
                const bool up = (lo & size) == 0;
                const bool swap = up ? lds_kless(d[hi], i[hi], d[lo], i[lo]) : lds_kless(d[lo], i[lo], d[hi], i[hi]);
                if (swap) {
                    unsigned long long td = d[lo]; d[lo] = d[hi]; d[hi] = td;
                    unsigned ti = i[lo]; i[lo] = i[hi]; i[hi] = ti;
                }
            }
            __syncthreads();
        }
    }
}

// ============================================================================ kNN =========
// Block-level selection state (LDS).  Survivors of the pruning bound go to one buffer; a
// 512-bin histogram of their distance bits (16 bins per octave over the 32 octaves below the
// largest possible candidate distance) yields the bound: B = upper edge of the smallest bin
// at which the cumulative count reaches k.  That is a valid upper bound of the block's k-th
// distance (>= k real candidates lie at or below it), shared by the four waves from the first
// survivors on, and it costs LDS atomics instead of per-wave sorting networks.
// Re-read an LDS word other waves update.  A volatile access through a generic pointer
// compiles to flat_load sc0 sc1, which counts against vmcnt and makes the compiler drain
// every outstanding global load (the scan's prefetch) before it; a compiler barrier + a plain
// access stays a ds_read with an lgkmcnt wait.
template <typename T>
__device__ __forceinline__ T lds_fresh(const T& v) {
    asm volatile("" ::: "memory");
    return v;
}

// write-through (sc1) stores: data another workgroup of the same launch reads (Guideline 16 R1)
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ void store_wt(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(((gu64*)(p)), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_wt(unsigned* p, unsigned v) {
    __hip_atomic_store(((gu32*)(p)), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kHistBins = 512;

// survivor buffer: 192 entries per wave (4 waves: stages 25.6 KB + this ~11.3 KB, 4 blocks/CU)
template <int NW>
struct KnnBlock {
    static constexpr int kCap = 192 * NW;
    unsigned hist[kHistBins];
    unsigned long long bd[kCap];
    unsigned bi[kCap];
    unsigned long long bound;  // distance bits; kSentinelD = none yet
    unsigned cnt;              // survivors appended (may exceed kCap: the rest spilled)
    unsigned final_cnt;
    unsigned next_it;          // next unclaimed 256-point iteration of the block's chunk
};

__device__ __forceinline__ int hist_bin(unsigned long long db, int base) {
    const long long b = (long long)(db >> 48) - base;
    return b < 0 ? 0 : (b >= kHistBins ? kHistBins - 1 : (int)b);
}

// One wave: smallest bin whose cumulative count reaches k (wave-uniform), -1 if none.
__device__ __forceinline__ int hist_kth_bin(const unsigned* hist, unsigned k) {
    const int lane = lane_id();
    unsigned c[8];
    unsigned tot = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        c[j] = hist[lane * 8 + j];
        tot += c[j];
    }
    const unsigned incl = wave_incl_scan(tot);  // inclusive prefix over lanes
    const unsigned long long m = __ballot(incl >= k);
    if (m == 0) return -1;
    const int first = __builtin_ctzll(m);
    // every lane finds its own crossing bin; the first crossing lane's is the answer
    int bin = kHistBins - 1;
    unsigned run = incl - tot;
    bool found = false;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        run += c[j];
        if (!found && run >= k) { bin = lane * 8 + j; found = true; }
    }
    return __builtin_amdgcn_readlane(bin, first);
}

// One wave, one scan: the crossing bins of two counts (as hist_kth_bin).
__device__ __forceinline__ void hist_kth_bins2(const unsigned* hist, unsigned k1, unsigned k2, int& b1, int& b2) {
    const int lane = lane_id();
    unsigned c[8];
    unsigned tot = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        c[j] = hist[lane * 8 + j];
        tot += c[j];
    }
    const unsigned incl = wave_incl_scan(tot);
    auto cross = [&](unsigned kk) -> int {
        const unsigned long long m = __ballot(incl >= kk);
        if (m == 0) return -1;
        int bin = kHistBins - 1;
        unsigned run = incl - tot;
        bool found = false;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            run += c[j];
            if (!found && run >= kk) { bin = lane * 8 + j; found = true; }
        }
        return __builtin_amdgcn_readlane(bin, __builtin_ctzll(m));
    };
    b1 = cross(k1);
    b2 = cross(k2);
}

// rank of this lane's (d, i) key among the keys of the lanes in `mask` (keys unique: indices are)
__device__ __forceinline__ unsigned wave_rank_in(unsigned long long mask, unsigned long long d, unsigned i) {
    unsigned r = 0;
    while (mask) {
        const int j = __builtin_ctzll(mask);
        mask &= mask - 1;
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)d, j);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(d >> 32), j);
        const unsigned ij = (unsigned)__builtin_amdgcn_readlane((int)i, j);
        const unsigned long long dj = ((unsigned long long)hi << 32) | lo;
        r += (dj < d || (dj == d && ij < i)) ? 1u : 0u;
    }
    return r;
}

// upper edge (distance bits) of histogram bin `bin`
__device__ __forceinline__ unsigned long long hist_edge(int bin, int base) {
    return ((unsigned long long)(bin + base + 1) << 48) - 1ull;
}

// One wave: the block bound from the survivor histogram (LDS atomic min).
template <class KB>
__device__ __forceinline__ void hist_bound(KB& kb, unsigned k, int base) {
    const int bin = hist_kth_bin(kb.hist, k);
    if (bin >= 0 && bin < kHistBins - 1 && lane_id() == 0) atomicMin(&kb.bound, hist_edge(bin, base));
}

// ---------------------------------------------------------------- final selection --------
// final_select<KPL, NT, OWN>: NT threads (NT/64 waves) reduce nlists ascending lists of
// list_len entries (plus the unsorted spill buffer) to the k smallest keys.
//  (1) T = an upper bound of the global k-th key: the upper edge of the histogram bin where the
//      cumulative count of list heads reaches k (>= k real entries lie at or below it).  The
//      scan's blocks add their head to a global histogram as they finish (off the critical
//      path), so here it is one load per bin; without it (rank merges) the heads are binned in
//      LDS.  When that bin is the lowest or the top one, T is exact instead: the k-th smallest
//      head (register sorts of 64-head batches, merged by a tree through LDS);
//  (2) every entry <= T is gathered (lists ascending: a list scan stops at the first entry
//      above T; ~k entries in all, nearly always within the kHeads entries preloaded per list);
//  (3) the gathered entries are placed by rank (each thread counts the smaller keys; keys are
//      unique, ties broken by position) and the k smallest written in order.
// Every global load of (1)-(2) is issued up front (the histogram, kHeads entries of OWN lists
// per thread and the spill count), so the selection pays one memory latency.  It runs as the
// knn_final kernel (separate launch, merges of rank results) and inside knn_scan's
// last-arriving block.
constexpr int kFinalThreads = 1024;
constexpr int kFinalCap = 4096;
constexpr int kHeads = 4;  // entries per list preloaded by the final selection (packed heads)

struct FinalIo {
    const unsigned long long* part_d;
    const unsigned* part_i;
    unsigned nlists, list_len, k;
    double* out_d;
    unsigned* out_i;
    unsigned* out_count;
    const unsigned long long* spill_d;  // null: no spill buffer (rank merges)
    const unsigned* spill_i;
    unsigned* spill_cnt;
    const unsigned long long* head_d;  // null, or the first kHeads entries of every list packed
    const unsigned* head_i;            // (head_d[kHeads l + j]): coalesced head loads
    int hist_base;                     // histogram origin (head_d != null)
    unsigned* ghist;                   // null, or the producers' head histogram (re-zeroed here)
};

struct FinalLds {  // LDS working set (the fused form reuses the scan's stages)
    unsigned long long* xd;  // tree exchange, (NT / 128) * 64 * KPL entries
    unsigned* xi;
    unsigned long long* bd;  // gathered entries
    unsigned* bi;
    unsigned cap;            // >= NT
    unsigned* cnt;
    unsigned long long* Td;
    unsigned* Ti;
    unsigned* hist;          // kHistBins words
};

// Phase timestamps of one kNN launch (measurement builds only, MODE 6 of knn_scan): per block
// 8 slots at [8 b], the final selection's at [8 nblocks + p]; 100 MHz real-time clock.
__device__ unsigned long long* g_knn_trace;
#define GEOHIP_TRACE(on, slot)                                                        \
    do {                                                                              \
        if ((on) && threadIdx.x == 0) g_knn_trace[(slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

__device__ __forceinline__ unsigned load_sc1(const unsigned* p) {
    return __hip_atomic_load(((const gu32*)(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Rank placement of m keys held in LDS (d 16-byte aligned, ix 8-byte aligned): entry t goes to
// position #{j : key_j < key_t or (key_j == key_t and j < t)} (unique positions even for equal
// keys); calls put(pos, d, i) for pos < limit.  The keys are read as broadcast LDS loads, 8 per
// batch (4 ds_read_b128 + 4 ds_read_b64 in flight) so the loop pays LDS latency once per batch.
__device__ __forceinline__ unsigned rank_less(unsigned long long jd, unsigned ji, unsigned j, unsigned long long kd,
                                              unsigned ki, unsigned t) {
    return (jd < kd || (jd == kd && (ji < ki || (ji == ki && j < t)))) ? 1u : 0u;
}
template <int NT, class Put>
__device__ __forceinline__ void rank_place(const unsigned long long* d, const unsigned* ix, unsigned m, unsigned limit,
                                           Put put) {
    if (m <= 64) {
        // G = NT / 64 lanes per key (consecutive lanes of one DPP row), each counting the smaller
        // keys among every G-th; the G partial counts are summed by lane-xor DPP moves
        constexpr int G = NT / 64 < 16 ? NT / 64 : 16;
        const unsigned t = threadIdx.x / G, g = threadIdx.x % G;
        unsigned r = 0;
        unsigned long long kd = 0;
        unsigned ki = 0;
        if (t < m) {
            kd = d[t];
            ki = ix[t];
#pragma unroll
            for (int u = 0; u < 64 / G; u++) {
                const unsigned j = g + (unsigned)(u * G);
                if (j < m) r += rank_less(d[j], ix[j], j, kd, ki, t);
            }
        }
#pragma unroll
        for (int o = 1; o < G; o <<= 1) r += xor_lane(r, o);
        if (g == 0 && t < m && r < limit) put(r, kd, ki);
        return;
    }
    if (NT >= 1024 && m <= 256) {
        // 4 lanes per key (one DPP quad), each counting the smaller keys among every 4th
        constexpr int G = 4;
        const unsigned t = threadIdx.x / G, g = threadIdx.x % G;
        unsigned r = 0;
        unsigned long long kd = 0;
        unsigned ki = 0;
        if (t < m) {
            kd = d[t];
            ki = ix[t];
#pragma unroll 8
            for (unsigned j = g; j < m; j += G) r += rank_less(d[j], ix[j], j, kd, ki, t);
        }
        r += xor_lane(r, 1);
        r += xor_lane(r, 2);
        if (g == 0 && t < m && r < limit) put(r, kd, ki);
        return;
    }
    for (unsigned t = threadIdx.x; t < m; t += NT) {
        const unsigned long long kd = d[t];
        const unsigned ki = ix[t];
        unsigned r = 0;
        unsigned j = 0;
        for (; j + 8 <= m; j += 8) {
            ulonglong2 dd[4];
            uint2 ii[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                dd[u] = *reinterpret_cast<const ulonglong2*>(d + j + 2 * u);
                ii[u] = *reinterpret_cast<const uint2*>(ix + j + 2 * u);
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                r += rank_less(dd[u].x, ii[u].x, j + 2 * u, kd, ki, t);
                r += rank_less(dd[u].y, ii[u].y, j + 2 * u + 1, kd, ki, t);
            }
        }
        for (; j < m; j++) r += rank_less(d[j], ix[j], j, kd, ki, t);
        if (r < limit) put(r, kd, ki);
    }
}

template <int KPL, int NT, int OWN, bool TRACE = false, bool DRY = false>
__device__ void final_select(const FinalIo& io, const FinalLds& s) {
    const size_t tb = (size_t)8 * gridDim.x;  // final-selection trace slots
    constexpr int N = 64 * KPL;
    constexpr int NW = NT / kWave;
    constexpr int HWPT = (kHistBins + NT - 1) / NT;  // histogram bins per thread
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    const unsigned nlists = io.nlists, list_len = io.list_len, k = io.k;
    if (threadIdx.x == 0) {
        *s.cnt = 0;
        *s.Td = kSentinelD;
        *s.Ti = kSentinelI;
    }
    // ---- (0) every global load up front
    unsigned nspill = 0;
    if (io.spill_cnt) nspill = load_sc1(io.spill_cnt);
    unsigned hc[HWPT][kGhistCopies];
#pragma unroll
    for (int w = 0; w < HWPT; w++) {
        const int b = threadIdx.x + w * NT;
#pragma unroll
        for (int c = 0; c < kGhistCopies; c++)
            hc[w][c] = (io.ghist && b < kHistBins) ? load_sc1(io.ghist + c * kHistBins + b) : 0u;
    }
    KE e[OWN][kHeads];  // first kHeads entries of every owned list
#pragma unroll
    for (int j = 0; j < OWN; j++) {
#pragma unroll
        for (int h = 0; h < kHeads; h++) e[j][h] = ksentinel();
        const unsigned own = threadIdx.x + (unsigned)(j * NT);
        if (own < nlists && io.head_d) {
            const ulonglong2 d01 = *reinterpret_cast<const ulonglong2*>(io.head_d + (size_t)kHeads * own);
            const ulonglong2 d23 = *reinterpret_cast<const ulonglong2*>(io.head_d + (size_t)kHeads * own + 2);
            const uint4 i4 = *reinterpret_cast<const uint4*>(io.head_i + (size_t)kHeads * own);
            e[j][0].d = d01.x; e[j][1].d = d01.y; e[j][2].d = d23.x; e[j][3].d = d23.y;
            e[j][0].i = i4.x; e[j][1].i = i4.y; e[j][2].i = i4.z; e[j][3].i = i4.w;
        } else if (own < nlists) {
            const size_t off = (size_t)own * list_len;
#pragma unroll
            for (int h = 0; h < kHeads; h++) {
                if ((unsigned)h < list_len) {
                    e[j][h].d = io.part_d[off + h];
                    e[j][h].i = io.part_i[off + h];
                }
            }
        }
    }
    GEOHIP_TRACE(TRACE, tb + 1);
    // ---- (1a) T from the head histogram
    bool resolved = false;
    const bool local_hist = !io.ghist && nlists >= k && io.head_d && OWN * NT >= (int)nlists;
    if (io.ghist || local_hist) {
#pragma unroll
        for (int w = 0; w < HWPT; w++) {
            const int b = threadIdx.x + w * NT;
            if (b < kHistBins) {
                unsigned v = 0;
#pragma unroll
                for (int c = 0; c < kGhistCopies; c++) {
                    v += hc[w][c];
                    if (io.ghist) store_wt(io.ghist + c * kHistBins + b, 0u);  // ready for the next window
                }
                s.hist[b] = v;
            }
        }
        __syncthreads();
        GEOHIP_TRACE(TRACE, tb + 5);
        if (local_hist) {
#pragma unroll
            for (int j = 0; j < OWN; j++)
                if (e[j][0].d != kSentinelD) atomicAdd(&s.hist[hist_bin(e[j][0].d, io.hist_base)], 1u);
            __syncthreads();
        }
        if (wid == 0 && nlists >= k) {
            const int bin = hist_kth_bin(s.hist, k);
            if (lane == 0 && bin > 0 && bin < kHistBins - 1) {
                *s.Td = hist_edge(bin, io.hist_base);
                *s.Ti = kSentinelI;
            }
        }
        __syncthreads();
        resolved = *s.Td != kSentinelD;
    }
    // ---- (1b) exact: T = k-th smallest head
    if (nlists >= k && !resolved) {
        WList<KPL> L;
#pragma unroll
        for (int q = 0; q < KPL; q++) L.s[q] = ksentinel();
#pragma unroll
        for (int j = 0; j < OWN; j++)
            if ((unsigned)(j * NT + wid * kWave) < nlists) wave_merge_batch<KPL>(L, wave_sort64(e[j][0]));
        for (unsigned g = (unsigned)(wid * kWave + OWN * NT); g < nlists; g += NT) {
            KE h = ksentinel();
            const unsigned p = g + lane;
            if (p < nlists) {
                h.d = io.part_d[(size_t)p * list_len];
                h.i = io.part_i[(size_t)p * list_len];
            }
            wave_merge_batch<KPL>(L, wave_sort64(h));
        }
        for (int step = 1; step < NW; step <<= 1) {
            __syncthreads();
            if ((wid & (2 * step - 1)) == step) {  // sender
                const int slot = wid >> 1;
#pragma unroll
                for (int q = 0; q < KPL; q++) {
                    s.xd[slot * N + q * 64 + lane] = L.s[q].d;
                    s.xi[slot * N + q * 64 + lane] = L.s[q].i;
                }
            }
            __syncthreads();
            if ((wid & (2 * step - 1)) == 0) {  // receiver of wid + step
                const int slot = (wid + step) >> 1;
                WList<KPL> B;
#pragma unroll
                for (int q = 0; q < KPL; q++) {
                    B.s[q].d = s.xd[slot * N + q * 64 + lane];
                    B.s[q].i = s.xi[slot * N + q * 64 + lane];
                }
                wave_merge_lists<KPL>(L, B);
            }
        }
        if (wid == 0) {
            const KE t = wave_list_get<KPL>(L, (int)k - 1);
            if (lane == 0) {
                *s.Td = t.d;
                *s.Ti = t.i;
            }
        }
    }
    __syncthreads();
    GEOHIP_TRACE(TRACE, tb + 2);
    const unsigned long long T_d = *s.Td;
    const unsigned T_i = *s.Ti;
    // ---- (2) gather every real entry <= T.  The preloaded entries go by a block-wide prefix
    // sum of per-thread counts (lists ascending: the passing entries of a list are a prefix);
    // the rare rest (lists whose kHeads entries all pass, lists past OWN * NT, spill) by atomics.
    auto pass = [&](const KE& v) -> bool { return v.d != kSentinelD && !lds_kless(T_d, T_i, v.d, v.i); };
    auto take = [&](const KE& e) -> bool {
        if (!pass(e)) return false;
        const unsigned pos = atomicAdd(s.cnt, 1u);
        if (pos < s.cap) {
            s.bd[pos] = e.d;
            s.bi[pos] = e.i;
        }
        return true;
    };
    unsigned npass[OWN];
    unsigned mine = 0;
#pragma unroll
    for (int j = 0; j < OWN; j++) {
        const unsigned own = threadIdx.x + (unsigned)(j * NT);
        unsigned c = 0;
#pragma unroll
        for (int h = 0; h < kHeads; h++) c += (c == (unsigned)h && own < nlists && pass(e[j][h])) ? 1u : 0u;
        npass[j] = c;
        mine += c;
    }
    const unsigned incl = wave_incl_scan(mine);
    unsigned* wsum = s.hist;  // free once T is known
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    unsigned wbase = 0, total_fast = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const unsigned v = wsum[w];
        wbase += w < wid ? v : 0u;
        total_fast += v;
    }
    {
        unsigned pos = wbase + incl - mine;
#pragma unroll
        for (int j = 0; j < OWN; j++) {
#pragma unroll
            for (int h = 0; h < kHeads; h++) {
                if ((unsigned)h < npass[j]) {
                    if (pos < s.cap) {
                        s.bd[pos] = e[j][h].d;
                        s.bi[pos] = e[j][h].i;
                    }
                    pos++;
                }
            }
        }
    }
    if (threadIdx.x == 0) *s.cnt = total_fast;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < OWN; j++) {
        const unsigned own = threadIdx.x + (unsigned)(j * NT);
        if (npass[j] == (unsigned)kHeads && own < nlists) {  // the rest of the list from memory (rare)
            const size_t off = (size_t)own * list_len;
            for (unsigned q = kHeads; q < list_len; q++) {
                KE v;
                v.d = io.part_d[off + q];
                v.i = io.part_i[off + q];
                if (!take(v)) break;
            }
        }
    }
    for (unsigned p = threadIdx.x + (unsigned)(OWN * NT); p < nlists; p += NT) {
        const size_t off = (size_t)p * list_len;
        for (unsigned q = 0; q < list_len; q++) {
            KE v;
            v.d = io.part_d[off + q];
            v.i = io.part_i[off + q];
            if (!take(v)) break;
        }
    }
    // survivors a scan block could not keep in LDS (unsorted, usually none)
    for (unsigned t = threadIdx.x; t < nspill; t += NT) {
        KE v;
        v.d = io.spill_d[t];
        v.i = io.spill_i[t];
        take(v);
    }
    __syncthreads();
    GEOHIP_TRACE(TRACE, tb + 3);
    if (io.spill_cnt && threadIdx.x == 0) *io.spill_cnt = 0;  // ready for the next window on this stream
    const unsigned total = *s.cnt;
    const unsigned outn = total < k ? total : k;
    auto put = [&](unsigned pos, unsigned long long d, unsigned i) {
        if (DRY) return;
        io.out_d[pos] = __longlong_as_double((long long)d);
        io.out_i[pos] = i;
    };
    if (total <= s.cap && total <= 2u * NT) {
        // ---- (3) rank placement of the gathered entries
        rank_place<NT>(s.bd, s.bi, total, k, put);
        for (unsigned t = outn + threadIdx.x; t < k; t += NT) put(t, kSentinelD, kSentinelI);
        if (threadIdx.x == 0 && !DRY) *io.out_count = outn;
        GEOHIP_TRACE(TRACE, tb + 4);
        return;
    }
    if (total <= s.cap) {
        int m = 1;
        while (m < (int)total) m <<= 1;
        for (int t = threadIdx.x + total; t < m; t += NT) {
            s.bd[t] = kSentinelD;
            s.bi[t] = kSentinelI;
        }
        __syncthreads();
        block_sort_lds(s.bd, s.bi, m);
        for (unsigned t = threadIdx.x; t < k; t += NT) {
            io.out_d[t] = __longlong_as_double((long long)(t < outn ? s.bd[t] : kSentinelD));
            io.out_i[t] = t < outn ? s.bi[t] : kSentinelI;
        }
        if (threadIdx.x == 0) *io.out_count = outn;
        return;
    }
    // pathological (massive exact ties): k rounds of "smallest key above the previous one"
    unsigned long long prev_d = 0;
    unsigned prev_i = 0;
    bool have_prev = false;
    unsigned got = 0;
    const size_t nl = (size_t)nlists * list_len;
    for (unsigned r = 0; r < k; r++) {
        unsigned long long best_d = kSentinelD;
        unsigned best_i = kSentinelI;
        for (size_t t = threadIdx.x; t < nl + nspill; t += NT) {
            const unsigned long long ed = t < nl ? io.part_d[t] : io.spill_d[t - nl];
            const unsigned ei = t < nl ? io.part_i[t] : io.spill_i[t - nl];
            if (ed == kSentinelD) continue;
            if (have_prev && !lds_kless(prev_d, prev_i, ed, ei)) continue;
            if (lds_kless(ed, ei, best_d, best_i)) {
                best_d = ed;
                best_i = ei;
            }
        }
        s.bd[threadIdx.x] = best_d;
        s.bi[threadIdx.x] = best_i;
        __syncthreads();
        for (int h = NT / 2; h > 0; h >>= 1) {
            if ((int)threadIdx.x < h && lds_kless(s.bd[threadIdx.x + h], s.bi[threadIdx.x + h], s.bd[threadIdx.x], s.bi[threadIdx.x])) {
                s.bd[threadIdx.x] = s.bd[threadIdx.x + h];
                s.bi[threadIdx.x] = s.bi[threadIdx.x + h];
            }
            __syncthreads();
        }
        const unsigned long long vd = s.bd[0];
        const unsigned vi = s.bi[0];
        __syncthreads();
        if (vd == kSentinelD) break;
        if (threadIdx.x == 0) {
            io.out_d[r] = __longlong_as_double((long long)vd);
            io.out_i[r] = vi;
        }
        prev_d = vd;
        prev_i = vi;
        have_prev = true;
        got = r + 1;
    }
    for (unsigned t = got + threadIdx.x; t < k; t += NT) {
        io.out_d[t] = __longlong_as_double((long long)kSentinelD);
        io.out_i[t] = kSentinelI;
    }
    if (threadIdx.x == 0) *io.out_count = got;
}

template <int KPL>
__global__ __launch_bounds__(kFinalThreads) void knn_final(FinalIo io) {
    constexpr int N = 64 * KPL;
    __shared__ unsigned long long xd[kFinalThreads / 128 * N];
    __shared__ unsigned xi[kFinalThreads / 128 * N];
    __shared__ unsigned long long bd[kFinalCap];
    __shared__ unsigned bi[kFinalCap];
    __shared__ unsigned cnt;
    __shared__ unsigned long long Td;
    __shared__ unsigned Ti;
    __shared__ unsigned hist[kHistBins];
    const FinalLds s{xd, xi, bd, bi, (unsigned)kFinalCap, &cnt, &Td, &Ti, hist};
    final_select<KPL, kFinalThreads, 1>(io, s);
}

__device__ __forceinline__ unsigned ticket_add(unsigned* p) {
    return __hip_atomic_fetch_add(((gu32*)(p)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ticket_zero(unsigned* p) {
    __hip_atomic_store(((gu32*)(p)), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// ======================================================================== kNN pass ========
// One launch per window (PointPointKNNQuery.java:125-191 + the windowAll
// merge KNNQuery.java:204-272).  The stream phase is knn_scan's: exact box classification,
// squared screen against the block bound, LDS-staged fdlibm distances, survivors and a 512-bin
// distance histogram in LDS (B = upper edge of the bin where the block's cumulative count
// reaches k: at least k real points at or below it).  At its end a block
//  * writes its survivors <= B to its list slot unsorted (ballot + LDS cursor, write-through),
//  * writes its 4 smallest sorted (heads, packed for coalesced reads) and its list length,
// and takes a 2-level arrival ticket.  The last block to arrive (Guideline 16 counter hand-off)
// loads the 4 heads of every block, takes T = upper edge of the bin where their cumulative count
// reaches k (>= k real points at or below it, so T bounds the window's k-th key), keeps the
// heads <= T, reads the whole list of the rare block whose 4 heads all pass, places the kept
// entries by rank and writes the k smallest.  No separate final launch, no sorted block lists.
constexpr int kPassNW = 16;                     // waves per block
constexpr unsigned kPassMaxBlocks = 256;        // one block per CU
constexpr unsigned kPassHeads = 8;
constexpr unsigned kLenWhole = 0x80000000u;     // list length flag: heads incomplete, read it whole
constexpr unsigned kLenSlots = 0x40000000u;     // list length flag: the block's slot set is complete (below)
// Slot-complete blocks (k <= kSlotMaxK): every block publishes the lowest nonzero bin of its
// survivor histogram (word kMinWord + block, bin + 1; 0 = none) -- the upper edge of that bin
// bounds the distance of a real point of the block, distinct blocks hold distinct points, so the
// upper edge of the bin where k of the published bins have accumulated bounds the window's k-th
// distance.  A block whose survivors at or below that bound T_b fit kPassHeads slots writes
// just those (its share of the window's k nearest is among them) and skips the list / head
// ranking; the last block re-arms the words.
constexpr unsigned kSlotMaxK = 256;
constexpr unsigned kMinWord = 6400;
constexpr unsigned kStatWord = (unsigned)(kKnnCounterBytes / 4) - 16;  // last final: entries, spilled, kept
constexpr unsigned kVbWord = kTicketStride * (kMaxTicketGroups + 1);      // chunk ticket (fused range)

template <int NW>
struct PassBlock {
    static constexpr int kCap = 192 * NW;
    unsigned hist[kHistBins];   // survivor distances (local bound)
    unsigned long long bd[kCap];
    unsigned bi[kCap];
    unsigned long long bound;   // block bound, distance bits
    unsigned long long top_d[kWave];  // kept survivors <= hcap (the head candidates)
    unsigned top_i[kWave];
    unsigned long long hcap;    // 4th bin edge: the block's 4 smallest lie at or below it
    unsigned cnt;               // survivors appended (may exceed kCap: the rest spilled)
    unsigned next_it;
    unsigned nsmall;
    unsigned cursor, last;
    unsigned fin[4];            // the final's LDS words
    unsigned long long tslot;   // slot bound T_b (kSentinelD: none)
    unsigned nslot;             // survivors at or below T_b
};

// One wave: the lowest bin holding a survivor, -1 if none (8 bins per lane).
__device__ __forceinline__ int hist_low_bin(const unsigned* hist) {
    const int lane = lane_id();
    int f = -1;
#pragma unroll
    for (int j = 7; j >= 0; j--)
        if (hist[lane * 8 + j]) f = lane * 8 + j;
    const unsigned long long m = __ballot(f >= 0);
    if (!m) return -1;
    return __builtin_amdgcn_readlane(f, __builtin_ctzll(m));
}

struct PassIo {
    unsigned long long* list_d;  // block b: [b * list_cap, b * list_cap + len[b])
    unsigned* list_i;
    unsigned list_cap;
    unsigned long long* head_d;  // block b: [kPassHeads * b, + kPassHeads), sentinel-padded
    unsigned* head_i;
    unsigned* len;               // nblocks list lengths
    unsigned long long* spill_d;
    unsigned long long* spill_d_unused;
    unsigned* spill_i;
    unsigned* ctr;               // zeroed scratch: [0] spill count, tickets from kTicketStride
    double* out_d;
    unsigned* out_i;
    unsigned* out_count;
    unsigned groups;
    unsigned long long* trace;   // measurement only: 8 timestamps per block (null in production)
};
#define PASS_TRACE(io, slot)                                                                      \
    do {                                                                                          \
        if ((io).trace && threadIdx.x == 0) (io).trace[16 * (size_t)blockIdx.x + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

// exact distances of up to 64 staged candidates; survivors (<= the block bound) appended to the
// block buffer and its histogram
// Fused range (knn_pass<.., RANGE>): staged indices carry kFlagKnn (a kNN candidate) and
// kFlagBand (a range candidate in the exact-distance band); one distance serves both.
constexpr unsigned kFlagKnn = 0x80000000u, kFlagBand = 0x40000000u, kIdxMask = 0x3fffffffu;
struct RangeSide {
    unsigned long long* mask;  // LDS hit bitmask of the block's chunk
    uint64_t base;             // first point of the chunk
    double r;
    unsigned grid;             // interleaved sweep (unordered range, grid > 0): the block's bit of
                               // point i is ((i / 256 - blockIdx.x) / grid) * 256 + i % 256
};
__device__ __forceinline__ unsigned range_bit(const RangeSide& rs, uint64_t i) {
    if (rs.grid) return (unsigned)(((i >> 8) - blockIdx.x) / rs.grid) * 256u + (unsigned)(i & 255u);
    return (unsigned)(i - rs.base);
}

template <class PB, bool RANGE = false>
__device__ __forceinline__ void pass_dist_batch(WaveStage& st, unsigned& ccnt, PB& kb, const KnnArgs& a,
                                                const PassIo& io, unsigned& appended, bool partial,
                                                const RangeSide& rs = RangeSide{nullptr, 0, 0.0, 0u}) {
    const int lane = lane_id();
    while (ccnt >= 64 || (partial && ccnt > 0)) {
        const unsigned take = ccnt >= 64 ? 64u : ccnt;
        const unsigned from = ccnt - take;
        bool ok = (unsigned)lane < take;
        double px = 0.0, py = 0.0;
        unsigned pi = 0;
        if (ok) {
            px = st.cx[from + lane];
            py = st.cy[from + lane];
            pi = st.ci[from + lane];
        }
        const unsigned long long B = lds_fresh(kb.bound);
        wave_lds_sync();
        ccnt = from;
        const double d = jts_pp_distance(a.qx, a.qy, px, py);
        const unsigned long long db = (unsigned long long)__double_as_longlong(d);
        if (RANGE) {
            if (ok && (pi & kFlagBand) && d <= rs.r) {
                const unsigned off = range_bit(rs, pi & kIdxMask);
                atomicOr(&rs.mask[off >> 6], 1ull << (off & 63));
            }
            ok = ok && (pi & kFlagKnn);
            pi &= kIdxMask;
        }
        ok = ok && db <= B;
        const unsigned long long m = __ballot(ok);
        if (m) {
            const unsigned nm = (unsigned)__popcll(m);
            unsigned pos = 0;
            if (lane == 0) pos = atomicAdd(&kb.cnt, nm);
            pos = __shfl(pos, 0);
            const unsigned slot = pos + lanes_below(m);
            unsigned gbase = 0;
            if (pos + nm > (unsigned)PB::kCap) {  // spill the overflow to global memory (rare)
                const unsigned first = pos > (unsigned)PB::kCap ? pos : (unsigned)PB::kCap;
                if (lane == 0) gbase = atomicAdd(&io.ctr[0], pos + nm - first);
                gbase = __shfl(gbase, 0) - (first - pos);
            }
            if (ok) {
                if (slot < (unsigned)PB::kCap) {
                    kb.bd[slot] = db;
                    kb.bi[slot] = pi;
                } else {
                    store_wt(&io.spill_d[gbase + (slot - pos)], db);
                    store_wt(&io.spill_i[gbase + (slot - pos)], pi);
                }
                atomicAdd(&kb.hist[hist_bin(db, a.hist_base)], 1u);
            }
            appended += nm;
        }
        wave_lds_sync();
    }
}

// wave min of (d, i) keys; every lane gets the result
__device__ __forceinline__ void wave_kmin(unsigned long long& d, unsigned& i) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long od = xor_lane64(d, o);
        const unsigned oi = xor_lane(i, o);
        if (od < d || (od == d && oi < i)) {
            d = od;
            i = oi;
        }
    }
}

// The window's k smallest, run by the last block (NT = 1024 threads).  Latency-bound: every
// dependent LDS round trip costs ~35 ns and a global one ~1 us, so the phases are few and wide:
//   A  loads: every block's 8 packed heads (2 per thread), its list length and last head (thread
//      b stands for block b), the spill count;
//   B  the heads' distance histogram (LDS atomics) and, per block, "read whole": its 8th head
//      beats T or its heads are flagged incomplete -- known only after T, so the blocks' last
//      heads go to LDS;
//   C  one wave: T = upper edge of the bin where the heads' cumulative count reaches k (k real
//      points at or below it: T bounds the window's k-th key; none if fewer than k heads);
//   D  gather the heads <= T of the blocks not read whole, the whole lists (rare), the spill
//      (ballot + one LDS atomic per wave and batch), then rank placement and the k smallest.
template <int NT>
__device__ __forceinline__ void pass_final(const PassIo& io, const KnnArgs& a, unsigned long long* gd, unsigned* gi,
                                           unsigned gcap, unsigned* hist, unsigned* sh,
                                           unsigned long long* blast_sh, unsigned* lens, unsigned* wl) {
    const unsigned k = a.k, nb = gridDim.x;
    const int lane = lane_id(), wid = threadIdx.x / kWave;
    constexpr unsigned kPer = kPassMaxBlocks * kPassHeads / NT;
    static_assert(kPer == 2, "final: 2 heads per thread");
    // ---- A: loads up front
    const unsigned nspill = load_sc1(io.ctr);
    unsigned long long hd[kPer];
    unsigned hi[kPer];
#pragma unroll
    for (unsigned u = 0; u < kPer; u++) {
        const unsigned t = threadIdx.x + u * NT;
        const bool ok = t < kPassHeads * nb;
        hd[u] = ok ? io.head_d[t] : kSentinelD;
        hi[u] = ok ? io.head_i[t] : kSentinelI;
    }
    const bool blk = threadIdx.x < nb;  // thread b also stands for block b
    const unsigned mylen = blk ? io.len[threadIdx.x] : 0u;
    const unsigned long long blast = blk ? io.head_d[kPassHeads * threadIdx.x + kPassHeads - 1] : kSentinelD;
    for (unsigned t = threadIdx.x; t < kHistBins; t += NT) hist[t] = 0;
    if (threadIdx.x == 0) {
        sh[0] = 0xffffffffu;  // T bin
        sh[2] = 0;            // gather cursor
        sh[3] = 0;            // whole lists
    }
    __syncthreads();
    PASS_TRACE(io, 11);
    // ---- B
#pragma unroll
    for (unsigned u = 0; u < kPer; u++)
        if (hd[u] != kSentinelD) atomicAdd(&hist[hist_bin(hd[u], a.hist_base)], 1u);
    if (blk) {
        // flagged: whole whatever T; slot-complete: never (its slots hold all it contributes)
        blast_sh[threadIdx.x] = (mylen & kLenWhole) ? 0ull : ((mylen & kLenSlots) ? kSentinelD : blast);
        lens[threadIdx.x] = mylen & ~(kLenWhole | kLenSlots);
    }
    if (blk) io.ctr[kMinWord + threadIdx.x] = 0u;  // slot-bound words re-armed for the next launch
    __syncthreads();
    // ---- C
    if (wid == 0) {
        const int bin = hist_kth_bin(hist, k);
        if (lane == 0 && bin >= 0 && bin < kHistBins - 1) sh[0] = (unsigned)bin;
    }
    __syncthreads();
    PASS_TRACE(io, 12);
    const unsigned long long T = sh[0] != 0xffffffffu ? hist_edge((int)sh[0], a.hist_base) : kSentinelD;
    // ---- D
    auto take = [&](bool ok, unsigned long long d, unsigned i) {
        ok = ok && d != kSentinelD && d <= T;
        const unsigned long long msk = __ballot(ok);
        if (!msk) return;
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(&sh[2], (unsigned)__popcll(msk));
        base = __shfl(base, 0);
        const unsigned p = base + lanes_below(msk);
        if (ok && p < gcap) {
            gd[p] = d;
            gi[p] = i;
        }
    };
    if (blk) {
        const unsigned long long bl = blast_sh[threadIdx.x];
        if (bl != kSentinelD && bl <= T) wl[atomicAdd(&sh[3], 1u)] = threadIdx.x;  // rare
    }
#pragma unroll
    for (unsigned u = 0; u < kPer; u++) {
        const unsigned t = threadIdx.x + u * NT;
        const unsigned b = t / kPassHeads;
        bool part = b < nb;
        if (part) {
            const unsigned long long bl = blast_sh[b];
            part = !(bl != kSentinelD && bl <= T);
        }
        take(part, hd[u], hi[u]);
    }
    __syncthreads();
    PASS_TRACE(io, 13);
    const unsigned nwhole = sh[3];
    for (unsigned w = (unsigned)wid; w < nwhole; w += NT / kWave) {  // one wave per whole list
        const unsigned b = wl[w];
        const unsigned L = lens[b];
        for (unsigned q0 = 0; q0 < L; q0 += kWave) {
            const unsigned q = q0 + (unsigned)lane;
            unsigned long long d = kSentinelD;
            unsigned i = kSentinelI;
            if (q < L) {
                d = io.list_d[(size_t)b * io.list_cap + q];
                i = io.list_i[(size_t)b * io.list_cap + q];
            }
            take(q < L, d, i);
        }
    }
    for (unsigned t0 = 0; t0 < nspill; t0 += NT) {
        const unsigned t = t0 + threadIdx.x;
        unsigned long long d = kSentinelD;
        unsigned i = kSentinelI;
        if (t < nspill) {
            d = io.spill_d[t];
            i = io.spill_i[t];
        }
        take(t < nspill, d, i);
    }
    __syncthreads();
    const unsigned m = sh[2];
    if (threadIdx.x == 0) {
        io.ctr[kStatWord] = nwhole;
        io.ctr[kStatWord + 1] = nspill;
        io.ctr[kStatWord + 2] = m;
    }
    PASS_TRACE(io, 6);
    auto put = [&](unsigned pos, unsigned long long d, unsigned i) {
        io.out_d[pos] = __longlong_as_double((long long)d);
        io.out_i[pos] = i;
    };
    unsigned outn = m < k ? m : k;
    if (m <= 2u * NT) {
        rank_place<NT>(gd, gi, m, k, put);
    } else if (m <= gcap) {  // many exact ties around T: bitonic sort in LDS
        unsigned p2 = 1;
        while (p2 < m) p2 <<= 1;
        for (unsigned t = threadIdx.x + m; t < p2; t += NT) {
            gd[t] = kSentinelD;
            gi[t] = kSentinelI;
        }
        __syncthreads();
        block_sort_lds(gd, gi, (int)p2);
        for (unsigned t = threadIdx.x; t < outn; t += NT) put(t, gd[t], gi[t]);
    } else {
        // pathological (more entries at or below T than LDS holds, e.g. a window of identical
        // points): k rounds of "smallest key above the previous one" over every list and the spill
        const size_t nl = (size_t)nb * io.list_cap;
        unsigned long long prev_d = 0;
        unsigned prev_i = 0;
        bool have_prev = false;
        unsigned got = 0;
        for (unsigned r = 0; r < k; r++) {
            unsigned long long best_d = kSentinelD;
            unsigned best_i = kSentinelI;
            for (size_t t = threadIdx.x; t < nl + nspill; t += NT) {
                unsigned long long ed = kSentinelD;
                unsigned ei = kSentinelI;
                if (t < nl) {
                    if (t % io.list_cap < (io.len[t / io.list_cap] & ~kLenWhole)) {
                        ed = io.list_d[t];
                        ei = io.list_i[t];
                    }
                } else {
                    ed = io.spill_d[t - nl];
                    ei = io.spill_i[t - nl];
                }
                if (ed == kSentinelD) continue;
                if (have_prev && !lds_kless(prev_d, prev_i, ed, ei)) continue;
                if (lds_kless(ed, ei, best_d, best_i)) {
                    best_d = ed;
                    best_i = ei;
                }
            }
            __syncthreads();
            gd[threadIdx.x] = best_d;
            gi[threadIdx.x] = best_i;
            __syncthreads();
            for (int h = NT / 2; h > 0; h >>= 1) {
                if ((int)threadIdx.x < h && lds_kless(gd[threadIdx.x + h], gi[threadIdx.x + h], gd[threadIdx.x], gi[threadIdx.x])) {
                    gd[threadIdx.x] = gd[threadIdx.x + h];
                    gi[threadIdx.x] = gi[threadIdx.x + h];
                }
                __syncthreads();
            }
            prev_d = gd[0];
            prev_i = gi[0];
            if (prev_d == kSentinelD) break;
            have_prev = true;
            if (threadIdx.x == 0) put(r, prev_d, prev_i);
            got = r + 1;
        }
        outn = got;
    }
    for (unsigned t = outn + threadIdx.x; t < k; t += NT) put(t, kSentinelD, kSentinelI);
    if (threadIdx.x == 0) {
        *io.out_count = outn;
        store_wt(io.ctr, 0u);            // spill count and the chunk ticket (fused range) re-armed
        store_wt(io.ctr + kVbWord, 0u);  // for the next window on this stream
    }
}

__device__ __forceinline__ bool pass_arrive_last(unsigned* tickets, unsigned G) {
    const unsigned nb = gridDim.x;
    if (G <= 1) {
        const bool last = ticket_add(tickets) == nb - 1;
        if (last) ticket_zero(tickets);
        return last;
    }
    const unsigned g = blockIdx.x % G;
    const unsigned members = nb / G + (g < nb % G ? 1u : 0u);
    unsigned* gc = tickets + (size_t)kTicketStride * g;
    if (ticket_add(gc) != members - 1) return false;
    ticket_zero(gc);
    const unsigned geff = nb < G ? nb : G;
    unsigned* top = tickets + (size_t)kTicketStride * G;
    const bool last = ticket_add(top) == geff - 1;
    if (last) ticket_zero(top);
    return last;
}

// ABL (measurement builds only, 0 in the product): bit 0 skips the list stores, bit 1 the heads
// (4 smallest), bit 2 the end-of-block bound refresh
__device__ __forceinline__ unsigned long long spread32(unsigned v) {  // bit b -> bit 2b
    unsigned long long x = v;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

// Hits of 64 consecutive mask words (word j held by lane j, ex = exclusive prefix of the
// words' hit counts) stored in ascending index order from output position obase: the wave walks
// only the nonzero words (ballot + find-first-set) and each word's hits go out from its lanes at
// consecutive positions (coalesced for dense words; sparse words cost one step each).
// Hits of 64 mask words (lane l holds word l, first point first_point) in ascending order from
// output position obase (advanced): each word's hits go to the wave's LDS stage (one ds_write per
// word), and the stage leaves as full 64-lane stores when it fills and at the end (emit_flush).
// One store instruction per word straight from the bits (partial waves, ~14 lanes for C1) made
// the emission store-issue-bound: ~8 us of the range pass's tail.
constexpr unsigned kEmitStage = 512;  // u32 entries per wave (the wave's idle candidate stage)
static_assert(kEmitStage * 4 <= kCandCap * 8, "the emission stage fits a wave's candidate stage");
__device__ __forceinline__ void emit_flush(unsigned* stg, unsigned& sc, unsigned long long& obase, unsigned* __restrict__ out,
                                           unsigned long long cap) {
    wave_lds_sync();
    for (unsigned t = (unsigned)lane_id(); t < sc; t += kWave)
        if (obase + t < cap) out[obase + t] = stg[t];
    wave_lds_sync();
    obase += sc;
    sc = 0;
}
__device__ __forceinline__ void emit_words(unsigned long long mine, unsigned first_point, unsigned* stg, unsigned& sc,
                                           unsigned long long& obase, unsigned* __restrict__ out, unsigned long long cap) {
    const int lane = lane_id();
    unsigned long long nz = __ballot(mine != 0ull);
    while (nz) {
        const int j = __builtin_ctzll(nz);
        nz &= nz - 1;
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)mine, j);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(mine >> 32), j);
        const unsigned long long bits = ((unsigned long long)hi << 32) | lo;
        if ((bits >> lane) & 1ull) stg[sc + lanes_below(bits)] = first_point + (unsigned)j * 64u + (unsigned)lane;
        sc += (unsigned)__popcll(bits);
        if (sc > kEmitStage - kWave) emit_flush(stg, sc, obase, out, cap);
    }
}

// The same, each of the 64 words with its own first point (lane l holds word l's in `firsts`):
// the interleaved sweep's words are 64-point runs of different fronts.
__device__ __forceinline__ void emit_words_at(unsigned long long mine, unsigned firsts, unsigned* stg, unsigned& sc,
                                              unsigned long long& obase, unsigned* __restrict__ out,
                                              unsigned long long cap) {
    const int lane = lane_id();
    unsigned long long nz = __ballot(mine != 0ull);
    while (nz) {
        const int j = __builtin_ctzll(nz);
        nz &= nz - 1;
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)mine, j);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(mine >> 32), j);
        const unsigned fp = (unsigned)__builtin_amdgcn_readlane((int)firsts, j);
        const unsigned long long bits = ((unsigned long long)hi << 32) | lo;
        if ((bits >> lane) & 1ull) stg[sc + lanes_below(bits)] = fp + (unsigned)lane;
        sc += (unsigned)__popcll(bits);
        if (sc > kEmitStage - kWave) emit_flush(stg, sc, obase, out, cap);
    }
}

// Range hits of a block chunk (LDS bitmask) written in ascending index order: the block
// publishes its count (status word tagged with the launch epoch, atomic exchange: visible at the
// device coherence point), sums the counts of every earlier chunk (wave 0, all loads in flight,
// s_sleep back-off), and each wave stores the hits of a contiguous run of mask words.  The block
// of the last chunk writes the total.  Earlier chunks were taken by blocks that started earlier,
// so the wait always ends.
// Unordered (UNORD): the block reserves its hits on the launch's cursor instead -- the slot of
// its run is known at once, no block waits for another (the kNN's last block writes the total).
template <int NW, bool UNORD = false>
__device__ __forceinline__ void pass_range_publish(const PassRangeIo& rio, const unsigned long long* bmask,
                                                   unsigned& bcount, unsigned long long& excl_sh, unsigned vb,
                                                   unsigned nw) {
    constexpr int NT = NW * 64;
    unsigned my = 0;
    for (unsigned t = threadIdx.x; t < nw; t += NT) my += (unsigned)__popcll(bmask[t]);
    if (my) atomicAdd(&bcount, my);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (UNORD)
            excl_sh = bcount ? atomicAdd(rio.cursor, (unsigned long long)bcount) : 0ull;
        else
            (void)__hip_atomic_exchange(rio.status + vb, (rio.epoch << 40) | (unsigned long long)bcount,
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// UNORD: the run was reserved at publish time (no look-back); word w covers the 64 points from
// ((w / 4) * nblocks + block) * 256 + (w % 4) * 64 (the interleaved fronts).
template <int NW, bool UNORD = false>
__device__ __forceinline__ void pass_range_emit(const PassRangeIo& rio, const unsigned long long* bmask,
                                                unsigned* wsum, unsigned& bcount, unsigned long long& excl_sh,
                                                unsigned vb, uint64_t p0, unsigned nw, unsigned* stg) {
    const int lane = lane_id(), wid = threadIdx.x / kWave;
    if (!UNORD && wid == 0) {
        const unsigned long long pre = poll_block_counts<kPassMaxBlocks / kWave>(rio.status, vb, rio.epoch, rio.spin_limit,
                                                                                  rio.inject, rio.fault);
        if (lane == 0) excl_sh = pre;
    }
    if (rio.trace && threadIdx.x == 0) rio.trace[16 * (size_t)blockIdx.x + 5] = __builtin_amdgcn_s_memrealtime();
    // per-wave word runs and their hit counts (prefix over waves)
    const unsigned wpw = (nw + NW - 1) / NW;
    const unsigned wb = (unsigned)wid * wpw;
    const unsigned we = wb + wpw < nw ? wb + wpw : nw;
    unsigned c = 0;
    for (unsigned w = wb + (unsigned)lane; w < we; w += kWave) c += (unsigned)__popcll(bmask[w]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) wsum[wid] = c;
    __syncthreads();
    unsigned long long obase = excl_sh;
    for (int w = 0; w < wid; w++) obase += wsum[w];
    const unsigned ibase = (unsigned)p0 + rio.a.point_base;
    unsigned sc = 0;
    for (unsigned w0 = wb; w0 < we; w0 += kWave) {
        const unsigned w = w0 + (unsigned)lane;
        const unsigned long long mine = w < we ? bmask[w] : 0ull;
        if (UNORD) {
            const unsigned first = (unsigned)((((uint64_t)(w >> 2) * gridDim.x + blockIdx.x) << 8) + (w & 3u) * 64u) +
                                   rio.a.point_base;
            emit_words_at(mine, first, stg, sc, obase, rio.out, rio.cap);
        } else {
            emit_words(mine, ibase + w0 * 64u, stg, sc, obase, rio.out, rio.cap);
        }
    }
    if (sc) emit_flush(stg, sc, obase, rio.out, rio.cap);
    if (!UNORD && threadIdx.x == 0 && vb == gridDim.x - 1) *rio.total = excl_sh + bcount;
    if (rio.trace && threadIdx.x == 0) rio.trace[16 * (size_t)blockIdx.x + 6] = __builtin_amdgcn_s_memrealtime();
}

// The range query of the same point, fused into the kNN pass (C5: kNN k + range r of one query):
// the point classification is shared, one fdlibm distance serves both, hits go to an LDS bitmask
// of the block's chunk (chunks taken in start order from a ticket) and are written in ascending
// index order behind a look-back over the earlier chunks' hit counts (as range_fused).
constexpr unsigned kFusedMaskWords = 2048;  // 131072 points per block chunk at most

template <int NW, int ABL = 0, bool RANGE = false, bool UNORD = false>
__global__ __launch_bounds__(NW * 64) void knn_pass(const double* __restrict__ x, const double* __restrict__ y,
                                                    uint64_t n, uint64_t chunk, KnnArgs args, PassIo io,
                                                    PassRangeIo rio) {
    constexpr int NT = NW * 64;
    using PB = PassBlock<NW>;
    __shared__ __attribute__((aligned(16))) WaveStage stage[NW];
    __shared__ PB kb;
    __shared__ unsigned long long rmask[RANGE ? kFusedMaskWords : 1];
    __shared__ unsigned rwsum[RANGE ? NW : 1];
    __shared__ unsigned rvb, rcount;
    __shared__ unsigned long long rexcl;
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    WaveStage& st = stage[wid];
    if (RANGE) {
        if (threadIdx.x == 0) {
            rvb = UNORD ? blockIdx.x : atomicAdd(io.ctr + kVbWord, 1u);  // ordered: chunks in start order
            rcount = 0;
        }
        __syncthreads();
    }
    const unsigned vb = RANGE ? rvb : blockIdx.x;
    const uint64_t blk_begin = (uint64_t)vb * chunk;
    uint64_t blk_end = blk_begin + chunk;
    if (blk_end > n) blk_end = n;
    const RangeSide rs{rmask, blk_begin, rio.a.r, UNORD ? gridDim.x : 0u};
    for (int t = threadIdx.x; t < kHistBins; t += NT) kb.hist[t] = 0;
    if (RANGE)
        for (unsigned t = threadIdx.x; t < kFusedMaskWords; t += NT) rmask[t] = 0ull;
    if (threadIdx.x == 0) {
        kb.bound = kSentinelD;
        kb.cnt = 0;
        kb.cursor = 0;
        kb.nsmall = 0;
        kb.next_it = 2 * NW;  // iterations wid and NW + wid start statically
    }
    PASS_TRACE(io, 0);
    if (io.trace && threadIdx.x == 0) {  // measurement only: the XCD this block runs on
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        io.trace[16 * (size_t)blockIdx.x + 15] = xcc & 0xfu;
    }
    const unsigned k = args.k;
    // Iteration order.  kNN alone: the block's iterations interleave with every other block's
    // (global iteration it * nblocks + block), so the grid sweeps the window as one front and
    // the blocks' stream ends bunch up (a chunk per block leaves a 4-7 us spread between the
    // first and the last block, measured by the phase trace).  The fused range keeps a contiguous
    // chunk per block (its hit bitmask covers the chunk).  ABL bit 4: chunks (measurement).
    // The unordered fused range interleaves too: its bitmask words follow the block's fronts.
    constexpr bool kInterleave = (!RANGE || UNORD) && !(ABL & 16);
    // (Rotating each block's slot within a front, so one XCD's blocks do not always read the same
    // 2 KB position mod 16 KB, measured slower in round 4: 42.3 against 38.7 us.)
    const uint64_t total_iters = (n + kPtsIter - 1) / kPtsIter;
    const uint64_t full_fronts = total_iters / gridDim.x, rem_front = total_iters % gridDim.x;
    const unsigned niters =
        kInterleave ? (unsigned)(full_fronts + ((rem_front && blockIdx.x < rem_front) ? 1u : 0u))
                    : (unsigned)((blk_end - blk_begin + kPtsIter - 1) / kPtsIter);
    if (kInterleave) blk_end = n;
    unsigned ccnt = 0;
    unsigned appended = 0, last_hist = 0;
    const Box b0 = args.u[0];
    const int nu = args.nu;
    auto in_union = [&](double px, double py) -> bool {
        bool c = in_box(b0, px, py);
        if (nu > 1)
            for (int b = 1; b < nu; b++) c = c || in_box(args.u[b], px, py);
        return c;
    };
    auto iter = [&](auto full, const double (&px)[4], const double (&py)[4], const bool (&valid)[4], uint64_t ib,
                    unsigned mw) {  // mw: the block's first mask word of this iteration (4 per iteration)
        constexpr bool FULL = decltype(full)::value;
        double T2 = __builtin_huge_val();
        const unsigned long long B = lds_fresh(kb.bound);
        if (B != kSentinelD) {
            const double t = __longlong_as_double((long long)B);
            T2 = __builtin_fmax((t * t) * kSqHi, 0x1.0p-960);
        }
        unsigned long long hb[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            bool c = in_union(px[s], py[s]);
            if (!FULL) c = c && valid[s];
            hb[s] = 0;
            // G and C (range) lie inside the union U (kNN): a slot with no point of U in the wave
            // is done after the box test (C5: 0.34% of the points lie in U)
            if (!__ballot(c)) continue;
            const double dx = args.qx - px[s], dy = args.qy - py[s];
            const double d2 = dx * dx + dy * dy;
            bool band = false;
            if (RANGE) {
                // PointPointRangeQuery.java:117-136: G -> hit; C -> dist <= r (squared screens first)
                bool g = rio.a.ng > 0 && in_box(rio.a.g[0], px[s], py[s]);
                for (int b = 1; b < rio.a.ng; b++) g = g || in_box(rio.a.g[b], px[s], py[s]);
                const bool cbox = !g && rio.a.nc && in_box(rio.a.c, px[s], py[s]);
                const bool ok = FULL || valid[s];
                bool hit = ok && (g || (rio.approximate && cbox));
                if (!rio.approximate && ok && cbox) {
                    if (d2 < rio.a.r2lo) hit = true;
                    else if (!(d2 > rio.a.r2hi)) band = true;
                }
                hb[s] = __ballot(hit);
            }
            c = c && !(d2 > T2);
            const bool stg = c || band;
            const unsigned long long m = __ballot(stg);
            if (stg) {
                const unsigned pos = ccnt + lanes_below(m);
                st.cx[pos] = px[s];
                st.cy[pos] = py[s];
                unsigned id = (unsigned)slot_index(ib, lane, s);
                if (RANGE) id |= (c ? kFlagKnn : 0u) | (band ? kFlagBand : 0u);
                st.ci[pos] = id;
            }
            ccnt += (unsigned)__popcll(m);
        }
        if (RANGE && lane < 4) {  // word q of this iteration covers points ib + 64 q .. + 63
            const int h = lane >> 1, half = lane & 1;
            const unsigned e = (unsigned)(hb[2 * h] >> (32 * half));
            const unsigned o = (unsigned)(hb[2 * h + 1] >> (32 * half));
            const unsigned long long word = spread32(e) | (spread32(o) << 1);
            if (word) atomicOr(&rmask[mw + lane], word);
        }
        wave_lds_sync();
        if (ccnt >= 64) {
            pass_dist_batch<PB, RANGE>(st, ccnt, kb, args, io, appended, false, rs);
            if (appended != last_hist && lds_fresh(kb.cnt) >= k) {
                hist_bound(kb, k, args.hist_base);
                last_hist = appended;
            }
        }
    };
    const std::integral_constant<bool, true> kFull;
    const std::integral_constant<bool, false> kPart;
    const bool all_valid[4] = {true, true, true, true};
    double ax[4], ay[4], bx[4], by[4];
    auto it_base = [&](unsigned it) {
        return kInterleave ? ((uint64_t)it * gridDim.x + blockIdx.x) * kPtsIter
                           : blk_begin + (uint64_t)it * kPtsIter;
    };
    auto is_full = [&](unsigned it) { return it_base(it) + kPtsIter <= blk_end; };
    auto load_full = [&](unsigned it, double (&px)[4], double (&py)[4]) {
        const uint64_t i0 = it_base(it) + 2 * (uint64_t)lane;
        // read once (candidates keep their coordinates in LDS): past the caches (same box, 3 reps:
        // C5 92-93 -> 84 us, C2 40.2-41.3 -> 38.4-38.7 us against plain loads)
        typedef double d2v __attribute__((ext_vector_type(2)));
        const d2v u0 = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(x + i0));
        const d2v u1 = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(x + i0 + 128));
        const d2v v0 = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(y + i0));
        const d2v v1 = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(y + i0 + 128));
        px[0] = u0.x; px[1] = u0.y; px[2] = u1.x; px[3] = u1.y;
        py[0] = v0.x; py[1] = v0.y; py[2] = v1.x; py[3] = v1.y;
    };
    auto claim = [&]() -> unsigned {
        unsigned v = 0;
        if (lane == 0) v = atomicAdd(&kb.next_it, 1u);
        return (unsigned)__builtin_amdgcn_readfirstlane((int)v);
    };
    auto run = [&](unsigned it, double (&px)[4], double (&py)[4]) {
        if (is_full(it)) {
            iter(kFull, px, py, all_valid, it_base(it), it * 4u);
        } else {
            double qx4[4], qy4[4];
            bool valid[4];
            load4(x, y, it_base(it), blk_end, lane, qx4, qy4, valid);
            iter(kPart, qx4, qy4, valid, it_base(it), it * 4u);
        }
    };
    unsigned ia = (unsigned)wid, ibb = (unsigned)(NW + wid);
    if (ia < niters && is_full(ia)) load_full(ia, ax, ay);
    if (ibb < niters && is_full(ibb)) load_full(ibb, bx, by);
    __syncthreads();
    // slot bound publication (kSlotMaxK): the waves claiming these iterations publish the
    // block's lowest survivor bin so far
    const bool slots = k <= kSlotMaxK;
    const unsigned pub1 = niters / 3, pub2 = 2 * niters / 3;
    auto publish = [&](unsigned claimed) {
        if (!slots || (claimed != pub1 && claimed != pub2)) return;
        const int bin = hist_low_bin(kb.hist);
        if (lane == 0 && bin >= 0 && bin < kHistBins - 1) store_wt(io.ctr + kMinWord + blockIdx.x, (unsigned)bin + 1u);
    };
    while (ia < niters || ibb < niters) {
        if (ia < niters) {
            const unsigned na = claim();
            run(ia, ax, ay);
            publish(na);
            ia = na;
            if (ia < niters && is_full(ia)) load_full(ia, ax, ay);
        }
        if (ibb < niters) {
            const unsigned nb2 = claim();
            run(ibb, bx, by);
            publish(nb2);
            ibb = nb2;
            if (ibb < niters && is_full(ibb)) load_full(ibb, bx, by);
        }
    }
    PASS_TRACE(io, 1);
    // the other blocks' published bins, in flight while the block's last batches finish
    unsigned gv[kPassMaxBlocks / kWave] = {};
    if (slots && wid == 0) {
#pragma unroll
        for (unsigned u = 0; u < kPassMaxBlocks / kWave; u++) {
            const unsigned b = (unsigned)lane + u * kWave;
            gv[u] = b < gridDim.x ? load_sc1(io.ctr + kMinWord + b) : 0u;
        }
    }
    pass_dist_batch<PB, RANGE>(st, ccnt, kb, args, io, appended, true, rs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // spilled survivors drained before the ticket
    __syncthreads();
    PASS_TRACE(io, 2);
    // the range hit count goes out first (later chunks wait for it); the hits themselves after
    // the kNN part, so the look-back wait never delays the kNN final
    // mask words of the block: its iterations x 4 (the ordered form's chunk [blk_begin, blk_end))
    const unsigned rnw = kInterleave ? niters * 4u
                                     : (blk_end > blk_begin ? (unsigned)((blk_end - blk_begin + 63) / 64) : 0u);
    if (RANGE) pass_range_publish<NW, UNORD>(rio, rmask, rcount, rexcl, vb, rnw);
    // ---- end of block: B (k-th bin edge) and H (kPassHeads-th bin edge) from one scan of the
    // survivor histogram; survivors <= B written unsorted to this block's list; those <= H (the
    // block's smallest, usually 8-12) placed by rank: the kPassHeads smallest are the block's
    // heads, in order.  A list whose heads may be incomplete (spilled survivors counted in the
    // histogram, > 64 entries <= H) is flagged in its length word so the final reads it whole.
    // Then the arrival (cdna_hip_programming.md §6 Guideline 16, counter form): the storing wave
    // drains its write-through stores and takes the ticket.  Common case (<= 256 survivors): wave
    // 0 alone, in registers, behind no further barrier; else every wave through LDS.
    const unsigned have = kb.cnt < (unsigned)PB::kCap ? kb.cnt : (unsigned)PB::kCap;  // block-uniform
    const size_t lbase = (size_t)blockIdx.x * io.list_cap;
    // ---- slot-complete end of block (k <= kSlotMaxK): T_b = upper edge of the bin where k of
    // the blocks' lowest survivor bins (this block's current one, the others' as published)
    // accumulate; the survivors <= T_b (the spill goes to the final on its own) into the slots
    bool slotted = false;
    if (slots && !(ABL & 7)) {
        unsigned* mh = reinterpret_cast<unsigned*>(&stage[0]);  // 512 words: the stages are idle
        if (wid == 0) {
            const int own = hist_low_bin(kb.hist);
#pragma unroll
            for (int j = 0; j < 8; j++) mh[lane * 8 + j] = 0u;
            wave_lds_sync();
#pragma unroll
            for (unsigned u = 0; u < kPassMaxBlocks / kWave; u++) {
                const unsigned b = (unsigned)lane + u * kWave;
                const int bin = b == blockIdx.x ? own : (int)gv[u] - 1;
                if (b < gridDim.x && bin >= 0 && bin < kHistBins - 1) atomicAdd(&mh[bin], 1u);
            }
            if (lane == 0 && own >= 0 && own < kHistBins - 1) store_wt(io.ctr + kMinWord + blockIdx.x, (unsigned)own + 1u);
            wave_lds_sync();
            const int tb = hist_kth_bin(mh, k);
            if (lane == 0) {
                kb.tslot = (tb >= 0 && tb < kHistBins - 1) ? hist_edge(tb, args.hist_base) : kSentinelD;
                kb.nslot = 0;
            }
        }
        __syncthreads();
        const unsigned long long T = kb.tslot;
        if (T != kSentinelD) {
            for (unsigned t = threadIdx.x; t < have; t += NT) {
                const unsigned long long d = kb.bd[t];
                if (d <= T) {
                    const unsigned p = atomicAdd(&kb.nslot, 1u);
                    if (p < kPassHeads) {
                        kb.top_d[p] = d;
                        kb.top_i[p] = kb.bi[t];
                    }
                }
            }
        }
        __syncthreads();
        const unsigned ns = kb.nslot;
        slotted = T != kSentinelD && ns <= kPassHeads;  // block-uniform
        if (slotted && wid == 0) {
            PASS_TRACE(io, 8);
            if ((unsigned)lane < kPassHeads) {
                const bool real = (unsigned)lane < ns;
                const unsigned long long d = real ? kb.top_d[lane] : kSentinelD;
                const unsigned i = real ? kb.top_i[lane] : kSentinelI;
                store_wt(&io.head_d[kPassHeads * blockIdx.x + lane], d);
                store_wt(&io.head_i[kPassHeads * blockIdx.x + lane], i);
                if (real) {  // the list holds the same set (the final's fallback paths read lists)
                    store_wt(&io.list_d[lbase + lane], d);
                    store_wt(&io.list_i[lbase + lane], i);
                }
            }
            if (lane == 0) store_wt(&io.len[blockIdx.x], ns | kLenSlots);
            PASS_TRACE(io, 10);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            PASS_TRACE(io, 3);
            if (lane == 0) kb.last = pass_arrive_last(io.ctr + kTicketStride, io.groups) ? 1u : 0u;
        }
    }
    auto bounds = [&](unsigned long long& Bv, unsigned long long& Hv) {  // wave 0
        int bb, hb;
        hist_kth_bins2(kb.hist, k, kPassHeads, bb, hb);
        Bv = kb.bound;
        if (!(ABL & 4) && kb.cnt >= k && bb >= 0 && bb < kHistBins - 1) {
            const unsigned long long e = hist_edge(bb, args.hist_base);
            if (e < Bv) Bv = e;
        }
        Hv = hb >= 0 && hb < kHistBins - 1 ? hist_edge(hb, args.hist_base) : kSentinelD;
        if (Hv > Bv) Hv = Bv;
    };
    // heads of the ns entries <= H held by the lanes of `ms` (wave 0), then the list length
    auto heads = [&](unsigned long long ms, unsigned long long d, unsigned i, unsigned ns, unsigned listed) {
        const bool small = (ms >> lane) & 1ull;
        const unsigned r = wave_rank_in(ms, d, i);
        if (small && r < kPassHeads) {
            store_wt(&io.head_d[kPassHeads * blockIdx.x + r], d);
            store_wt(&io.head_i[kPassHeads * blockIdx.x + r], i);
        }
        if ((unsigned)lane >= ns && (unsigned)lane < kPassHeads) {
            store_wt(&io.head_d[kPassHeads * blockIdx.x + lane], kSentinelD);
            store_wt(&io.head_i[kPassHeads * blockIdx.x + lane], kSentinelI);
        }
        // heads complete: every list entry <= H is among the ranked ones, and either kPassHeads
        // of them exist or the list holds nothing else
        const bool complete = ns <= (unsigned)kWave && (ns >= kPassHeads || ns == listed);
        if (lane == 0) store_wt(&io.len[blockIdx.x], listed | (complete ? 0u : kLenWhole));
        PASS_TRACE(io, 10);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PASS_TRACE(io, 3);
        if (lane == 0) kb.last = pass_arrive_last(io.ctr + kTicketStride, io.groups) ? 1u : 0u;
    };
    if (slotted) {
        // done above
    } else if (have <= 4u * kWave) {
        if (wid == 0) {  // up to 4 survivors per lane: list offsets by ballot prefix, no atomics
            unsigned long long Bv, Hv;
            bounds(Bv, Hv);
            PASS_TRACE(io, 8);
            unsigned listed = 0, ns = 0;
            for (unsigned s0 = 0; s0 < have; s0 += kWave) {
                const unsigned t = s0 + (unsigned)lane;
                unsigned long long d = kSentinelD;
                unsigned i = kSentinelI;
                if (t < have) {
                    d = kb.bd[t];
                    i = kb.bi[t];
                }
                const bool keep = t < have && d <= Bv;
                const unsigned long long m = __ballot(keep);
                if (keep && !(ABL & 1)) {
                    const unsigned p = listed + lanes_below(m);
                    store_wt(&io.list_d[lbase + p], d);
                    store_wt(&io.list_i[lbase + p], i);
                }
                listed += (unsigned)__popcll(m);
                const bool small = keep && d <= Hv;
                const unsigned long long ms = __ballot(small);
                if (small) {
                    const unsigned p = ns + lanes_below(ms);
                    if (p < (unsigned)kWave) {
                        kb.top_d[p] = d;
                        kb.top_i[p] = i;
                    }
                }
                ns += (unsigned)__popcll(ms);
            }
            wave_lds_sync();
            PASS_TRACE(io, 9);
            const unsigned nl = ns < (unsigned)kWave ? ns : (unsigned)kWave;
            unsigned long long d = kSentinelD;
            unsigned i = kSentinelI;
            if ((unsigned)lane < nl) {
                d = kb.top_d[lane];
                i = kb.top_i[lane];
            }
            heads(__ballot((unsigned)lane < nl), d, i, ns, listed);
        }
    } else {
        if (wid == 0) {
            unsigned long long Bv, Hv;
            bounds(Bv, Hv);
            if (lane == 0) {
                kb.bound = Bv;
                kb.hcap = Hv;
            }
        }
        __syncthreads();
        PASS_TRACE(io, 8);
        const unsigned long long B = kb.bound;
        const unsigned long long H = kb.hcap;
        for (unsigned t0 = 0; t0 < have; t0 += NT) {
            const unsigned t = t0 + threadIdx.x;
            unsigned long long d = kSentinelD;
            unsigned i = kSentinelI;
            if (t < have) {
                d = kb.bd[t];
                i = kb.bi[t];
            }
            const bool keep = d <= B && t < have;
            const unsigned long long m = __ballot(keep);
            unsigned wb = 0;
            if (lane == 0 && m) wb = atomicAdd(&kb.cursor, (unsigned)__popcll(m));
            wb = __shfl(wb, 0);
            if (keep && !(ABL & 1)) {
                const unsigned p = wb + lanes_below(m);
                store_wt(&io.list_d[lbase + p], d);
                store_wt(&io.list_i[lbase + p], i);
            }
            const bool small = keep && d <= H;
            const unsigned long long ms = __ballot(small);
            unsigned sb = 0;
            if (lane == 0 && ms) sb = atomicAdd(&kb.nsmall, (unsigned)__popcll(ms));
            sb = __shfl(sb, 0);
            if (small) {
                const unsigned p = sb + lanes_below(ms);
                if (p < (unsigned)kWave) {
                    kb.top_d[p] = d;
                    kb.top_i[p] = i;
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the list stores, before the ticket
        __syncthreads();
        PASS_TRACE(io, 9);
        if (wid == 0) {
            const unsigned ns = kb.nsmall;
            const unsigned nl = ns < (unsigned)kWave ? ns : (unsigned)kWave;
            unsigned long long d = kSentinelD;
            unsigned i = kSentinelI;
            if ((unsigned)lane < nl) {
                d = kb.top_d[lane];
                i = kb.top_i[lane];
            }
            heads(__ballot((unsigned)lane < nl), d, i, ns, kb.cursor);
        }
    }
    __syncthreads();
    PASS_TRACE(io, 4);
    if (kb.last == 0) {
        if (RANGE)
            pass_range_emit<NW, UNORD>(rio, rmask, rwsum, rcount, rexcl, vb, blk_begin, rnw,
                                       reinterpret_cast<unsigned*>(st.cx));
        return;
    }
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    PASS_TRACE(io, 5);
    // LDS for the final: the (idle) wave stages hold the gathered entries
    constexpr unsigned kGcap = (unsigned)(sizeof(stage) / 12) < 8u * NT ? (unsigned)(sizeof(stage) / 12) : 8u * NT;
    char* sb = reinterpret_cast<char*>(&stage[0]);
    unsigned long long* gd = reinterpret_cast<unsigned long long*>(sb);
    unsigned* gi = reinterpret_cast<unsigned*>(sb + (size_t)kGcap * 8);
    if (ABL & 8) {  // measurement: a first (cold) run of the final, then the timed (warm) one
        const unsigned long long sp = load_sc1(io.ctr);  // the spill count the final re-arms
        pass_final<NT>(io, args, gd, gi, kGcap - (kGcap & 1u), kb.hist, kb.fin, kb.bd, kb.bi, kb.bi + kPassMaxBlocks);
        __syncthreads();
        if (threadIdx.x == 0) store_wt(io.ctr, (unsigned)sp);
        __syncthreads();
        PASS_TRACE(io, 5);
    }
    pass_final<NT>(io, args, gd, gi, kGcap - (kGcap & 1u), kb.hist, kb.fin, kb.bd, kb.bi, kb.bi + kPassMaxBlocks);
    PASS_TRACE(io, 7);
    if (RANGE) {
        if (UNORD && threadIdx.x == 0) {  // every block reserved before it arrived: the total, re-armed
            *rio.total = atomicAdd(rio.cursor, 0ull);
            __hip_atomic_store(rio.cursor, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        pass_range_emit<NW, UNORD>(rio, rmask, rwsum, rcount, rexcl, vb, blk_begin, rnw,
                                   reinterpret_cast<unsigned*>(st.cx));
    }
}

// ============================================================================ range =======
constexpr int kUnitPts = 1024;  // one wave's unit: 4 iterations of 256 points; 16 mask words


struct RangeStage {
    double cx[kCandCap];
    double cy[kCandCap];
    unsigned ci[kCandCap];
    unsigned long long mask[kUnitPts / 64];
};

__device__ __forceinline__ void range_flush(RangeStage& st, unsigned& ccnt, const RangeArgs& a, uint64_t unit_base,
                                            bool partial) {
    const int lane = lane_id();
    while (ccnt >= 64 || (partial && ccnt > 0)) {
        const unsigned take = ccnt >= 64 ? 64u : ccnt;
        const unsigned from = ccnt - take;
        bool ok = (unsigned)lane < take;
        double px = 0.0, py = 0.0;
        unsigned pi = 0;
        if (ok) {
            px = st.cx[from + lane];
            py = st.cy[from + lane];
            pi = st.ci[from + lane];
        }
        wave_lds_sync();
        ccnt = from;
        ok = ok && (jts_pp_distance(a.qx, a.qy, px, py) <= a.r);
        if (ok) {
            const unsigned off = (unsigned)(pi - unit_base);
            atomicOr(&st.mask[off >> 6], 1ull << (off & 63));
        }
        wave_lds_sync();
    }
}

template <bool APPROX>
__global__ __launch_bounds__(kBlock) void range_scan(const double* __restrict__ x, const double* __restrict__ y,
                                                     uint64_t n, RangeArgs a,
                                                     unsigned long long* __restrict__ bitmask,
                                                     unsigned* __restrict__ unit_count) {
    __shared__ RangeStage stage[kBlock / kWave];
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    RangeStage& st = stage[wid];
    const uint64_t unit = (uint64_t)blockIdx.x * (kBlock / kWave) + wid;
    const uint64_t unit_base = unit * kUnitPts;
    if (unit_base >= n) return;
    if (lane < kUnitPts / 64) st.mask[lane] = 0ull;
    wave_lds_sync();
    unsigned ccnt = 0;
    for (int it = 0; it < kUnitPts / kPtsIter; it++) {
        const uint64_t base = unit_base + (uint64_t)it * kPtsIter;
        if (base >= n) break;
        double px[4], py[4];
        bool valid[4];
        load4(x, y, base, n, lane, px, py, valid);
        unsigned long long hb[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            bool g = false;
            for (int b = 0; b < a.ng; b++) g = g || in_box(a.g[b], px[s], py[s]);
            const bool cbox = !g && a.nc && in_box(a.c, px[s], py[s]);
            bool hit = valid[s] && (g || (APPROX && cbox));
            bool cand = false;
            if (!APPROX && valid[s] && cbox) {
                // squared screen: certainly inside / outside r without the exact distance
                const double dx = a.qx - px[s], dy = a.qy - py[s];
                const double d2 = dx * dx + dy * dy;
                if (d2 < a.r2lo) hit = true;
                else if (!(d2 > a.r2hi)) cand = true;
            }
            hb[s] = __ballot(hit);
            if (!APPROX) {
                const unsigned long long m = __ballot(cand);
                if (cand) {
                    const unsigned pos = ccnt + lanes_below(m);
                    st.cx[pos] = px[s];
                    st.cy[pos] = py[s];
                    st.ci[pos] = (unsigned)slot_index(base, lane, s);
                }
                ccnt += (unsigned)__popcll(m);
            }
        }
        // iteration word q (0..3) covers points base + 64q .. +63: slots (2h, 2h+1), lane half
        if (lane < 4) {
            const int h = lane >> 1, half = lane & 1;
            const unsigned e = (unsigned)(hb[2 * h] >> (32 * half));
            const unsigned o = (unsigned)(hb[2 * h + 1] >> (32 * half));
            const unsigned long long word = spread32(e) | (spread32(o) << 1);
            if (word) atomicOr(&st.mask[it * 4 + lane], word);
        }
        wave_lds_sync();
        if (!APPROX && ccnt >= 64) range_flush(st, ccnt, a, unit_base, false);
    }
    if (!APPROX) range_flush(st, ccnt, a, unit_base, true);
    wave_lds_sync();
    unsigned c = 0;
    if (lane < kUnitPts / 64) {
        const unsigned long long wv = st.mask[lane];
        bitmask[unit * (kUnitPts / 64) + lane] = wv;
        c = (unsigned)__popcll(wv);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) unit_count[unit] = c;
}

// ---- fused range pass: one launch per window.  Block vb (start order,
// from a ticket) owns units [vb U, (vb + 1) U); its 16 waves claim units from an LDS counter
// and leave each unit's hit bitmask in LDS.  The block publishes its hit count (status word
// tagged with the launch epoch), sums the counts of every earlier block (<= 255, one parallel
// read; earlier blocks started earlier and never wait on later ones), and writes its hits in
// ascending order at that offset.  The last block writes the total and re-arms the ticket.
constexpr int kRangeNW = 16;
constexpr unsigned kRangeMaxUnits = 160;  // units (1024 points) per block: 20 KB of LDS bitmask
constexpr unsigned kRangeMaxBlocks = 256;

struct RangeLookback {
    unsigned long long* status;  // kRangeMaxBlocks words: (epoch << 40) | count
    unsigned* ticket;            // zero before the first launch; re-armed by the last block
    unsigned long long epoch;    // 1 .. 2^24 - 1, new per launch
    unsigned* fault;             // set when a look-back wait gives up (poll_block_counts)
    unsigned spin_limit, inject;
};

// (Round-4 ablations of this kernel, rocprof on one box: full 47.9 us; counts only 38.7; loads
// only 30.2; no emission 40.2; no look-back wait 46.7.)
template <bool APPROX>
__global__ __launch_bounds__(kRangeNW * kWave) void range_fused(const double* __restrict__ x,
                                                                const double* __restrict__ y, uint64_t n, RangeArgs a,
                                                                unsigned upb, RangeLookback lb,
                                                                unsigned* __restrict__ out, uint64_t cap,
                                                                uint64_t* __restrict__ total) {
    constexpr int NT = kRangeNW * kWave;
    __shared__ RangeStage stage[kRangeNW];
    __shared__ unsigned long long bmask[kRangeMaxUnits * 16];
    __shared__ unsigned wpre[kRangeMaxUnits * 16];
    __shared__ unsigned wsum[kRangeNW];
    __shared__ unsigned vb_sh, next_unit, bcount;
    __shared__ unsigned long long excl_sh;
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    if (threadIdx.x == 0) {
        vb_sh = atomicAdd(lb.ticket, 1u);
        next_unit = kRangeNW;
        bcount = 0;
        excl_sh = 0;
    }
    __syncthreads();
    const unsigned vb = vb_sh;
    const uint64_t units = (n + kUnitPts - 1) / kUnitPts;
    const uint64_t u0 = (uint64_t)vb * upb;
    const unsigned nu = u0 >= units ? 0u : (unsigned)(units - u0 < upb ? units - u0 : upb);
    const uint64_t p0 = u0 * kUnitPts;
    const uint64_t p1 = p0 + (uint64_t)nu * kUnitPts < n ? p0 + (uint64_t)nu * kUnitPts : n;
    const unsigned niters = nu ? (unsigned)((p1 - p0 + kPtsIter - 1) / kPtsIter) : 0u;
    for (unsigned t = threadIdx.x; t < nu * 16; t += NT) bmask[t] = 0ull;
    __syncthreads();
    RangeStage& st = stage[wid];
    // Waves claim 256-point iterations from an LDS counter (a unit per claim left up to a third
    // of a block's waves idle at its end); hits go straight into the block's LDS bitmask, the
    // next claimed iteration's points load while the current one is classified.
    auto flush = [&](unsigned& ccnt, bool partial) {
        while (ccnt >= 64 || (partial && ccnt > 0)) {
            const unsigned take = ccnt >= 64 ? 64u : ccnt;
            const unsigned from = ccnt - take;
            bool ok = (unsigned)lane < take;
            double px = 0.0, py = 0.0;
            unsigned pi = 0;
            if (ok) {
                px = st.cx[from + lane];
                py = st.cy[from + lane];
                pi = st.ci[from + lane];
            }
            wave_lds_sync();
            ccnt = from;
            ok = ok && (jts_pp_distance(a.qx, a.qy, px, py) <= a.r);
            if (ok) {
                const unsigned off = (unsigned)(pi - p0);
                atomicOr(&bmask[off >> 6], 1ull << (off & 63));
            }
            wave_lds_sync();
        }
    };
    // the point query's boxes in registers (G is one box unless the plan is unusual)
    const Box g0 = a.g[0], c0 = a.c;
    unsigned ccnt = 0;
    double cx4[4], cy4[4];
    bool cv[4];
    unsigned it = (unsigned)wid;
    if (it < niters) load4(x, y, p0 + (uint64_t)it * kPtsIter, p1, lane, cx4, cy4, cv);
    while (it < niters) {
        const uint64_t base = p0 + (uint64_t)it * kPtsIter;
        unsigned c = 0;
        if (lane == 0) c = atomicAdd(&next_unit, 1u);
        const unsigned nit = (unsigned)__builtin_amdgcn_readfirstlane((int)c);
        double nx4[4], ny4[4];
        bool nv[4] = {false, false, false, false};
        if (nit < niters) load4(x, y, p0 + (uint64_t)nit * kPtsIter, p1, lane, nx4, ny4, nv);
        unsigned long long hb[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) {
            bool g = a.ng > 0 && in_box(g0, cx4[s4], cy4[s4]);
            for (int b = 1; b < a.ng; b++) g = g || in_box(a.g[b], cx4[s4], cy4[s4]);
            const bool cbox = !g && a.nc && in_box(c0, cx4[s4], cy4[s4]);
            bool hit = cv[s4] && (g || (APPROX && cbox));
            bool cand = false;
            if (!APPROX && cv[s4] && cbox) {
                const double dx = a.qx - cx4[s4], dy = a.qy - cy4[s4];
                const double d2 = dx * dx + dy * dy;
                if (d2 < a.r2lo) hit = true;
                else if (!(d2 > a.r2hi)) cand = true;
            }
            hb[s4] = __ballot(hit);
            if (!APPROX) {
                const unsigned long long m = __ballot(cand);
                if (cand) {
                    const unsigned pos = ccnt + lanes_below(m);
                    st.cx[pos] = cx4[s4];
                    st.cy[pos] = cy4[s4];
                    st.ci[pos] = (unsigned)slot_index(base, lane, s4);
                }
                ccnt += (unsigned)__popcll(m);
            }
        }
        // word q (0..3) of this iteration covers points base + 64q .. +63: slots (2h, 2h+1)
        if (lane < 4) {
            const int h = lane >> 1, half = lane & 1;
            const unsigned e = (unsigned)(hb[2 * h] >> (32 * half));
            const unsigned o = (unsigned)(hb[2 * h + 1] >> (32 * half));
            const unsigned long long word = spread32(e) | (spread32(o) << 1);
            if (word) atomicOr(&bmask[(unsigned)((base - p0) >> 6) + lane], word);
        }
        wave_lds_sync();
        if (!APPROX && ccnt >= 64) flush(ccnt, false);
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) {
            cx4[s4] = nx4[s4];
            cy4[s4] = ny4[s4];
            cv[s4] = nv[s4];
        }
        it = nit;
    }
    if (!APPROX) flush(ccnt, true);
    __syncthreads();
    {
        unsigned my = 0;
        for (unsigned t = threadIdx.x; t < nu * 16; t += NT) my += (unsigned)__popcll(bmask[t]);
        if (my) atomicAdd(&bcount, my);
    }
    __syncthreads();
    // publish this block's count
    const unsigned long long tag = lb.epoch << 40;
    // published with an atomic exchange: performed at the device coherence point, so the other
    // XCDs' polling loads see it at once (a plain store may sit in this XCD's L2)
    if (threadIdx.x == 0)
        (void)__hip_atomic_exchange(lb.status + vb, tag | (unsigned long long)bcount, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
    // per-word exclusive prefix of the block's bitmask (ascending point order)
    const unsigned nw = nu * 16;
    const unsigned per = (nw + NT - 1) / NT;
    const unsigned w0 = threadIdx.x * per;
    unsigned tsum = 0;
    for (unsigned k = 0; k < per; k++)
        if (w0 + k < nw) tsum += (unsigned)__popcll(bmask[w0 + k]);
    const unsigned incl = wave_incl_scan(tsum);
    if (lane == kWave - 1) wsum[wid] = incl;
    __syncthreads();
    unsigned wbase = 0;
    for (int w = 0; w < wid; w++) wbase += wsum[w];
    unsigned run = wbase + incl - tsum;
    for (unsigned k = 0; k < per; k++)
        if (w0 + k < nw) {
            wpre[w0 + k] = run;
            run += (unsigned)__popcll(bmask[w0 + k]);
        }
    // exclusive offset = sum of every earlier block's count: one wave polls (with back-off) so
    // blocks that finish early do not flood the status words while others still stream
    if (wid == 0) {
        // lane l reads predecessors l, l + 64, l + 128, l + 192 with all four loads in flight
        // (a dependent chain of device-scope loads costs a memory round trip each)
        const unsigned long long pre = poll_block_counts<kRangeMaxBlocks / kWave>(lb.status, vb, lb.epoch, lb.spin_limit,
                                                                                   lb.inject, lb.fault);
        if (lane == 0) excl_sh = pre;
    }
    __syncthreads();
    const unsigned long long excl = excl_sh;
    // Emission: each wave owns a contiguous run of words, so its hits are one contiguous run of
    // the output, written word after word (consecutive stores complete each other's lines).  Lane
    // l loads word w0 + l once; the per-word bits and offsets then come by readlane, so no LDS
    // round trip sits between two words' stores.
    {
        const unsigned wpw = (nw + kRangeNW - 1) / kRangeNW;
        const unsigned wb = (unsigned)wid * wpw;
        const unsigned we = wb + wpw < nw ? wb + wpw : nw;
        unsigned long long obase = excl + (wb < we ? wpre[wb] : 0u);
        const unsigned ibase = (unsigned)(u0 * kUnitPts) + a.point_base;
        unsigned* stg = reinterpret_cast<unsigned*>(st.cx);  // the wave's idle candidate stage
        unsigned sc = 0;
        for (unsigned w0 = wb; w0 < we; w0 += kWave) {
            const unsigned long long mine = w0 + lane < we ? bmask[w0 + lane] : 0ull;
            emit_words(mine, ibase + w0 * 64u, stg, sc, obase, out, cap);
        }
        if (sc) emit_flush(stg, sc, obase, out, cap);
    }
    if (threadIdx.x == 0 && vb == gridDim.x - 1) {
        *total = excl + bcount;
        __hip_atomic_store(lb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- range with unordered-set output (geohip_ctx_set_range_order GEOHIP_ORDER_ANY) ---------
// The reference's window result is a set: the window function collects the filter's hits as they
// arrive from the parallel filter instances (PointPointRangeQuery.java:117-136), no order promised.
// Without an order no block waits for another block's count: every wave sweeps the window in one
// grid-wide front (wave iteration gw, gw + W, ...: the blocks' stream ends bunch up, as in
// knn_pass), its hits go to an LDS buffer, and at the end each block reserves its waves' hits with
// ONE atomic and the waves store them (full 64-lane stores).  A wave whose buffer fills first
// reserves and stores a run of kSetRun on its own.  One device-scope word serves a few tens of
// returning atomics per microsecond (MI355X_MICROARCH.md "dequeue": ~88/us), so runs are long
// (a first form with 512-hit runs, ~4.3k reservations per C1-shape window, ran 67 us against 48 for
// the ordered pass) and the block's final reservation doubles as its arrival count: the word holds
// (hits << 20) | blocks arrived, and the block whose add completes the count writes the total and
// re-arms the word for the next launch.  The decisions are range_fused's (G box -> hit; C box ->
// squared screens, then the exact distance).
constexpr int kSetNW = 16;
constexpr unsigned kSetRun = 1024;   // hits per early reservation
constexpr unsigned kSetBuf = 1408;   // u32 hits per wave: <= 1023 + 319 pending at a check (5.5 KB)
constexpr unsigned kSetCand = 128;   // candidates per wave, flushed per slot at 64 (<= 63 + 64)
constexpr unsigned kSetArrivalBits = 20;

template <bool APPROX>
__global__ __launch_bounds__(kSetNW * kWave) void range_set(const double* __restrict__ x, const double* __restrict__ y,
                                                            uint64_t n, RangeArgs a, RangeSetIo io,
                                                            unsigned* __restrict__ out, uint64_t cap,
                                                            uint64_t* __restrict__ total) {
    __shared__ unsigned hbuf[kSetNW][kSetBuf];
    __shared__ double ccx[APPROX ? 1 : kSetNW][kSetCand], ccy[APPROX ? 1 : kSetNW][kSetCand];
    __shared__ unsigned cci[APPROX ? 1 : kSetNW][kSetCand];
    __shared__ unsigned s_left[kSetNW];
    __shared__ unsigned long long s_base;
    const int lane = lane_id(), wid = threadIdx.x / kWave;
    unsigned* hb = hbuf[wid];
    double* cx = ccx[APPROX ? 0 : wid];
    double* cy = ccy[APPROX ? 0 : wid];
    unsigned* ci = cci[APPROX ? 0 : wid];
    const uint64_t W = (uint64_t)gridDim.x * kSetNW;
    const uint64_t iters = (n + kPtsIter - 1) / kPtsIter;
    unsigned hc = 0;  // hits staged (wave-uniform)
    unsigned ccnt = 0;
    auto push = [&](bool hit, unsigned idx) {
        const unsigned long long m = __ballot(hit);
        if (hit) hb[hc + lanes_below(m)] = idx + a.point_base;
        hc += (unsigned)__popcll(m);
    };
    auto store = [&](unsigned long long b, unsigned from, unsigned m) {  // hb[from, from + m) -> out[b, b + m)
        for (unsigned t = (unsigned)lane; t < m; t += kWave)
            if (b + t < cap) out[b + t] = hb[from + t];
    };
    auto cand_flush = [&]() {  // the newest <= 64 candidates: exact distance, hits pushed
        const unsigned take = ccnt >= 64 ? 64u : ccnt;
        const unsigned from = ccnt - take;
        bool ok = (unsigned)lane < take;
        double px = 0.0, py = 0.0;
        unsigned pi = 0;
        if (ok) {
            px = cx[from + lane];
            py = cy[from + lane];
            pi = ci[from + lane];
        }
        wave_lds_sync();
        ccnt = from;
        ok = ok && (jts_pp_distance(a.qx, a.qy, px, py) <= a.r);
        push(ok, pi);
    };
    const Box g0 = a.g[0], c0 = a.c;
    uint64_t it = (uint64_t)blockIdx.x * kSetNW + (uint64_t)wid;
    double px4[4], py4[4];
    bool v4[4] = {false, false, false, false};
    if (it < iters) load4(x, y, it * kPtsIter, n, lane, px4, py4, v4);
    while (it < iters) {
        const uint64_t base = it * kPtsIter;
        const uint64_t nit = it + W;
        double nx4[4], ny4[4];
        bool nv[4] = {false, false, false, false};
        if (nit < iters) load4(x, y, nit * kPtsIter, n, lane, nx4, ny4, nv);
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) {
            bool g = a.ng > 0 && in_box(g0, px4[s4], py4[s4]);
            for (int b = 1; b < a.ng; b++) g = g || in_box(a.g[b], px4[s4], py4[s4]);
            const bool cbox = !g && a.nc && in_box(c0, px4[s4], py4[s4]);
            bool hit = v4[s4] && (g || (APPROX && cbox));
            bool cand = false;
            if (!APPROX && v4[s4] && cbox) {
                const double dx = a.qx - px4[s4], dy = a.qy - py4[s4];
                const double d2 = dx * dx + dy * dy;
                if (d2 < a.r2lo) hit = true;
                else if (!(d2 > a.r2hi)) cand = true;
            }
            const unsigned idx = (unsigned)slot_index(base, lane, s4);
            push(hit, idx);
            if (!APPROX) {
                const unsigned long long m = __ballot(cand);
                if (cand) {
                    const unsigned pos = ccnt + lanes_below(m);
                    cx[pos] = px4[s4];
                    cy[pos] = py4[s4];
                    ci[pos] = idx;
                }
                ccnt += (unsigned)__popcll(m);
                if (ccnt >= 64) {
                    wave_lds_sync();
                    cand_flush();
                }
            }
        }
        if (hc >= kSetRun) {  // rare (dense hits): a run of its own, the rest moved to the front
            wave_lds_sync();
            unsigned lo = 0, hi = 0;
            if (lane == 0) {
                const unsigned long long b = atomicAdd(io.word, (unsigned long long)kSetRun << kSetArrivalBits);
                lo = (unsigned)b;
                hi = (unsigned)(b >> 32);
            }
            const unsigned long long w = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)hi) << 32) |
                                         (unsigned)__builtin_amdgcn_readfirstlane((int)lo);
            store(w >> kSetArrivalBits, 0, kSetRun);
            wave_lds_sync();
            const unsigned rest = hc - kSetRun;
            for (unsigned t0 = 0; t0 < rest; t0 += kWave) {
                const unsigned t = t0 + (unsigned)lane;
                const unsigned v = t < rest ? hb[kSetRun + t] : 0u;
                wave_lds_sync();
                if (t < rest) hb[t] = v;
                wave_lds_sync();
            }
            hc = rest;
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) {
            px4[s4] = nx4[s4];
            py4[s4] = ny4[s4];
            v4[s4] = nv[s4];
        }
        it = nit;
    }
    if (!APPROX) {
        wave_lds_sync();
        while (ccnt) cand_flush();
    }
    // the block's hits: one reservation, which is also its arrival
    if (lane == 0) s_left[wid] = hc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned sum = 0;
        for (int w = 0; w < kSetNW; w++) sum += s_left[w];
        const unsigned long long old =
            atomicAdd(io.word, ((unsigned long long)sum << kSetArrivalBits) | 1ull);
        s_base = old >> kSetArrivalBits;
        if ((unsigned)(old & ((1u << kSetArrivalBits) - 1)) == gridDim.x - 1) {  // every block has reserved
            *total = (old >> kSetArrivalBits) + sum;
            __hip_atomic_store(io.word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
        }
    }
    __syncthreads();
    unsigned off = 0;
    for (int w = 0; w < wid; w++) off += s_left[w];
    store(s_base + off, 0, hc);
}

// exclusive scan of unit counts by one workgroup; total -> *total
__global__ __launch_bounds__(1024) void scan_units(const unsigned* __restrict__ cnt, uint64_t units,
                                                   uint64_t* __restrict__ offs, uint64_t* __restrict__ total) {
    __shared__ uint64_t part[1024];
    const uint64_t per = (units + blockDim.x - 1) / blockDim.x;
    const uint64_t b = threadIdx.x * per;
    uint64_t e = b + per;
    if (e > units) e = units;
    uint64_t s = 0;
    for (uint64_t u = b; u < e; u++) s += cnt[u];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < (int)blockDim.x; o <<= 1) {
        uint64_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = part[threadIdx.x] - s;
    for (uint64_t u = b; u < e; u++) {
        offs[u] = run;
        run += cnt[u];
    }
    if (threadIdx.x == blockDim.x - 1) *total = part[threadIdx.x];
}

__global__ __launch_bounds__(kBlock) void range_emit(const unsigned long long* __restrict__ bitmask,
                                                     const uint64_t* __restrict__ offs, uint64_t units,
                                                     unsigned* __restrict__ out, uint64_t cap, unsigned point_base) {
    const int lane = lane_id();
    const uint64_t unit = (uint64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
    if (unit >= units) return;
    const int wq = lane >> 2, q = lane & 3;
    unsigned bits = (unsigned)((bitmask[unit * 16 + wq] >> (16 * q)) & 0xffffull);
    const unsigned c = (unsigned)__popc(bits);
    unsigned incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    uint64_t pos = offs[unit] + (incl - c);
    const unsigned base = (unsigned)(unit * kUnitPts) + (unsigned)(wq * 64 + q * 16) + point_base;
    while (bits) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1;
        if (pos < cap) out[pos] = base + (unsigned)b;
        pos++;
    }
}

// ============================================================================ misc ========
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ double unit_uniform(uint64_t seed, uint64_t k) {
    return (double)(splitmix64(seed * 0x632BE59BD9B4E019ull + k) >> 11) * 0x1.0p-53;
}

__global__ void synth_uniform(double* __restrict__ x, double* __restrict__ y, uint64_t n, uint64_t base,
                              uint64_t seed, double min_x, double rx, double min_y, double ry) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = base + i;
        const double ux = unit_uniform(seed, 2 * g);
        const double uy = unit_uniform(seed, 2 * g + 1);
        x[i] = min_x + ux * rx;
        y[i] = min_y + uy * ry;
    }
}

__global__ void selftest_fp64(const double* __restrict__ a, const double* __restrict__ b, uint64_t n,
                              double* __restrict__ o_sqrt, double* __restrict__ o_div,
                              double* __restrict__ o_hypot, double* __restrict__ o_mulsub) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const double av = a[i], bv = b[i];
        o_sqrt[i] = __builtin_sqrt(av < 0 ? -av : av);
        o_div[i] = av / bv;
        o_hypot[i] = fdlibm_hypot(av, bv);
        o_mulsub[i] = av * bv - bv * bv;  // contraction would change these bits
    }
}

// ============================================================================ launchers ===
// kNN pass geometry: <= 256 blocks of 16 waves, block chunks of whole 256-point iterations
void knn_pass_geometry(uint64_t n, unsigned* nblocks, uint64_t* chunk) {
    uint64_t c = (n + kPassMaxBlocks - 1) / kPassMaxBlocks;
    c = (c + kPtsIter - 1) / kPtsIter * kPtsIter;
    if (c < 1024) c = 1024;
    *chunk = c;
    *nblocks = (unsigned)((n + c - 1) / c);
}

size_t knn_pass_list_entries(unsigned nblocks) {
    return (size_t)nblocks * (PassBlock<kPassNW>::kCap + kPassHeads) + nblocks;
}

bool knn_pass_fuses_range(uint64_t n) {
    unsigned nb = 0;
    uint64_t ch = 0;
    knn_pass_geometry(n, &nb, &ch);
    return ch <= 64ull * kFusedMaskWords && n < (1ull << 30);
}

hipError_t launch_knn_pass(const double* x, const double* y, uint64_t n, const KnnArgs& args,
                           unsigned long long* list_d, unsigned* list_i, unsigned long long* spill_d, unsigned* spill_i,
                           unsigned* ctr, double* out_d, unsigned* out_i, unsigned* out_count, hipStream_t st,
                           hipEvent_t ev0, hipEvent_t ev1, unsigned long long* trace, int abl,
                           const PassRangeIo* range) {
    unsigned nblocks = 0;
    uint64_t chunk = 0;
    knn_pass_geometry(n, &nblocks, &chunk);
    if (n == 0 || args.nu == 0) {  // no candidates: the empty result
        const FinalIo io{list_d, list_i, 0u, 64u, args.k, out_d, out_i, out_count, nullptr, nullptr, nullptr, nullptr,
                         nullptr, 0, nullptr};
        knn_final<1><<<1, kFinalThreads, 0, st>>>(io);
        return hipGetLastError();
    }
    const unsigned cap = (unsigned)PassBlock<kPassNW>::kCap;
    const size_t lists = (size_t)nblocks * cap;
    // list entries, then the packed heads, then the list lengths (in the index array)
    const PassIo io{list_d, list_i, cap, list_d + lists, list_i + lists, list_i + lists + (size_t)kPassHeads * nblocks,
                    spill_d, nullptr, spill_i, ctr, out_d, out_i, out_count, 16u, trace};
    PassRangeIo rio;
    memset(&rio, 0, sizeof rio);
    // ev0 / ev1 (timing on): stamped by the kernel's own dispatch begin / end
    const dim3 g(nblocks), b(kPassNW * 64);
    if (range) {
        if (!knn_pass_fuses_range(n)) return hipErrorInvalidValue;
        rio = *range;
        if (rio.unordered)
            hipExtLaunchKernelGGL(knn_pass<kPassNW, 0, true, true>, g, b, 0, st, ev0, ev1, 0, x, y, n, chunk, args, io, rio);
        else
            hipExtLaunchKernelGGL(knn_pass<kPassNW, 0, true>, g, b, 0, st, ev0, ev1, 0, x, y, n, chunk, args, io, rio);
    } else {
        switch (abl) {
            case 1: hipExtLaunchKernelGGL(knn_pass<kPassNW, 1>, g, b, 0, st, ev0, ev1, 0, x, y, n, chunk, args, io, rio); break;
            case 2: hipExtLaunchKernelGGL(knn_pass<kPassNW, 2>, g, b, 0, st, ev0, ev1, 0, x, y, n, chunk, args, io, rio); break;
            case 8: hipExtLaunchKernelGGL(knn_pass<kPassNW, 8>, g, b, 0, st, ev0, ev1, 0, x, y, n, chunk, args, io, rio); break;
            case 16: hipExtLaunchKernelGGL(knn_pass<kPassNW, 16>, g, b, 0, st, ev0, ev1, 0, x, y, n, chunk, args, io, rio); break;
            default: hipExtLaunchKernelGGL(knn_pass<kPassNW>, g, b, 0, st, ev0, ev1, 0, x, y, n, chunk, args, io, rio); break;
        }
    }
    return hipGetLastError();
}

// Rank merge for k > 256: every entry of the (<= 8192) gathered lists sorted in LDS by one
// workgroup (bitonic), the k smallest real entries written.
constexpr unsigned kMergeCap = 8192;
__global__ __launch_bounds__(1024) void knn_merge_sort(const unsigned long long* __restrict__ d,
                                                       const unsigned* __restrict__ ix, unsigned m, unsigned k,
                                                       double* __restrict__ out_d, unsigned* __restrict__ out_i,
                                                       unsigned* __restrict__ out_count) {
    __shared__ __attribute__((aligned(16))) unsigned long long sd[kMergeCap];
    __shared__ unsigned si[kMergeCap];
    __shared__ unsigned nreal;
    unsigned p2 = 1;
    while (p2 < m) p2 <<= 1;
    if (threadIdx.x == 0) nreal = 0;
    __syncthreads();
    unsigned mine = 0;
    for (unsigned t = threadIdx.x; t < p2; t += blockDim.x) {
        sd[t] = t < m ? d[t] : kSentinelD;
        si[t] = t < m ? ix[t] : kSentinelI;
        mine += (t < m && sd[t] != kSentinelD) ? 1u : 0u;
    }
    if (mine) atomicAdd(&nreal, mine);
    __syncthreads();
    block_sort_lds(sd, si, (int)p2);
    const unsigned outn = nreal < k ? nreal : k;
    for (unsigned t = threadIdx.x; t < k; t += blockDim.x) {
        out_d[t] = __longlong_as_double((long long)(t < outn ? sd[t] : kSentinelD));
        out_i[t] = t < outn ? si[t] : kSentinelI;
    }
    if (threadIdx.x == 0) *out_count = outn;
}

// per-chunk kNN lists of a host window staged in chunks: window index = chunk * chunk_pts + local
__global__ void knn_rebase(unsigned* __restrict__ idx, unsigned nlists, unsigned k, uint64_t chunk_pts) {
    const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nlists * k) return;
    const unsigned v = idx[t];
    if (v != kSentinelI) idx[t] = v + (unsigned)((uint64_t)(t / k) * chunk_pts);
}
hipError_t launch_knn_rebase(unsigned* idx, unsigned nlists, unsigned k, uint64_t chunk_pts, hipStream_t st) {
    const unsigned m = nlists * k;
    if (m) knn_rebase<<<(m + 255) / 256, 256, 0, st>>>(idx, nlists, k, chunk_pts);
    return hipGetLastError();
}

// Pane merge (sliding windows with pane reuse): the window's k smallest
// from n panes' sorted top-k lists held in a ring of slots, each pane's indices rebased by the
// pane's offset in the window.  One launch, no sort: entry e of list a (position p) lands at
// output rank p + sum over the other lists of the entries below it (binary search; keys are
// unique after the rebase, panes being disjoint), which is its place in the merged order.
__device__ __forceinline__ bool pane_less(unsigned long long ad, unsigned ai, unsigned long long bd, unsigned bi) {
    return ad < bd || (ad == bd && ai < bi);
}
// entries of list (d, i)[0, len) below key (kd, ki), rebased by off (sentinels never below)
__device__ __forceinline__ unsigned pane_below(const unsigned long long* d, const unsigned* i, unsigned len,
                                               unsigned off, unsigned long long kd, unsigned ki) {
    unsigned lo = 0, hi = len;
    while (lo < hi) {
        const unsigned mid = (lo + hi) >> 1;
        const unsigned long long md = d[mid];
        const unsigned mi = i[mid];
        const bool below = md != kSentinelD && mi != kSentinelI && pane_less(md, mi + off, kd, ki);
        if (below) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__global__ __launch_bounds__(256) void knn_merge_panes(const unsigned long long* __restrict__ ring_d,
                                                       const unsigned* __restrict__ ring_i, PaneMerge pm,
                                                       double* __restrict__ out_d, unsigned* __restrict__ out_i,
                                                       unsigned* __restrict__ out_count) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    const unsigned L = pm.list_len;
    // real entries of every pane (a list is its real entries, then sentinels)
    unsigned total = 0;
    for (unsigned b = 0; b < pm.n; b++) {
        const unsigned long long* d = ring_d + (size_t)pm.slot[b] * L;
        const unsigned* ix = ring_i + (size_t)pm.slot[b] * L;
        unsigned lo = 0, hi = L;
        while (lo < hi) {
            const unsigned mid = (lo + hi) >> 1;
            if (d[mid] != kSentinelD && ix[mid] != kSentinelI) lo = mid + 1;
            else hi = mid;
        }
        total += lo;
    }
    if (t < pm.k && t >= total) {
        out_d[t] = __longlong_as_double((long long)kSentinelD);
        out_i[t] = kSentinelI;
    }
    if (t == 0) *out_count = total < pm.k ? total : pm.k;
    if (t >= pm.n * L) return;
    const unsigned a = t / L, p = t % L;
    const unsigned long long* da = ring_d + (size_t)pm.slot[a] * L;
    const unsigned* ia = ring_i + (size_t)pm.slot[a] * L;
    const unsigned long long kd = da[p];
    const unsigned raw = ia[p];
    if (kd == kSentinelD || raw == kSentinelI) return;
    const unsigned ki = raw + pm.off[a];
    unsigned rank = p;
    for (unsigned b = 0; b < pm.n && rank < pm.k; b++)
        if (b != a)
            rank += pane_below(ring_d + (size_t)pm.slot[b] * L, ring_i + (size_t)pm.slot[b] * L, L, pm.off[b], kd, ki);
    if (rank < pm.k) {
        out_d[rank] = __longlong_as_double((long long)kd);
        out_i[rank] = ki;
    }
}

// The same merge by one workgroup when the panes' lists fit LDS (n L <= kPaneLds): every entry
// loaded once (one round trip instead of the dependent binary-search loads of the global form --
// 2 x 50-entry panes: 6.8 us of which nearly all latency), list lengths and ranks from LDS.
constexpr unsigned kPaneLds = 4096;
__global__ __launch_bounds__(1024) void knn_merge_panes_lds(const unsigned long long* __restrict__ ring_d,
                                                            const unsigned* __restrict__ ring_i, PaneMerge pm,
                                                            double* __restrict__ out_d, unsigned* __restrict__ out_i,
                                                            unsigned* __restrict__ out_count) {
    __shared__ unsigned long long sd[kPaneLds];
    __shared__ unsigned si[kPaneLds];
    __shared__ unsigned slen[kMaxPanes];
    const unsigned L = pm.list_len, m = pm.n * L;
    if (threadIdx.x < kMaxPanes) slen[threadIdx.x] = L;
    for (unsigned t = threadIdx.x; t < m; t += 1024) {
        const unsigned a = t / L, p = t - a * L;
        sd[t] = ring_d[(size_t)pm.slot[a] * L + p];
        si[t] = ring_i[(size_t)pm.slot[a] * L + p];
    }
    __syncthreads();
    // a list is its real entries, then sentinels: its length = its first sentinel
    for (unsigned t = threadIdx.x; t < m; t += 1024)
        if (sd[t] == kSentinelD || si[t] == kSentinelI) atomicMin(&slen[t / L], t - (t / L) * L);
    __syncthreads();
    unsigned total = 0;
    for (unsigned b = 0; b < pm.n; b++) total += slen[b];
    for (unsigned t = threadIdx.x; t < pm.k; t += 1024)
        if (t >= total) {
            out_d[t] = __longlong_as_double((long long)kSentinelD);
            out_i[t] = kSentinelI;
        }
    if (threadIdx.x == 0) *out_count = total < pm.k ? total : pm.k;
    for (unsigned t = threadIdx.x; t < m; t += 1024) {
        const unsigned a = t / L, p = t - a * L;
        if (p >= slen[a]) continue;
        const unsigned long long kd = sd[t];
        const unsigned ki = si[t] + pm.off[a];
        unsigned rank = p;
        for (unsigned b = 0; b < pm.n && rank < pm.k; b++)
            if (b != a) rank += pane_below(sd + b * L, si + b * L, slen[b], pm.off[b], kd, ki);
        if (rank < pm.k) {
            out_d[rank] = __longlong_as_double((long long)kd);
            out_i[rank] = ki;
        }
    }
}

hipError_t launch_knn_merge_panes(const unsigned long long* ring_d, const unsigned* ring_i, const PaneMerge& pm,
                                  double* out_d, unsigned* out_i, unsigned* out_count, hipStream_t st, hipEvent_t ev0,
                                  hipEvent_t ev1) {
    if ((uint64_t)pm.n * pm.list_len <= kPaneLds) {
        hipExtLaunchKernelGGL(knn_merge_panes_lds, dim3(1), dim3(1024), 0, st, ev0, ev1, 0, ring_d, ring_i, pm, out_d, out_i,
                              out_count);
        return hipGetLastError();
    }
    const unsigned m = pm.n * pm.list_len > pm.k ? pm.n * pm.list_len : pm.k;
    hipExtLaunchKernelGGL(knn_merge_panes, dim3((m + 255) / 256), dim3(256), 0, st, ev0, ev1, 0, ring_d, ring_i, pm, out_d,
                          out_i, out_count);
    return hipGetLastError();
}

hipError_t launch_knn_merge(const unsigned long long* d, const unsigned* i, unsigned nlists, unsigned list_len,
                            unsigned k, double* out_d, unsigned* out_i, unsigned* out_count, hipStream_t st) {
    if (k > 256) {
        const uint64_t m = (uint64_t)nlists * list_len;
        if (m > kMergeCap) return hipErrorInvalidValue;
        knn_merge_sort<<<1, 1024, 0, st>>>(d, i, (unsigned)m, k, out_d, out_i, out_count);
        return hipGetLastError();
    }
    const FinalIo io{d, i, nlists, list_len, k, out_d, out_i, out_count, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                     nullptr};
    if (k <= 64) knn_final<1><<<1, kFinalThreads, 0, st>>>(io);
    else if (k <= 128) knn_final<2><<<1, kFinalThreads, 0, st>>>(io);
    else knn_final<4><<<1, kFinalThreads, 0, st>>>(io);
    return hipGetLastError();
}


bool range_is_one_kernel(uint64_t n) {
    const uint64_t units = (n + kUnitPts - 1) / kUnitPts;
    return units > 0 && units <= (uint64_t)kRangeMaxBlocks * kRangeMaxUnits;
}

hipError_t launch_range(const double* x, const double* y, uint64_t n, const RangeArgs& a, int approximate,
                        unsigned long long* bitmask, unsigned* unit_count, uint64_t* offs, uint64_t* total,
                        unsigned* out, uint64_t cap, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1,
                        unsigned long long* lb_status, unsigned* lb_ticket, unsigned long long epoch,
                        unsigned* lb_fault, unsigned lb_spins, unsigned lb_inject) {
    const uint64_t units = (n + kUnitPts - 1) / kUnitPts;
    if (units == 0) return hipMemsetAsync(total, 0, sizeof(uint64_t), st);
    if (lb_status && units <= (uint64_t)kRangeMaxBlocks * kRangeMaxUnits) {
        // one fused launch: <= 256 blocks of upb units
        const unsigned upb = (unsigned)((units + kRangeMaxBlocks - 1) / kRangeMaxBlocks);
        const unsigned nblocks = (unsigned)((units + upb - 1) / upb);
        const RangeLookback lb{lb_status, lb_ticket, epoch, lb_fault, lb_spins, lb_inject};
        // one kernel: ev0 / ev1 stamped by its dispatch
        const dim3 g(nblocks), b(kRangeNW * kWave);
        if (approximate)
            hipExtLaunchKernelGGL(range_fused<true>, g, b, 0, st, ev0, ev1, 0, x, y, n, a, upb, lb, out, cap, total);
        else
            hipExtLaunchKernelGGL(range_fused<false>, g, b, 0, st, ev0, ev1, 0, x, y, n, a, upb, lb,
                                  out, cap, total);
        return hipGetLastError();
    }
    const uint64_t blocks = (units + 3) / 4;
    if (ev0) (void)hipEventRecord(ev0, st);
    if (approximate) range_scan<true><<<(unsigned)blocks, kBlock, 0, st>>>(x, y, n, a, bitmask, unit_count);
    else range_scan<false><<<(unsigned)blocks, kBlock, 0, st>>>(x, y, n, a, bitmask, unit_count);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    scan_units<<<1, 1024, 0, st>>>(unit_count, units, offs, total);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    range_emit<<<(unsigned)blocks, kBlock, 0, st>>>(bitmask, offs, units, out, cap, a.point_base);
    if (ev1) (void)hipEventRecord(ev1, st);  // timed region: all three kernels
    return hipGetLastError();
}

hipError_t launch_range_set(const double* x, const double* y, uint64_t n, const RangeArgs& a, int approximate,
                            const RangeSetIo& io, uint64_t* total, unsigned* out, uint64_t cap, unsigned cus,
                            hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
    const uint64_t iters = (n + kPtsIter - 1) / kPtsIter;
    if (iters == 0) return hipMemsetAsync(total, 0, sizeof(uint64_t), st);
    // one block of 16 waves per CU (128 KB of LDS), fewer for small windows
    const uint64_t want = (iters + kSetNW - 1) / kSetNW;
    const unsigned nblocks = (unsigned)(want < cus ? want : cus);
    const dim3 g(nblocks), b(kSetNW * kWave);
    if (approximate)
        hipExtLaunchKernelGGL(range_set<true>, g, b, 0, st, ev0, ev1, 0, x, y, n, a, io, out, cap, total);
    else
        hipExtLaunchKernelGGL(range_set<false>, g, b, 0, st, ev0, ev1, 0, x, y, n, a, io, out, cap, total);
    return hipGetLastError();
}

hipError_t launch_synth_uniform(double* x, double* y, uint64_t n, uint64_t base, uint64_t seed, double min_x,
                                double max_x, double min_y, double max_y, hipStream_t st) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    synth_uniform<<<(unsigned)blocks, 256, 0, st>>>(x, y, n, base, seed, min_x, max_x - min_x, min_y, max_y - min_y);
    return hipGetLastError();
}

hipError_t launch_selftest_fp64(const double* a, const double* b, uint64_t n, double* o_sqrt, double* o_div,
                                double* o_hypot, double* o_mulsub, hipStream_t st) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    selftest_fp64<<<(unsigned)blocks, 256, 0, st>>>(a, b, n, o_sqrt, o_div, o_hypot, o_mulsub);
    return hipGetLastError();
}

}  // namespace geohip
