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
#include <hip/hip_runtime.h>
#include <stdint.h>

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
constexpr int kBlkCap = 768;  // 4 blocks/CU: stages 25.6 KB + this ~11.3 KB <= 40 KB

struct KnnBlock {
    unsigned hist[kHistBins];
    unsigned long long bd[kBlkCap];
    unsigned bi[kBlkCap];
    unsigned long long bound;  // distance bits; kSentinelD = none yet
    unsigned cnt;              // survivors appended (may exceed kBlkCap: the rest spilled)
    unsigned final_cnt;
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
    unsigned incl = tot;  // inclusive prefix over lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    const unsigned long long m = __ballot(incl >= k);
    if (m == 0) return -1;
    const int first = __builtin_ctzll(m);
    int bin = kHistBins - 1;
    if (lane == first) {
        unsigned run = incl - tot;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            run += c[j];
            if (run >= k) { bin = lane * 8 + j; break; }
        }
    }
    return __shfl(bin, first);
}

// upper edge (distance bits) of histogram bin `bin`
__device__ __forceinline__ unsigned long long hist_edge(int bin, int base) {
    return ((unsigned long long)(bin + base + 1) << 48) - 1ull;
}

// One wave: the block bound from the survivor histogram (LDS atomic min).
__device__ __forceinline__ void hist_bound(KnnBlock& kb, unsigned k, int base) {
    const int bin = hist_kth_bin(kb.hist, k);
    if (bin >= 0 && bin < kHistBins - 1 && lane_id() == 0) atomicMin(&kb.bound, hist_edge(bin, base));
}

// exact distances of up to 64 staged candidates, survivors appended to the block buffer
__device__ __forceinline__ void knn_dist_batch(WaveStage& st, unsigned& ccnt, KnnBlock& kb, const KnnArgs& a,
                                               unsigned long long* __restrict__ spill_d,
                                               unsigned* __restrict__ spill_i, unsigned* __restrict__ spill_cnt,
                                               unsigned& appended, bool partial) {
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
        ok = ok && db <= B;
        const unsigned long long m = __ballot(ok);
        if (m) {
            const unsigned nm = (unsigned)__popcll(m);
            unsigned pos = 0;
            if (lane == 0) pos = atomicAdd(&kb.cnt, nm);
            pos = __shfl(pos, 0);
            const unsigned slot = pos + lanes_below(m);
            unsigned gbase = 0;
            if (pos + nm > (unsigned)kBlkCap) {  // spill the overflow to global memory (rare)
                const unsigned first = pos > (unsigned)kBlkCap ? pos : (unsigned)kBlkCap;
                if (lane == 0) gbase = atomicAdd(spill_cnt, pos + nm - first);
                gbase = __shfl(gbase, 0) - (first - pos);
            }
            if (ok) {
                if (slot < (unsigned)kBlkCap) {
                    kb.bd[slot] = db;
                    kb.bi[slot] = pi;
                } else {
                    store_wt(&spill_d[gbase + (slot - pos)], db);
                    store_wt(&spill_i[gbase + (slot - pos)], pi);
                }
                atomicAdd(&kb.hist[hist_bin(db, a.hist_base)], 1u);
            }
            appended += nm;
        }
        wave_lds_sync();
    }
}

// ---------------------------------------------------------------- final selection --------
// final_select<KPL, NT, OWN>: NT threads (NT/64 waves) reduce nlists ascending lists of
// list_len entries (plus the unsorted spill buffer) to the k smallest keys.
//  (1) every wave sorts its 64-head batches in registers and the wave runs are merged by a
//      tree through LDS: T = k-th smallest head, an upper bound of the global k-th key (the k
//      smallest heads are k real entries);
//  (2) every entry <= T is gathered (lists ascending: a list scan stops at the first entry
//      above T; ~k entries in all, nearly always within the two entries preloaded per list);
//  (3) one wave sorts them in registers and writes the top k.
// Every global load of (1)-(2) is issued up front (OWN lists of two entries per thread and the
// spill count), so the selection pays one memory latency.  It runs as the knn_final kernel
// (merges of rank results) and inside knn_scan's last-arriving block.
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
    int hist_base;                     // histogram origin for the head-histogram T (head_d != null)
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
    unsigned* hist;          // kHistBins words (used with FinalIo::head_d)
};

template <int KPL, int NT, int OWN>
__device__ void final_select(const FinalIo& io, const FinalLds& s) {
    constexpr int N = 64 * KPL;
    constexpr int KPL2 = 2 * KPL;
    constexpr int NW = NT / kWave;
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    const unsigned nlists = io.nlists, list_len = io.list_len, k = io.k;
    if (threadIdx.x == 0) {
        *s.cnt = 0;
        *s.Td = kSentinelD;
        *s.Ti = kSentinelI;
    }
    unsigned nspill = 0;
    if (io.spill_cnt) nspill = __hip_atomic_load(io.spill_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    // (1a) T from a histogram of the heads (LDS atomics, one wave scan): the upper edge of the
    // bin where the cumulative head count reaches k.  >= k heads lie at or below it, so it is a
    // valid T; left unresolved (exact path below) when that bin is the lowest or the top one.
    bool resolved = false;
    if (nlists >= k && io.head_d && OWN * NT >= (int)nlists) {
        for (int t = threadIdx.x; t < kHistBins; t += NT) s.hist[t] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < OWN; j++)
            if (e[j][0].d != kSentinelD) atomicAdd(&s.hist[hist_bin(e[j][0].d, io.hist_base)], 1u);
        __syncthreads();
        if (wid == 0) {
            const int bin = hist_kth_bin(s.hist, k);
            if (lane == 0 && bin > 0 && bin < kHistBins - 1) {
                *s.Td = hist_edge(bin, io.hist_base);
                *s.Ti = kSentinelI;
            }
        }
        __syncthreads();
        resolved = *s.Td != kSentinelD;
    }
    // (1b) exact: T = k-th smallest head
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
    const unsigned long long T_d = *s.Td;
    const unsigned T_i = *s.Ti;
    // (2) gather every real entry <= T
    auto take = [&](const KE& e) -> bool {
        if (e.d == kSentinelD || lds_kless(T_d, T_i, e.d, e.i)) return false;
        const unsigned pos = atomicAdd(s.cnt, 1u);
        if (pos < s.cap) {
            s.bd[pos] = e.d;
            s.bi[pos] = e.i;
        }
        return true;
    };
#pragma unroll
    for (int j = 0; j < OWN; j++) {
        const unsigned own = threadIdx.x + (unsigned)(j * NT);
        if (own >= nlists) continue;
        bool more = true;
#pragma unroll
        for (int h = 0; h < kHeads; h++) more = more && take(e[j][h]);
        if (more) {  // all preloaded entries taken: the rest of the list from memory (rare)
            const size_t off = (size_t)own * list_len;
            for (unsigned q = kHeads; q < list_len; q++) {
                KE e;
                e.d = io.part_d[off + q];
                e.i = io.part_i[off + q];
                if (!take(e)) break;
            }
        }
    }
    for (unsigned p = threadIdx.x + (unsigned)(OWN * NT); p < nlists; p += NT) {
        const size_t off = (size_t)p * list_len;
        for (unsigned q = 0; q < list_len; q++) {
            KE e;
            e.d = io.part_d[off + q];
            e.i = io.part_i[off + q];
            if (!take(e)) break;
        }
    }
    // survivors a scan block could not keep in LDS (unsorted, usually none)
    for (unsigned t = threadIdx.x; t < nspill; t += NT) {
        KE e;
        e.d = io.spill_d[t];
        e.i = io.spill_i[t];
        take(e);
    }
    __syncthreads();
    if (io.spill_cnt && threadIdx.x == 0) *io.spill_cnt = 0;  // ready for the next window on this stream
    const unsigned total = *s.cnt;
    const unsigned outn = total < k ? total : k;
    if (total <= (unsigned)(64 * KPL2)) {
        // (3) one wave: register bitonic sort of <= 128*KPL entries
        if (wid == 0) {
            WList<KPL2> S;
#pragma unroll
            for (int q = 0; q < KPL2; q++) {
                const unsigned e = (unsigned)(q * 64 + lane);
                S.s[q] = ksentinel();
                if (e < total) {
                    S.s[q].d = s.bd[e];
                    S.s[q].i = s.bi[e];
                }
            }
            wave_sort_list<KPL2>(S);
#pragma unroll
            for (int q = 0; q < KPL2; q++) {
                const unsigned e = (unsigned)(q * 64 + lane);
                if (e < k) {
                    io.out_d[e] = __longlong_as_double((long long)(e < outn ? S.s[q].d : kSentinelD));
                    io.out_i[e] = e < outn ? S.s[q].i : kSentinelI;
                }
            }
            if (lane == 0) *io.out_count = outn;
        }
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

// Where a scan writes its result.  ticket != null: the block lists are stored write-through
// (sc1) and the last block to take a ticket runs final_select into out_* (one launch per
// window); ticket == null: only the block lists are written (knn_final merges them).
struct KnnOut {
    double* out_d;
    unsigned* out_i;
    unsigned* out_count;
    unsigned* ticket;  // zero before the first launch; the last arriver re-zeroes it
};


// MODE (ablation builds for measurement only; the product launches MODE 0):
//   0 full, 1 loads only, 2 loads + classification, 3 + LDS staging and distances (no selection),
//   5 full + counters (survivors, spilled), 7 full without the end-of-block selection
template <int KPL, int MODE = 0>
__global__ __launch_bounds__(kBlock) void knn_scan(const double* __restrict__ x, const double* __restrict__ y,
                                                   uint64_t n, uint64_t chunk, KnnArgs args,
                                                   unsigned long long* __restrict__ part_d,
                                                   unsigned* __restrict__ part_i,
                                                   unsigned long long* __restrict__ spill_d,
                                                   unsigned* __restrict__ spill_i, unsigned* __restrict__ spill_cnt,
                                                   KnnOut out) {
    __shared__ WaveStage stage[kBlock / kWave];
    __shared__ KnnBlock kb;
    const int lane = lane_id();
    const int wid = threadIdx.x / kWave;
    WaveStage& st = stage[wid];
    const uint64_t blk_begin = (uint64_t)blockIdx.x * chunk;
    uint64_t blk_end = blk_begin + chunk;
    if (blk_end > n) blk_end = n;
    for (int t = threadIdx.x; t < kHistBins; t += kBlock) kb.hist[t] = 0;
    if (threadIdx.x == 0) {
        kb.bound = kSentinelD;
        kb.cnt = 0;
    }
    __syncthreads();

    const unsigned k = args.k;
    unsigned ccnt = 0;
    unsigned appended = 0, last_hist = 0;

    // software pipeline: the next iteration's 4 KB per wave is in flight while this one is
    // classified
    constexpr uint64_t kStride = (uint64_t)(kBlock / kWave) * kPtsIter;
    uint64_t base = blk_begin + (uint64_t)wid * kPtsIter;
    double sink = 0.0;
    double nx[4], ny[4];
    bool nv[4];
    if (base < blk_end) load4(x, y, base, blk_end, lane, nx, ny, nv);
    for (; base < blk_end; base += kStride) {
        double px[4], py[4];
        bool valid[4];
#pragma unroll
        for (int s = 0; s < 4; s++) { px[s] = nx[s]; py[s] = ny[s]; valid[s] = nv[s]; }
        if (base + kStride < blk_end) load4(x, y, base + kStride, blk_end, lane, nx, ny, nv);
        if (MODE == 1) {
#pragma unroll
            for (int s = 0; s < 4; s++) sink += px[s] + py[s];
            continue;
        }
        // squared screen against the block bound: only candidates that may beat it reach the
        // exact fdlibm distance
        double T2 = __builtin_huge_val();
        if (MODE == 0 || MODE >= 5) {
            const unsigned long long B = lds_fresh(kb.bound);
            if (B != kSentinelD) {
                const double t = __longlong_as_double((long long)B);
                T2 = (t * t) * kSqHi;
            }
        }
#pragma unroll
        for (int s = 0; s < 4; s++) {
            bool c = false;
            for (int b = 0; b < args.nu; b++) c = c || in_box(args.u[b], px[s], py[s]);
            c = c && valid[s];
            if (MODE == 0 || MODE >= 5) {
                const double dx = args.qx - px[s], dy = args.qy - py[s];
                const double d2 = dx * dx + dy * dy;
                c = c && !(d2 > T2);
            }
            const unsigned long long m = __ballot(c);
            if (MODE == 2) {
                sink += (double)__popcll(m);
                continue;
            }
            if (c) {
                const unsigned pos = ccnt + lanes_below(m);
                st.cx[pos] = px[s];
                st.cy[pos] = py[s];
                st.ci[pos] = (unsigned)slot_index(base, lane, s);
            }
            ccnt += (unsigned)__popcll(m);
        }
        if (MODE == 2) continue;
        wave_lds_sync();
        if (MODE == 3) {
            while (ccnt >= 64) {
                const unsigned from = ccnt - 64;
                sink += jts_pp_distance(args.qx, args.qy, st.cx[from + lane], st.cy[from + lane]);
                wave_lds_sync();
                ccnt = from;
            }
            continue;
        }
        if (ccnt >= 64) {
            knn_dist_batch(st, ccnt, kb, args, spill_d, spill_i, spill_cnt, appended, false);
            // refresh the block bound once this wave has added survivors
            if (appended != last_hist && lds_fresh(kb.cnt) >= k) {
                hist_bound(kb, k, args.hist_base);
                last_hist = appended;
            }
        }
    }
    if (MODE >= 1 && MODE <= 3) {
        if (sink == 12345.678) part_d[blockIdx.x] = 1;  // keep the ablated work alive
        return;
    }
    knn_dist_batch(st, ccnt, kb, args, spill_d, spill_i, spill_cnt, appended, true);
    if (MODE == 5) {
        if (lane == 0) atomicAdd(&part_i[0], appended);
        return;
    }
    if (MODE == 7) {
        if (appended == 12345) part_d[blockIdx.x] = 1;
        return;
    }

    // ---- end of block: keep the survivors <= final bound, sort once, write the block list
    constexpr int N = 64 * KPL;
    constexpr int KPL2 = 2 * KPL;
    __syncthreads();
    if (wid == 0 && kb.cnt >= k) hist_bound(kb, k, args.hist_base);
    if (threadIdx.x == 0) kb.final_cnt = 0;
    __syncthreads();
    const unsigned long long B = kb.bound;
    const unsigned have = kb.cnt < (unsigned)kBlkCap ? kb.cnt : (unsigned)kBlkCap;
    // compact survivors <= B into the (now idle) wave stages
    unsigned long long* cd = reinterpret_cast<unsigned long long*>(&stage[0].cx[0]);
    unsigned* ci = reinterpret_cast<unsigned*>(&stage[2].cx[0]);
    for (unsigned t0 = 0; t0 < have; t0 += kBlock) {
        const unsigned t = t0 + threadIdx.x;
        const bool keep = t < have && kb.bd[t] <= B;
        const unsigned long long m = __ballot(keep);
        unsigned wbase = 0;
        if (lane == 0 && m) wbase = atomicAdd(&kb.final_cnt, (unsigned)__popcll(m));
        wbase = __shfl(wbase, 0);
        if (keep) {
            const unsigned pos = wbase + lanes_below(m);
            cd[pos] = kb.bd[t];
            ci[pos] = kb.bi[t];
        }
    }
    __syncthreads();
    const unsigned fc = kb.final_cnt;
    const size_t off = (size_t)blockIdx.x * N;
    // packed heads behind the lists (FinalIo::head_d)
    unsigned long long* head_d = part_d + (size_t)gridDim.x * N;
    unsigned* head_i = part_i + (size_t)gridDim.x * N;
    if (fc <= 64u && KPL == 1) {
        if (wid == 0) {  // common case: one 64-lane register sort
            KE e = ksentinel();
            if ((unsigned)lane < fc) { e.d = cd[lane]; e.i = ci[lane]; }
            e = wave_sort64(e);
            store_wt(&part_d[off + lane], e.d);
            store_wt(&part_i[off + lane], e.i);
            if (lane < kHeads) {
                store_wt(&head_d[kHeads * blockIdx.x + lane], e.d);
                store_wt(&head_i[kHeads * blockIdx.x + lane], e.i);
            }
        }
    } else if (fc <= (unsigned)(64 * KPL2)) {
        if (wid == 0) {
            WList<KPL2> S;
#pragma unroll
            for (int s = 0; s < KPL2; s++) {
                const unsigned e = (unsigned)(s * 64 + lane);
                S.s[s] = ksentinel();
                if (e < fc) { S.s[s].d = cd[e]; S.s[s].i = ci[e]; }
            }
            wave_sort_list<KPL2>(S);
#pragma unroll
            for (int s = 0; s < KPL; s++) {
                store_wt(&part_d[off + s * 64 + lane], S.s[s].d);
                store_wt(&part_i[off + s * 64 + lane], S.s[s].i);
            }
            if (lane < kHeads) {
                store_wt(&head_d[kHeads * blockIdx.x + lane], S.s[0].d);
                store_wt(&head_i[kHeads * blockIdx.x + lane], S.s[0].i);
            }
        }
    } else {
        // many exact ties around the bound: sort all kept survivors in LDS (uniform branch)
        int m2 = 1;
        while (m2 < (int)fc) m2 <<= 1;
        for (int t = threadIdx.x + fc; t < m2; t += kBlock) { cd[t] = kSentinelD; ci[t] = kSentinelI; }
        __syncthreads();
        block_sort_lds(cd, ci, m2);
        for (int t = threadIdx.x; t < N; t += kBlock) {
            store_wt(&part_d[off + t], t < (int)fc ? cd[t] : kSentinelD);
            store_wt(&part_i[off + t], t < (int)fc ? ci[t] : kSentinelI);
            if (t < kHeads) {
                store_wt(&head_d[kHeads * blockIdx.x + t], cd[t]);  // fc > 64*KPL2 >= kHeads
                store_wt(&head_i[kHeads * blockIdx.x + t], ci[t]);
            }
        }
    }
    if (out.ticket == nullptr) return;

    // ---- fused final selection (cdna_hip_programming.md §6 Guideline 16, counter form): the
    // block list (and any spill) was stored sc1; every storing wave drains, the block meets,
    // one lane takes a ticket; the last arriver acquires once and merges all block lists.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(((gu32*)(out.ticket)), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        kb.final_cnt = t == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (kb.final_cnt == 0) return;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // LDS: gathered entries in the (idle) wave stages, tree exchange in kb.bd/kb.bi
    static_assert(sizeof(stage) >= 2048 * 12, "fused final: gather buffer");
    static_assert(sizeof(kb.bd) >= 2 * N * 8 && sizeof(kb.bi) >= 2 * N * 4, "fused final: tree exchange");
    char* sb = reinterpret_cast<char*>(&stage[0]);
    const FinalLds fl{kb.bd, kb.bi, reinterpret_cast<unsigned long long*>(sb), reinterpret_cast<unsigned*>(sb + 2048 * 8),
                      2048u, &kb.cnt, &kb.bound, &kb.final_cnt, kb.hist};
    const FinalIo io{part_d, part_i, gridDim.x, (unsigned)N, k, out.out_d, out.out_i, out.out_count,
                     spill_d, spill_i, spill_cnt, head_d, head_i, args.hist_base};
    final_select<KPL, kBlock, 1024 / kBlock>(io, fl);
    if (threadIdx.x == 0) __hip_atomic_store(((gu32*)(out.ticket)), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ============================================================================ range =======
constexpr int kUnitPts = 1024;  // one wave's unit: 4 iterations of 256 points; 16 mask words

__device__ __forceinline__ unsigned long long spread32(unsigned v) {  // bit b -> bit 2b
    unsigned long long x = v;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

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
                                                     unsigned* __restrict__ out, uint64_t cap) {
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
    const unsigned base = (unsigned)(unit * kUnitPts) + (unsigned)(wq * 64 + q * 16);
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
static int g_knn_fused = 1;
void set_knn_fused(int fused) { g_knn_fused = fused; }

template <int KPL>
static void launch_knn_final_heads(unsigned long long* part_d, unsigned* part_i, unsigned nblocks, unsigned k,
                                   double* out_d, unsigned* out_i, unsigned* out_count,
                                   unsigned long long* spill_d, unsigned* spill_i, unsigned* spill_cnt, int hist_base,
                                   hipStream_t st) {
    const unsigned L = 64u * KPL;
    const FinalIo io{part_d, part_i, nblocks, L, k, out_d, out_i, out_count, spill_d, spill_i, spill_cnt,
                     part_d + (size_t)nblocks * L, part_i + (size_t)nblocks * L, hist_base};
    knn_final<KPL><<<1, kFinalThreads, 0, st>>>(io);
}

hipError_t launch_knn(const double* x, const double* y, uint64_t n, const KnnArgs& args, int kpl,
                      unsigned long long* part_d, unsigned* part_i, unsigned nblocks, uint64_t chunk, double* out_d,
                      unsigned* out_i, unsigned* out_count, unsigned long long* spill_d, unsigned* spill_i,
                      unsigned* spill_cnt, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
    const unsigned k = args.k;
    const unsigned L = 64u * (unsigned)kpl;
    if (nblocks == 0) {  // empty window: the final selection alone writes the empty result
        const FinalIo io{part_d, part_i, 0u, L, k, out_d, out_i, out_count, spill_d, spill_i, spill_cnt, nullptr, nullptr, 0};
        if (k <= 64) knn_final<1><<<1, kFinalThreads, 0, st>>>(io);
        else if (k <= 128) knn_final<2><<<1, kFinalThreads, 0, st>>>(io);
        else knn_final<4><<<1, kFinalThreads, 0, st>>>(io);
        return hipGetLastError();
    }
    // fused: spill_cnt[1] is the arrival ticket of the in-kernel final selection
    const KnnOut out = g_knn_fused ? KnnOut{out_d, out_i, out_count, spill_cnt + 1} : KnnOut{nullptr, nullptr, nullptr, nullptr};
    if (ev0) (void)hipEventRecord(ev0, st);
    switch (kpl) {
        case 1: knn_scan<1><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, out); break;
        case 2: knn_scan<2><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, out); break;
        case 4: knn_scan<4><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, out); break;
        default: return hipErrorInvalidValue;
    }
    if (ev1) (void)hipEventRecord(ev1, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || g_knn_fused) return e;
    switch (kpl) {
        case 1: launch_knn_final_heads<1>(part_d, part_i, nblocks, k, out_d, out_i, out_count, spill_d, spill_i, spill_cnt, args.hist_base, st); break;
        case 2: launch_knn_final_heads<2>(part_d, part_i, nblocks, k, out_d, out_i, out_count, spill_d, spill_i, spill_cnt, args.hist_base, st); break;
        default: launch_knn_final_heads<4>(part_d, part_i, nblocks, k, out_d, out_i, out_count, spill_d, spill_i, spill_cnt, args.hist_base, st); break;
    }
    return hipGetLastError();
}

hipError_t launch_knn_scan_variant(int mode, const double* x, const double* y, uint64_t n, const KnnArgs& args,
                                   unsigned long long* part_d, unsigned* part_i, unsigned nblocks, uint64_t chunk,
                                   unsigned long long* spill_d, unsigned* spill_i, unsigned* spill_cnt, double* out_d,
                                   unsigned* out_i, unsigned* out_count, hipStream_t st) {
    const KnnOut fused{out_d, out_i, out_count, spill_cnt + 1};
    const KnnOut lists{nullptr, nullptr, nullptr, nullptr};
    switch (mode) {
        case 0: knn_scan<1, 0><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, fused); break;
        case 1: knn_scan<1, 1><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, lists); break;
        case 2: knn_scan<1, 2><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, lists); break;
        case 3: knn_scan<1, 3><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, lists); break;
        case 5: knn_scan<1, 5><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, lists); break;
        case 7: knn_scan<1, 7><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, lists); break;
        case 8: knn_scan<1, 0><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, lists); break;
        case 9:
            knn_scan<1, 0><<<nblocks, kBlock, 0, st>>>(x, y, n, chunk, args, part_d, part_i, spill_d, spill_i, spill_cnt, lists);
            launch_knn_final_heads<1>(part_d, part_i, nblocks, args.k, out_d, out_i, out_count, spill_d, spill_i, spill_cnt,
                                      args.hist_base, st);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_knn_merge(const unsigned long long* d, const unsigned* i, unsigned nlists, unsigned list_len,
                            unsigned k, double* out_d, unsigned* out_i, unsigned* out_count, hipStream_t st) {
    const FinalIo io{d, i, nlists, list_len, k, out_d, out_i, out_count, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
    if (k <= 64) knn_final<1><<<1, kFinalThreads, 0, st>>>(io);
    else if (k <= 128) knn_final<2><<<1, kFinalThreads, 0, st>>>(io);
    else knn_final<4><<<1, kFinalThreads, 0, st>>>(io);
    return hipGetLastError();
}

hipError_t launch_range(const double* x, const double* y, uint64_t n, const RangeArgs& a, int approximate,
                        unsigned long long* bitmask, unsigned* unit_count, uint64_t* offs, uint64_t* total,
                        unsigned* out, uint64_t cap, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
    const uint64_t units = (n + kUnitPts - 1) / kUnitPts;
    const uint64_t blocks = (units + 3) / 4;
    if (units == 0) return hipMemsetAsync(total, 0, sizeof(uint64_t), st);
    if (ev0) (void)hipEventRecord(ev0, st);
    if (approximate) range_scan<true><<<(unsigned)blocks, kBlock, 0, st>>>(x, y, n, a, bitmask, unit_count);
    else range_scan<false><<<(unsigned)blocks, kBlock, 0, st>>>(x, y, n, a, bitmask, unit_count);
    if (ev1) (void)hipEventRecord(ev1, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    scan_units<<<1, 1024, 0, st>>>(unit_count, units, offs, total);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    range_emit<<<(unsigned)blocks, kBlock, 0, st>>>(bitmask, offs, units, out, cap);
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
