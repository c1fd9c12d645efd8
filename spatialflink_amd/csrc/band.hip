// band.hip -- key-band owner partition of a window's points for the multi-GPU join.
//
// The device form of the reference's keyBy(gridID) shuffle (PointPointJoinQuery.java:137-150,
// JoinQuery.getReplicatedPointQueryStream keyed by the data point's gridID): rank s of W owns the
// x-major key band of grid columns [ceil(s nb / W), ceil((s+1) nb / W)), i.e. column cx belongs
// to rank cx * W / nb.  One launch pair packs the window's points grouped by owner, in arrival
// order inside each group, ready for one all-to-all: x, y and the point's window index.  Points
// whose key is not a valid cell of the nb x nb key space match no Nbr block (UniformGrid.java:
// 261-293) and are dropped, as the torch orchestration did.
//
//   band_count    per-block owner histogram (LDS atomics), block-major chunks of the window
//   band_scan     one block: exclusive scan over (owner, block) -> each block's base per owner,
//                 and the per-owner totals
//   band_scatter  per block, 256 points per step: ranks inside the wave by peeling owner groups
//                 (ballot), wave offsets through LDS, stable stores x / y / index
// HBM-bound: reads 16 B/point twice, writes 24 B per kept point.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string.h>

#include <string>

#include "device_common.h"
#include "geohip.h"
#include "join.h"

namespace geohip {
namespace {

constexpr int kBandTB = 256;
constexpr int kBandMaxBlocks = 1024;
constexpr int kBandMaxWorld = 64;

__device__ __forceinline__ int32_t band_d2i(double v) {
    if (v != v) return 0;
    if (v >= 2147483647.0) return INT32_MAX;
    if (v <= -2147483648.0) return INT32_MIN;
    return (int32_t)v;
}

struct BandArgs {
    const double* x;
    const double* y;
    uint64_t n, chunk;
    double mnx, mny, l;
    int32_t nb, world;
    Box u[kMaxPointBoxes + 1];  // nu > 0: only points of the query's G u C cells (planner boxes)
    int32_t nu;
    int32_t bw;                 // > 0: block-cyclic owners (column block cx / bw -> rank mod world)
};

// HelperClass.assignGridCellID (HelperClass.java:104-116) per axis, then the owner of the key's
// column -- its contiguous band (the join: a query's halo stays within few bands) or, for a single
// point query, its column block dealt round-robin (the reference's keyBy(gridID) hashes keys; one
// query's G u C box spans 2 Lc + 1 columns, which contiguous bands put on one rank); -1 when the
// key is not a cell of the key space (or, with a query filter, when the point lies in none of its
// guaranteed and candidate cells)
__device__ __forceinline__ int band_owner(const BandArgs& a, uint64_t i) {
    if (a.nu) {
        bool in = false;
        for (int b = 0; b < a.nu; b++) in = in || in_box(a.u[b], a.x[i], a.y[i]);
        if (!in) return -1;
    }
    const int32_t cx = band_d2i(__builtin_floor((a.x[i] - a.mnx) / a.l));
    const int32_t cy = band_d2i(__builtin_floor((a.y[i] - a.mny) / a.l));
    if (cx < 0 || cy < 0 || cx >= a.nb || cy >= a.nb) return -1;
    if (a.bw > 0) return (int)((cx / a.bw) % a.world);
    return (int)(((int64_t)cx * a.world) / a.nb);
}

__global__ __launch_bounds__(kBandTB) void band_count(BandArgs a, unsigned* __restrict__ hist) {
    __shared__ unsigned h[kBandMaxWorld];
    for (int t = threadIdx.x; t < a.world; t += kBandTB) h[t] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * a.chunk;
    const uint64_t hi = lo + a.chunk < a.n ? lo + a.chunk : a.n;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += kBandTB) {
        const int o = band_owner(a, i);
        if (o >= 0) atomicAdd(&h[o], 1u);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < a.world; t += kBandTB) hist[(size_t)t * gridDim.x + blockIdx.x] = h[t];
}

// exclusive scan of hist[world * nblk] (owner-major) into off; counts[o] = owner o's total
__global__ __launch_bounds__(1024) void band_scan(const unsigned* __restrict__ hist, uint32_t m, uint32_t nblk,
                                                  int world, unsigned long long* __restrict__ off,
                                                  unsigned long long* __restrict__ counts) {
    __shared__ unsigned long long part[1024];
    const uint32_t per = (m + 1023) / 1024;
    const uint32_t b0 = threadIdx.x * per, b1 = b0 + per < m ? b0 + per : m;
    unsigned long long s = 0;
    for (uint32_t i = b0; i < b1; i++) s += hist[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele over the 1024 partials
        const unsigned long long v = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0ull;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    unsigned long long run = threadIdx.x ? part[threadIdx.x - 1] : 0ull;
    for (uint32_t i = b0; i < b1; i++) {
        off[i] = run;
        run += hist[i];
    }
    __syncthreads();
    if ((int)threadIdx.x < world) {
        const uint32_t o = threadIdx.x;
        const unsigned long long a = off[(size_t)o * nblk];
        const unsigned long long b = o + 1 < (uint32_t)world ? off[(size_t)(o + 1) * nblk] : part[1023];
        counts[o] = b - a;
    }
}

__global__ __launch_bounds__(kBandTB) void band_scatter(BandArgs a, const unsigned long long* __restrict__ off,
                                                        int64_t base, double* __restrict__ ox,
                                                        double* __restrict__ oy, int64_t* __restrict__ oidx) {
    __shared__ unsigned long long cursor[kBandMaxWorld];
    __shared__ unsigned wcnt[kBandTB / kWave][kBandMaxWorld];
    const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    for (int t = threadIdx.x; t < a.world; t += kBandTB) cursor[t] = off[(size_t)t * gridDim.x + blockIdx.x];
    const uint64_t lo = (uint64_t)blockIdx.x * a.chunk;
    const uint64_t hi = lo + a.chunk < a.n ? lo + a.chunk : a.n;
    for (uint64_t s = lo; s < hi; s += kBandTB) {
        for (int t = threadIdx.x; t < (kBandTB / kWave) * a.world; t += kBandTB) (&wcnt[0][0])[t / a.world * kBandMaxWorld + t % a.world] = 0;
        __syncthreads();
        const uint64_t i = s + threadIdx.x;
        const int o = i < hi ? band_owner(a, i) : -1;
        // rank among the wave's lanes of the same owner: peel one owner group per step
        unsigned rank = 0;
        unsigned long long left = __ballot(o >= 0);
        while (left) {
            const int first = __builtin_ctzll(left);
            const int og = __shfl(o, first);
            const unsigned long long grp = __ballot(o == og);
            if (o == og) rank = (unsigned)__popcll(grp & ((1ull << lane) - 1ull));
            if (lane == first) wcnt[wid][og] = (unsigned)__popcll(grp);
            left &= ~grp;
        }
        __syncthreads();
        if (o >= 0) {
            unsigned long long p = cursor[o] + rank;
            for (int w = 0; w < wid; w++) p += wcnt[w][o];
            ox[p] = a.x[i];
            oy[p] = a.y[i];
            oidx[p] = base + (int64_t)i;
        }
        __syncthreads();
        for (int t = threadIdx.x; t < a.world; t += kBandTB) {
            unsigned long long add = 0;
            for (int w = 0; w < kBandTB / kWave; w++) add += wcnt[w][t];
            cursor[t] += add;
        }
        __syncthreads();
    }
}

}  // namespace

// Column block width of the single-query layout: at least 8 blocks per rank across the query's
// 2 Lc + 1 candidate columns (C5, Lc = 24: width 1 at 2..8 ranks), so each rank's share of the box
// is within one block of the mean.
int32_t query_block_width(int32_t layers_c, uint32_t world) {
    const int64_t cols = 2 * (int64_t)(layers_c > 0 ? layers_c : 0) + 1;
    const int64_t w = cols / (8 * (int64_t)world);
    return (int32_t)(w > 1 ? (w < (1 << 20) ? w : (1 << 20)) : 1);
}

int band_pack_impl(geohip_ctx* ctx, const geohip_grid* grid, int32_t nb, uint32_t world, const double* x,
                   const double* y, uint64_t n, int64_t base, double* out_x, double* out_y, int64_t* out_idx,
                   uint64_t* out_counts, const PointPlan* filter) {
    if (!grid || !out_counts) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null grid / out_counts");
    if (ctx_mem(ctx) != GEOHIP_MEM_DEVICE) return ctx_fail(ctx, GEOHIP_ERR_ARG, "band_pack_async needs GEOHIP_MEM_DEVICE");
    if (world == 0 || world > (uint32_t)kBandMaxWorld)
        return ctx_fail(ctx, world ? GEOHIP_ERR_UNSUPPORTED : GEOHIP_ERR_ARG, "world must be 1..64");
    if (nb <= 0) return ctx_fail(ctx, GEOHIP_ERR_ARG, "nb must be > 0");
    if (!(grid->cell_len > 0.0)) return ctx_fail(ctx, GEOHIP_ERR_ARG, "cell_len must be > 0");
    if (n && (!x || !y || !out_x || !out_y || !out_idx)) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null arrays");
    hipStream_t st = ctx_stream(ctx);
    if (n == 0) {
        if (hipMemsetAsync(out_counts, 0, 8 * (size_t)world, st) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
        return GEOHIP_OK;
    }
    const uint64_t want_blocks = (n + 16ull * kBandTB - 1) / (16ull * kBandTB);
    const uint32_t nblk = (uint32_t)(want_blocks < (uint64_t)kBandMaxBlocks ? want_blocks : kBandMaxBlocks);
    BandArgs a;
    memset(&a, 0, sizeof a);
    a.x = x;
    a.y = y;
    a.n = n;
    a.chunk = (n + nblk - 1) / nblk;
    a.mnx = grid->min_x;
    a.mny = grid->min_y;
    a.l = grid->cell_len;
    a.nb = nb;
    a.world = (int32_t)world;
    if (filter) {
        for (int b = 0; b < filter->nu; b++) a.u[b] = filter->u[b];
        a.nu = filter->nu;
        a.bw = query_block_width(filter->layers_c, world);
        if (a.nu == 0) {  // no candidate cell at all (r <= 0): nothing to send
            if (hipMemsetAsync(out_counts, 0, 8 * (size_t)world, st) != hipSuccess)
                return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
            return GEOHIP_OK;
        }
    }
    const uint32_t m = world * nblk;
    void* ph = nullptr;
    void* po = nullptr;
    int rc = ctx_ensure(ctx, 0, 4 * (size_t)m, &ph);
    if (!rc) rc = ctx_ensure(ctx, 1, 8 * (size_t)m, &po);
    if (rc) return rc;
    unsigned* hist = reinterpret_cast<unsigned*>(ph);
    unsigned long long* off = reinterpret_cast<unsigned long long*>(po);
    band_count<<<nblk, kBandTB, 0, st>>>(a, hist);
    band_scan<<<1, 1024, 0, st>>>(hist, m, nblk, (int)world, off, reinterpret_cast<unsigned long long*>(out_counts));
    band_scatter<<<nblk, kBandTB, 0, st>>>(a, off, base, out_x, out_y, out_idx);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("band_pack launch: ") + hipGetErrorString(e));
    return GEOHIP_OK;
}

}  // namespace geohip
