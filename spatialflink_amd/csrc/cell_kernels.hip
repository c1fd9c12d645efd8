// cell_kernels.hip -- cell-bucketed kernels of libgeohip for gfx950: point-point window join
// (PointPointJoinQuery.java:113-172 + JoinQuery.java:73-90) and point-polygon window range
// (PointPolygonRangeQuery.java:76-124).
//
// Both bucket the window's points by grid cell with a counting sort (per-cell histogram by
// atomics, exclusive scan, scatter into SoA x/y/idx/cell), so a query reads only the
// contiguous point ranges of its cell columns (x-major keys: one column of a cell rectangle
// is one contiguous range).  One workgroup per query walks the concatenated ranges in
// 256-point tiles, computes the exact JTS distance (fdlibm hypot / point-polygon), compacts
// hits into an LDS pair buffer and flushes it with one global atomic per 8K pairs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "device_common.h"
#include "join.h"
#include "ppoly.h"

namespace geohip {

constexpr int kTB = 256;           // threads per block
constexpr int kPairBuf = 8192;     // LDS pair buffer (64 KB)
constexpr unsigned kNoCell = 0xffffffffu;

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

// ------------------------------------------------------------------ bucketing -------------
// key = cx * nb + cy for 0 <= cx, cy < nb, else kNoCell.
__global__ void bucket_count(const double* __restrict__ x, const double* __restrict__ y, uint64_t n, double mnx,
                             double mny, double l, int32_t nb, unsigned* __restrict__ key,
                             unsigned* __restrict__ count, unsigned* __restrict__ outside) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t cx = d_axis_cell(x[i], mnx, l);
        const int32_t cy = d_axis_cell(y[i], mny, l);
        unsigned k = kNoCell;
        if (cx >= 0 && cy >= 0 && cx < nb && cy < nb) {
            k = (unsigned)cx * (unsigned)nb + (unsigned)cy;
            atomicAdd(&count[k], 1u);
        } else {
            atomicAdd(outside, 1u);
        }
        key[i] = k;
    }
}

// exclusive scan, 3 phases: per-block totals, scan of totals, per-block rescan + offset
constexpr int kScanPer = 16;
constexpr int kScanSeg = kTB * kScanPer;

__device__ __forceinline__ unsigned block_excl_scan(unsigned v, unsigned* sh, unsigned* total) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < kTB; o <<= 1) {
        unsigned a = t >= o ? sh[t - o] : 0u;
        __syncthreads();
        sh[t] += a;
        __syncthreads();
    }
    const unsigned incl = sh[t];
    *total = sh[kTB - 1];
    __syncthreads();
    return incl - v;
}

__global__ void scan_seg_totals(const unsigned* __restrict__ in, uint64_t n, unsigned* __restrict__ seg_tot) {
    __shared__ unsigned sh[kTB];
    const uint64_t base = (uint64_t)blockIdx.x * kScanSeg + (uint64_t)threadIdx.x * kScanPer;
    unsigned s = 0;
    for (int j = 0; j < kScanPer; j++)
        if (base + j < n) s += in[base + j];
    unsigned tot;
    block_excl_scan(s, sh, &tot);
    if (threadIdx.x == 0) seg_tot[blockIdx.x] = tot;
}

__global__ void scan_totals(unsigned* __restrict__ seg_tot, uint64_t nseg, unsigned* __restrict__ grand) {
    __shared__ unsigned sh[kTB];
    unsigned carry = 0;
    for (uint64_t b = 0; b < nseg; b += kTB) {
        const uint64_t i = b + threadIdx.x;
        const unsigned v = i < nseg ? seg_tot[i] : 0u;
        unsigned tot;
        const unsigned ex = block_excl_scan(v, sh, &tot);
        if (i < nseg) seg_tot[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *grand = carry;
}

// out[i] = sum(in[0..i)); out[n] = total
__global__ void scan_apply(const unsigned* __restrict__ in, uint64_t n, const unsigned* __restrict__ seg_off,
                           const unsigned* __restrict__ grand, unsigned* __restrict__ out) {
    __shared__ unsigned sh[kTB];
    const uint64_t base = (uint64_t)blockIdx.x * kScanSeg + (uint64_t)threadIdx.x * kScanPer;
    unsigned v[kScanPer];
    unsigned s = 0;
    for (int j = 0; j < kScanPer; j++) {
        v[j] = base + j < n ? in[base + j] : 0u;
        s += v[j];
    }
    unsigned tot;
    unsigned run = seg_off[blockIdx.x] + block_excl_scan(s, sh, &tot);
    for (int j = 0; j < kScanPer; j++) {
        if (base + j < n) out[base + j] = run;
        run += v[j];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = *grand;
}

__global__ void bucket_scatter(const double* __restrict__ x, const double* __restrict__ y, uint64_t n,
                               const unsigned* __restrict__ key, const unsigned* __restrict__ start,
                               unsigned* __restrict__ cursor, double* __restrict__ sx, double* __restrict__ sy,
                               unsigned* __restrict__ sidx, unsigned* __restrict__ skey,
                               unsigned* __restrict__ outside_idx, unsigned* __restrict__ outside_cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned k = key[i];
        if (k != kNoCell) {
            const unsigned pos = start[k] + atomicAdd(&cursor[k], 1u);
            sx[pos] = x[i];
            sy[pos] = y[i];
            sidx[pos] = (unsigned)i;
            if (skey) skey[pos] = k;
        } else if (outside_idx) {
            outside_idx[atomicAdd(outside_cnt, 1u)] = (unsigned)i;
        }
    }
}

struct Bucketed {
    const double* sx;
    const double* sy;
    const unsigned* sidx;
    const unsigned* skey;
    const unsigned* start;  // nb*nb + 1
    const unsigned* outside_idx;
    unsigned n_outside;
    int32_t nb;
};

// ------------------------------------------------------------------ pair buffer ----------
struct PairBuf {
    unsigned a[kPairBuf];
    unsigned b[kPairBuf];
    unsigned cnt;
    unsigned long long base;
};

__device__ __forceinline__ void pairbuf_push(PairBuf& pb, bool hit, unsigned a, unsigned b) {
    const unsigned long long m = __ballot(hit);
    unsigned wbase = 0;
    if (lane_id() == 0 && m) wbase = atomicAdd(&pb.cnt, (unsigned)__popcll(m));
    wbase = __shfl(wbase, 0);
    if (hit) {
        const unsigned pos = wbase + lanes_below(m);
        pb.a[pos] = a;
        pb.b[pos] = b;
    }
}

// all threads: write the buffer to out at a globally reserved offset, reset it
__device__ __forceinline__ void pairbuf_flush(PairBuf& pb, unsigned long long* total, unsigned* out, uint64_t cap) {
    __syncthreads();
    const unsigned c = pb.cnt;
    if (c) {
        if (threadIdx.x == 0) pb.base = atomicAdd(total, (unsigned long long)c);
        __syncthreads();
        const unsigned long long base = pb.base;
        if (out) {
            for (unsigned t = threadIdx.x; t < c; t += blockDim.x) {
                const unsigned long long p = base + t;
                if (p < cap) {
                    out[2 * p] = pb.a[t];
                    out[2 * p + 1] = pb.b[t];
                }
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) pb.cnt = 0;
    }
    __syncthreads();
}

// Walk the concatenated point ranges of columns x0..x1 (rows y0..y1) of one query in
// 256-point tiles: fn(sorted position) on every point, then tile_end() (block-uniform).
struct ColWalk {
    unsigned colpref[kTB + 1];
    unsigned colbeg[kTB];
};

template <typename F, typename E>
__device__ __forceinline__ void walk_columns(ColWalk& cw, const unsigned* __restrict__ start, int32_t nb, int32_t x0,
                                             int32_t x1, int32_t y0, int32_t y1, F fn, E tile_end) {
    for (int32_t cb = x0; cb <= x1; cb += kTB) {
        const int32_t ncol = min(kTB, x1 - cb + 1);
        unsigned len = 0, beg = 0;
        if ((int)threadIdx.x < ncol) {
            const uint64_t c = (uint64_t)(cb + threadIdx.x) * (uint64_t)nb;
            beg = start[c + y0];
            len = start[c + y1 + 1] - beg;
        }
        __shared__ unsigned scan_sh[kTB];
        unsigned tot;
        const unsigned ex = block_excl_scan(len, scan_sh, &tot);
        if ((int)threadIdx.x < ncol) {
            cw.colpref[threadIdx.x] = ex;
            cw.colbeg[threadIdx.x] = beg;
        }
        if (threadIdx.x == 0) cw.colpref[ncol] = tot;
        __syncthreads();
        for (unsigned t0 = 0; t0 < tot; t0 += kTB) {
            const unsigned v = t0 + threadIdx.x;
            if (v < tot) {
                int lo = 0, hi = ncol - 1;  // last column with colpref <= v
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (cw.colpref[mid] <= v) lo = mid; else hi = mid - 1;
                }
                fn(cw.colbeg[lo] + (v - cw.colpref[lo]));
            } else {
                fn(0xffffffffu);
            }
            tile_end();
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ join -----------------
struct QRect {
    int32_t x0, x1, y0, y1;  // bucket space, clipped; x0 > x1 = empty
};

template <bool COUNT_ONLY, bool APPROX>
__global__ __launch_bounds__(kTB) void join_probe(Bucketed bk, const double* __restrict__ qx,
                                                  const double* __restrict__ qy, const QRect* __restrict__ rect,
                                                  uint64_t nq, double r, unsigned long long* __restrict__ total,
                                                  unsigned* __restrict__ out, uint64_t cap) {
    __shared__ PairBuf pb;
    __shared__ ColWalk cw;
    __shared__ unsigned long long bcount;
    if (threadIdx.x == 0) { pb.cnt = 0; bcount = 0; }
    __syncthreads();
    for (uint64_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const QRect R = rect[q];
        if (R.x0 > R.x1 || R.y0 > R.y1) continue;
        const double px = qx[q], py = qy[q];
        unsigned my = 0;
        walk_columns(
            cw, bk.start, bk.nb, R.x0, R.x1, R.y0, R.y1,
            [&](unsigned pos) {
                bool hit = false;
                unsigned pid = 0;
                if (pos != 0xffffffffu) {
                    const double dx = bk.sx[pos], dy = bk.sy[pos];
                    pid = bk.sidx[pos];
                    // getDistance(p, q): p.point.distance(q.point)
                    hit = APPROX || jts_pp_distance(dx, dy, px, py) <= r;
                }
                if (COUNT_ONLY) my += hit ? 1u : 0u;
                else pairbuf_push(pb, hit, pid, (unsigned)q);
            },
            [&]() {
                if (!COUNT_ONLY) {
                    __syncthreads();
                    if (pb.cnt > kPairBuf - kTB) pairbuf_flush(pb, total, out, cap);
                }
            });
        if (COUNT_ONLY && my) atomicAdd(&bcount, (unsigned long long)my);
    }
    if (COUNT_ONLY) {
        __syncthreads();
        if (threadIdx.x == 0 && bcount) atomicAdd(total, bcount);
    } else {
        pairbuf_flush(pb, total, out, cap);
    }
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
    uint32_t pad;
};

// JTS DistanceOp(point, polygon) predicate "distance <= r" (r < MAX_VALUE):
// PointLocator (envelope, RayCrossingCounter) -> 0; else min over segments of
// Distance.pointToSegment.  Boolean-equivalent early exits.
__device__ bool point_polygon_within(double px, double py, const double* __restrict__ vx,
                                     const double* __restrict__ vy, int nv, const double bb[4], double r) {
    const bool in_env = !(px > bb[2] || px < bb[0] || py > bb[3] || py < bb[1]);
    if (in_env) {
        int crossings = 0;
        bool boundary = false;
        for (int i = 1; i < nv; i++) {
            const double p1x = vx[i], p1y = vy[i], p2x = vx[i - 1], p2y = vy[i - 1];
            if (p1x < px && p2x < px) continue;
            if (px == p2x && py == p2y) { boundary = true; break; }
            if (p1y == py && p2y == py) {
                double mn = p1x, mx = p2x;
                if (mn > mx) { mn = p2x; mx = p1x; }
                if (px >= mn && px <= mx) { boundary = true; break; }
                continue;
            }
            if ((p1y > py && p2y <= py) || (p2y > py && p1y <= py)) {
                const double x1 = p1x - px, y1 = p1y - py, x2 = p2x - px, y2 = p2y - py;
                int s = exact_det_sign(x1, y1, x2, y2);
                if (s == 0) { boundary = true; break; }
                if (y2 < y1) s = -s;
                if (s > 0) crossings++;
            }
        }
        if (boundary || (crossings & 1)) return true;  // not EXTERIOR: distance 0
    }
    for (int i = 0; i < nv - 1; i++) {
        const double ax = vx[i], ay = vy[i], bx = vx[i + 1], by = vy[i + 1];
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
        if (d <= r) return true;
    }
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

constexpr int kMaxLdsVerts = 2048;

template <bool COUNT_ONLY, bool APPROX>
__global__ __launch_bounds__(kTB) void ppoly_probe(Bucketed bk, const PolyDev* __restrict__ polys, uint32_t npoly,
                                                   const double* __restrict__ vx, const double* __restrict__ vy,
                                                   const int32_t* __restrict__ rects, double r, int r_is_max,
                                                   unsigned long long* __restrict__ total, unsigned* __restrict__ out,
                                                   uint64_t cap) {
    __shared__ PairBuf pb;
    __shared__ ColWalk cw;
    __shared__ double lvx[kMaxLdsVerts];
    __shared__ double lvy[kMaxLdsVerts];
    __shared__ unsigned long long bcount;
    if (threadIdx.x == 0) { pb.cnt = 0; bcount = 0; }
    __syncthreads();
    for (uint32_t p = blockIdx.x; p < npoly; p += gridDim.x) {
        const PolyDev P = polys[p];
        if (P.wx0 > P.wx1 || P.wy0 > P.wy1) continue;
        const bool in_lds = P.nv <= (uint32_t)kMaxLdsVerts;
        __syncthreads();
        if (in_lds)
            for (uint32_t t = threadIdx.x; t < P.nv; t += blockDim.x) {
                lvx[t] = vx[P.voff + t];
                lvy[t] = vy[P.voff + t];
            }
        __syncthreads();
        const double* rvx = in_lds ? lvx : vx + P.voff;
        const double* rvy = in_lds ? lvy : vy + P.voff;
        unsigned my = 0;
        walk_columns(
            cw, bk.start, bk.nb, P.wx0, P.wx1, P.wy0, P.wy1,
            [&](unsigned pos) {
                bool hit = false;
                unsigned pid = 0;
                if (pos != 0xffffffffu) {
                    const unsigned key = bk.skey[pos];
                    const int32_t cx = (int32_t)(key / (unsigned)bk.nb), cy = (int32_t)(key % (unsigned)bk.nb);
                    const bool g = in_rects(rects + 4 * P.goff, P.ng, cx, cy);
                    const bool c = !g && in_rects(rects + 4 * P.coff, P.nc, cx, cy);
                    if (g || c) {
                        pid = bk.sidx[pos];
                        if (g || r_is_max) {
                            hit = true;
                        } else {
                            const double px = bk.sx[pos], py = bk.sy[pos];
                            if (APPROX) hit = bbox_distance(px, py, P.bb) <= r;
                            else hit = point_polygon_within(px, py, rvx, rvy, (int)P.nv, P.bb, r);
                        }
                    }
                }
                if (COUNT_ONLY) my += hit ? 1u : 0u;
                else pairbuf_push(pb, hit, p, pid);
            },
            [&]() {
                if (!COUNT_ONLY) {
                    __syncthreads();
                    if (pb.cnt > kPairBuf - kTB) pairbuf_flush(pb, total, out, cap);
                }
            });
        if (COUNT_ONLY && my) atomicAdd(&bcount, (unsigned long long)my);
    }
    if (COUNT_ONLY) {
        __syncthreads();
        if (threadIdx.x == 0 && bcount) atomicAdd(total, bcount);
    } else {
        pairbuf_flush(pb, total, out, cap);
    }
}

// out-of-grid points vs guaranteed rects reaching outside the grid (Lg == 0 bbox keys)
template <bool COUNT_ONLY>
__global__ __launch_bounds__(kTB) void ppoly_outside(const double* __restrict__ x, const double* __restrict__ y,
                                                     const unsigned* __restrict__ oidx, unsigned nout, double mnx,
                                                     double mny, double l, const PolyDev* __restrict__ polys,
                                                     uint32_t npoly, const int32_t* __restrict__ rects,
                                                     unsigned long long* __restrict__ total, unsigned* __restrict__ out,
                                                     uint64_t cap) {
    __shared__ PairBuf pb;
    __shared__ unsigned long long bcount;
    if (threadIdx.x == 0) { pb.cnt = 0; bcount = 0; }
    __syncthreads();
    for (uint32_t p = blockIdx.x; p < npoly; p += gridDim.x) {
        const PolyDev P = polys[p];
        if (!P.outside) continue;
        unsigned my = 0;
        for (unsigned t0 = 0; t0 < nout; t0 += kTB) {
            const unsigned t = t0 + threadIdx.x;
            bool hit = false;
            unsigned pid = 0;
            if (t < nout) {
                pid = oidx[t];
                const int32_t cx = d_axis_cell(x[pid], mnx, l), cy = d_axis_cell(y[pid], mny, l);
                hit = in_rects(rects + 4 * P.goff, P.ng, cx, cy);
            }
            if (COUNT_ONLY) {
                my += hit ? 1u : 0u;
            } else {
                pairbuf_push(pb, hit, p, pid);
                __syncthreads();
                if (pb.cnt > kPairBuf - kTB) pairbuf_flush(pb, total, out, cap);
            }
        }
        if (COUNT_ONLY && my) atomicAdd(&bcount, (unsigned long long)my);
    }
    if (COUNT_ONLY) {
        __syncthreads();
        if (threadIdx.x == 0 && bcount) atomicAdd(total, bcount);
    } else {
        pairbuf_flush(pb, total, out, cap);
    }
}

// ================================================================== host side =============
namespace {

enum JSlot { J_KEY, J_COUNT, J_START, J_SEG, J_SX, J_SY, J_SIDX, J_SKEY, J_MISC, J_AUX, J_POLY, J_OUT, J_RECT };

struct Scratch {
    geohip_ctx* ctx;
    int rc = GEOHIP_OK;
    template <typename T>
    T* get(int slot, size_t bytes) {
        void* p = nullptr;
        if (rc) return nullptr;
        rc = ctx_ensure(ctx, slot, bytes, &p);
        return reinterpret_cast<T*>(p);
    }
};

unsigned grid_blocks(uint64_t n) {
    uint64_t b = (n + kTB - 1) / kTB;
    if (b > 8192) b = 8192;
    if (b == 0) b = 1;
    return (unsigned)b;
}

int check_grid_basic(geohip_ctx* ctx, const geohip_grid* g, const char* what) {
    if (!g) return ctx_fail(ctx, GEOHIP_ERR_ARG, std::string(what) + ": null grid");
    if (!(g->n > 0) || !(g->cell_len > 0) || !std::isfinite(g->cell_len) || !std::isfinite(g->min_x) ||
        !std::isfinite(g->min_y))
        return ctx_fail(ctx, GEOHIP_ERR_ARG, std::string(what) + ": invalid grid");
    if (g->n > 99999) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, std::string(what) + ": more than 99999 cells per side");
    return GEOHIP_OK;
}

// Counting sort of the points by cell of `g` over [0, nb)^2.
int bucketize(geohip_ctx* ctx, Scratch& S, const double* dx, const double* dy, uint64_t n, const geohip_grid& g,
              int32_t nb, bool keep_keys, bool keep_outside, Bucketed* bk, unsigned* n_outside_host) {
    hipStream_t st = ctx_stream(ctx);
    const uint64_t ncell = (uint64_t)nb * (uint64_t)nb;
    if (ncell > (1ull << 27)) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "grid too large for cell bucketing (> 2^27 cells)");
    unsigned* key = S.get<unsigned>(J_KEY, n * 4);
    unsigned* count = S.get<unsigned>(J_COUNT, (ncell + 1) * 4);
    unsigned* start = S.get<unsigned>(J_START, (ncell + 1) * 4);
    const uint64_t nseg = (ncell + kScanSeg - 1) / kScanSeg;
    unsigned* seg = S.get<unsigned>(J_SEG, (nseg + 1) * 4 + 64);
    double* sx = S.get<double>(J_SX, n * 8);
    double* sy = S.get<double>(J_SY, n * 8);
    unsigned* sidx = S.get<unsigned>(J_SIDX, n * 4);
    unsigned* skey = keep_keys ? S.get<unsigned>(J_SKEY, n * 4) : nullptr;
    unsigned* misc = S.get<unsigned>(J_MISC, 64);
    unsigned* oidx = keep_outside ? S.get<unsigned>(J_AUX, n * 4 + 16) : nullptr;
    if (S.rc) return S.rc;
    // misc[0] = outside count (histogram), misc[1] = outside cursor, misc[2] = grand total
    if (hipMemsetAsync(count, 0, (ncell + 1) * 4, st) != hipSuccess || hipMemsetAsync(misc, 0, 64, st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    if (n) bucket_count<<<grid_blocks(n), kTB, 0, st>>>(dx, dy, n, g.min_x, g.min_y, g.cell_len, nb, key, count, misc);
    scan_seg_totals<<<(unsigned)nseg, kTB, 0, st>>>(count, ncell, seg);
    scan_totals<<<1, kTB, 0, st>>>(seg, nseg, misc + 2);
    scan_apply<<<(unsigned)nseg, kTB, 0, st>>>(count, ncell, seg, misc + 2, start);
    if (hipMemsetAsync(count, 0, ncell * 4, st) != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    if (n)
        bucket_scatter<<<grid_blocks(n), kTB, 0, st>>>(dx, dy, n, key, start, count, sx, sy, sidx, skey, oidx, misc + 1);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("bucketing: ") + hipGetErrorString(e));
    if (n_outside_host) {
        uint64_t* pin = ctx_pinned(ctx);
        if (hipMemcpyAsync(pin, misc, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "outside count readback failed");
        *n_outside_host = (unsigned)(pin[0] & 0xffffffffu);
    }
    bk->sx = sx;
    bk->sy = sy;
    bk->sidx = sidx;
    bk->skey = skey;
    bk->start = start;
    bk->outside_idx = oidx;
    bk->n_outside = n_outside_host ? *n_outside_host : 0;
    bk->nb = nb;
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

}  // namespace

int join_pp_impl(geohip_ctx* ctx, const geohip_grid* gd, const geohip_grid* gq, const double* dx, const double* dy,
                 uint64_t nd, const double* qx, const double* qy, uint64_t nq, double r, int approximate,
                 uint32_t* out_pairs, uint64_t cap, uint64_t* out_count, bool count_only) {
    if (!out_count) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out_count");
    *out_count = 0;
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
    // plan the replicated query blocks on the host (HelperClass.getIntCellIndices semantics)
    std::vector<double> hqx, hqy;
    const double* pqx = qx;
    const double* pqy = qy;
    if (dev && nq) {
        hqx.resize(nq);
        hqy.resize(nq);
        if (hipMemcpy(hqx.data(), qx, nq * 8, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(hqy.data(), qy, nq * 8, hipMemcpyDeviceToHost) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "query readback failed");
        pqx = hqx.data();
        pqy = hqy.data();
    }
    const int32_t nb = gq->n;
    std::vector<QRect> rects(nq);
    for (uint64_t i = 0; i < nq; i++) {
        QRect R{0, nb - 1, 0, nb - 1};
        if (!all_cells) {
            int32_t cx, cy, ci, cj;
            cell_of(*gq, pqx[i], pqy[i], &cx, &cy);
            if (cx >= -9999 && cx <= 99999 && cy >= -9999 && cy <= 99999) { ci = cx; cj = cy; }
            else if (!key_roundtrip(cx, cy, &ci, &cj))
                return ctx_fail(ctx, GEOHIP_ERR_ARG, "NumberFormatException in getIntCellIndices (query point key)");
            const int64_t a0 = (int64_t)ci - lc, a1 = (int64_t)ci + lc, b0 = (int64_t)cj - lc, b1 = (int64_t)cj + lc;
            const int32_t lo_i = (int32_t)(uint32_t)(uint64_t)a0, hi_i = (int32_t)(uint32_t)(uint64_t)a1;
            const int32_t lo_j = (int32_t)(uint32_t)(uint64_t)b0, hi_j = (int32_t)(uint32_t)(uint64_t)b1;
            if (lo_i > hi_i || lo_j > hi_j) {
                R = QRect{1, 0, 1, 0};
            } else {
                if (hi_i == INT32_MAX || hi_j == INT32_MAX)
                    return ctx_fail(ctx, GEOHIP_ERR_ARG, "reference neighbour loop does not terminate");
                R = QRect{std::max(lo_i, 0), std::min(hi_i, nb - 1), std::max(lo_j, 0), std::min(hi_j, nb - 1)};
            }
        }
        rects[i] = R;
    }
    Scratch S{ctx};
    const double *ddx, *ddy, *dqx, *dqy;
    rc = ctx_stage_xy(ctx, dx, dy, nd, 0, &ddx, &ddy);
    if (!rc) rc = ctx_stage_xy(ctx, qx, qy, nq, 1, &dqx, &dqy);
    if (rc) return rc;
    Bucketed bk;
    rc = bucketize(ctx, S, ddx, ddy, nd, *gd, nb, false, false, &bk, nullptr);
    if (rc) return rc;
    QRect* drect = S.get<QRect>(J_RECT, nq * sizeof(QRect) + 16);
    if (S.rc) return S.rc;
    // total counter lives after the bucketing words in J_MISC
    unsigned long long* total = nullptr;
    {
        void* p = nullptr;
        rc = ctx_ensure(ctx, J_MISC, 64, &p);
        if (rc) return rc;
        total = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(p) + 32);
    }
    if (nq && hipMemcpyAsync(drect, rects.data(), nq * sizeof(QRect), hipMemcpyHostToDevice, st) != hipSuccess)
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "rect upload failed");
    if (hipMemsetAsync(total, 0, 8, st) != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
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
    hipEvent_t e0, e1;
    ctx_timing_events(ctx, &e0, &e1);
    if (e0) hipEventRecord(e0, st);
    const unsigned blocks = (unsigned)std::min<uint64_t>(nq ? nq : 1, 1u << 20);
    if (nq) {
        if (count_only || !cap) {
            if (approximate) join_probe<true, true><<<blocks, kTB, 0, st>>>(bk, dqx, dqy, drect, nq, r, total, nullptr, 0);
            else join_probe<true, false><<<blocks, kTB, 0, st>>>(bk, dqx, dqy, drect, nq, r, total, nullptr, 0);
        } else {
            if (approximate) join_probe<false, true><<<blocks, kTB, 0, st>>>(bk, dqx, dqy, drect, nq, r, total, out, cap);
            else join_probe<false, false><<<blocks, kTB, 0, st>>>(bk, dqx, dqy, drect, nq, r, total, out, cap);
        }
    }
    if (e1) hipEventRecord(e1, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("join launch: ") + hipGetErrorString(e));
    uint64_t tot = 0;
    rc = read_total(ctx, total, &tot);
    if (rc) return rc;
    *out_count = tot;
    if (!count_only && !dev && cap) {
        const uint64_t m = std::min<uint64_t>(tot, cap);
        if (m && hipMemcpy(out_pairs, out, m * 8, hipMemcpyDeviceToHost) != hipSuccess)
            return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "pair readback failed");
    }
    if (!count_only && tot > cap) return ctx_fail(ctx, GEOHIP_ERR_CAPACITY, "output capacity too small; *out_count = required");
    return GEOHIP_OK;
}

int ppoly_impl(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
               const uint32_t* ring_off, const double* vx, const double* vy, uint32_t npoly, double r, int approximate,
               uint32_t* out_pairs, uint64_t cap, uint64_t* out_count) {
    if (!out_count) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out_count");
    *out_count = 0;
    int rc = check_grid_basic(ctx, grid, "grid");
    if (rc) return rc;
    if (n >= 0xffffffffull) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "window larger than 2^32-1 points");
    if (npoly && (!ring_off || !vx || !vy)) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null polygon arrays");
    if (cap && !out_pairs) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out_pairs");
    hipStream_t st = ctx_stream(ctx);
    const bool dev = ctx_mem(ctx) == GEOHIP_MEM_DEVICE;
    const int32_t nb = grid->n;
    // polygon planning (host): ring closure, envelope, G / C rectangles (plan.cpp)
    std::vector<PolyDev> pd(npoly);
    std::vector<double> hvx, hvy;
    std::vector<int32_t> hrects;
    bool any_outside = false;
    for (uint32_t p = 0; p < npoly; p++) {
        PolyPlan pl;
        std::string err;
        const uint32_t b = ring_off[p], e = ring_off[p + 1];
        if (e < b) return ctx_fail(ctx, GEOHIP_ERR_ARG, "ring_off not ascending");
        rc = plan_polygon(*grid, vx + b, vy + b, e - b, r, &pl, &err);
        if (rc) return ctx_fail(ctx, rc, err);
        PolyDev& P = pd[p];
        memset(&P, 0, sizeof P);
        P.voff = (uint32_t)hvx.size();
        P.nv = (uint32_t)pl.rx.size();
        hvx.insert(hvx.end(), pl.rx.begin(), pl.rx.end());
        hvy.insert(hvy.end(), pl.ry.begin(), pl.ry.end());
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
    }
    Scratch S{ctx};
    const double *dx, *dy;
    rc = ctx_stage_xy(ctx, x, y, n, 0, &dx, &dy);
    if (rc) return rc;
    Bucketed bk;
    unsigned n_out = 0;
    rc = bucketize(ctx, S, dx, dy, n, *grid, nb, true, any_outside, &bk, any_outside ? &n_out : nullptr);
    if (rc) return rc;
    // polygon tables in one device blob: PolyDev[] | vx | vy | rects
    const size_t sz_p = npoly * sizeof(PolyDev), sz_v = hvx.size() * 8, sz_r = hrects.size() * 4;
    void* pblob = nullptr;
    rc = ctx_ensure(ctx, J_POLY, sz_p + 2 * sz_v + sz_r + 64, &pblob);
    if (rc) return rc;
    char* bp = reinterpret_cast<char*>(pblob);
    PolyDev* dpoly = reinterpret_cast<PolyDev*>(bp);
    double* dvx = reinterpret_cast<double*>(bp + ((sz_p + 15) & ~(size_t)15));
    double* dvy = dvx + hvx.size();
    int32_t* drects = reinterpret_cast<int32_t*>(dvy + hvy.size());
    if ((sz_p && hipMemcpyAsync(dpoly, pd.data(), sz_p, hipMemcpyHostToDevice, st) != hipSuccess) ||
        (sz_v && hipMemcpyAsync(dvx, hvx.data(), sz_v, hipMemcpyHostToDevice, st) != hipSuccess) ||
        (sz_v && hipMemcpyAsync(dvy, hvy.data(), sz_v, hipMemcpyHostToDevice, st) != hipSuccess) ||
        (sz_r && hipMemcpyAsync(drects, hrects.data(), sz_r, hipMemcpyHostToDevice, st) != hipSuccess))
        return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "polygon upload failed");
    unsigned long long* total = nullptr;
    {
        void* p = nullptr;
        rc = ctx_ensure(ctx, J_MISC, 64, &p);
        if (rc) return rc;
        total = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(p) + 32);
    }
    if (hipMemsetAsync(total, 0, 8, st) != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
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
    const int r_is_max = r >= 1.7976931348623157e308;
    hipEvent_t e0, e1;
    ctx_timing_events(ctx, &e0, &e1);
    if (e0) hipEventRecord(e0, st);
    const unsigned blocks = npoly ? npoly : 1;
    if (npoly) {
        if (!cap) {
            if (approximate) ppoly_probe<true, true><<<blocks, kTB, 0, st>>>(bk, dpoly, npoly, dvx, dvy, drects, r, r_is_max, total, nullptr, 0);
            else ppoly_probe<true, false><<<blocks, kTB, 0, st>>>(bk, dpoly, npoly, dvx, dvy, drects, r, r_is_max, total, nullptr, 0);
        } else {
            if (approximate) ppoly_probe<false, true><<<blocks, kTB, 0, st>>>(bk, dpoly, npoly, dvx, dvy, drects, r, r_is_max, total, out, cap);
            else ppoly_probe<false, false><<<blocks, kTB, 0, st>>>(bk, dpoly, npoly, dvx, dvy, drects, r, r_is_max, total, out, cap);
        }
        if (any_outside && n_out) {
            if (!cap)
                ppoly_outside<true><<<blocks, kTB, 0, st>>>(dx, dy, bk.outside_idx, n_out, grid->min_x, grid->min_y,
                                                            grid->cell_len, dpoly, npoly, drects, total, nullptr, 0);
            else
                ppoly_outside<false><<<blocks, kTB, 0, st>>>(dx, dy, bk.outside_idx, n_out, grid->min_x, grid->min_y,
                                                             grid->cell_len, dpoly, npoly, drects, total, out, cap);
        }
    }
    if (e1) hipEventRecord(e1, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("ppoly launch: ") + hipGetErrorString(e));
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

}  // namespace geohip
