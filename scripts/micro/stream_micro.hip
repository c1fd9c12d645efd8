// Microbenchmark (measurement only): what one launch that streams a 10M-point SoA window
// (x, y fp64 = 160 MB) costs on this chip, per launch geometry, with the windows cycled through
// a ring larger than the Infinity Cache.  Floors for knn_pass: an empty launch of the same
// geometry and a loads-only pass (4 x 16 B per lane per 256-point iteration, two in flight).
//   hipcc -O3 --offload-arch=gfx950 stream_micro.hip -o /tmp/stream_micro && /tmp/stream_micro
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void empty_k(double* out) {
    if (threadIdx.x == 0 && out == nullptr) out[blockIdx.x] = 0.0;
}

// contiguous chunk per block, waves take 256-point iterations round robin (static)
__global__ void stream_k(const double* __restrict__ x, const double* __restrict__ y, uint64_t n, uint64_t chunk,
                         double* out) {
    const unsigned lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint64_t b0 = (uint64_t)blockIdx.x * chunk;
    uint64_t b1 = b0 + chunk;
    if (b1 > n) b1 = n;
    double acc = 0.0;
    for (uint64_t i = b0 + (uint64_t)wid * 256; i + 256 <= b1; i += (uint64_t)nw * 256) {
        const uint64_t j = i + 2 * lane;
        const double2 u0 = *reinterpret_cast<const double2*>(x + j);
        const double2 u1 = *reinterpret_cast<const double2*>(x + j + 128);
        const double2 v0 = *reinterpret_cast<const double2*>(y + j);
        const double2 v1 = *reinterpret_cast<const double2*>(y + j + 128);
        acc += (u0.x < v0.y) + (u1.x < v1.y) + (u0.y < v0.x) + (u1.y < v1.x);
    }
    if (acc == 12345.0) out[blockIdx.x] = acc;
}

// grid-stride over 256-point iterations (one wave per iteration, iterations interleaved over
// the whole grid)
__global__ void stream_gs(const double* __restrict__ x, const double* __restrict__ y, uint64_t n, double* out) {
    const unsigned lane = threadIdx.x & 63;
    const uint64_t gw = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwt = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    double acc = 0.0;
    for (uint64_t i = gw * 256; i + 256 <= n; i += nwt * 256) {
        const uint64_t j = i + 2 * lane;
        const double2 u0 = *reinterpret_cast<const double2*>(x + j);
        const double2 u1 = *reinterpret_cast<const double2*>(x + j + 128);
        const double2 v0 = *reinterpret_cast<const double2*>(y + j);
        const double2 v1 = *reinterpret_cast<const double2*>(y + j + 128);
        acc += (u0.x < v0.y) + (u1.x < v1.y) + (u0.y < v0.x) + (u1.y < v1.x);
    }
    if (acc == 12345.0) out[blockIdx.x] = acc;
}

// dynamic: the window is split into 8 regions, one per counter; a wave claims U-iteration units
// from counter (block % 8) and, once that region is drained, from the next ones.  The claim of
// the next unit is issued before the current unit's loads (its latency hides behind them).
template <int U>
__global__ void stream_dyn(const double* __restrict__ x, const double* __restrict__ y, uint64_t n,
                           unsigned* ctr, double* out) {
    const unsigned lane = threadIdx.x & 63;
    const uint64_t iters = n / 256;
    const uint64_t units = (iters + U - 1) / U;
    const uint64_t per = (units + 7) / 8;
    unsigned c = blockIdx.x & 7, tried = 0;
    auto claim = [&]() -> uint64_t {
        while (tried < 8) {
            unsigned v = 0;
            if (lane == 0) v = __hip_atomic_fetch_add(ctr + 16 * c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = __builtin_amdgcn_readfirstlane(v);
            const uint64_t u = (uint64_t)c * per + v;
            if (v < per && u < units) return u;
            c = (c + 1) & 7;
            tried++;
        }
        return ~0ull;
    };
    double acc = 0.0;
    uint64_t u = claim();
    while (u != ~0ull) {
        const uint64_t nu = claim();
        const uint64_t i0 = u * U * 256, i1 = (u + 1) * U * 256 < iters * 256 ? (u + 1) * U * 256 : iters * 256;
        for (uint64_t i = i0; i < i1; i += 256) {
            const uint64_t j = i + 2 * lane;
            const double2 u0 = *reinterpret_cast<const double2*>(x + j);
            const double2 u1 = *reinterpret_cast<const double2*>(x + j + 128);
            const double2 v0 = *reinterpret_cast<const double2*>(y + j);
            const double2 v1 = *reinterpret_cast<const double2*>(y + j + 128);
            acc += (u0.x < v0.y) + (u1.x < v1.y) + (u0.y < v0.x) + (u1.y < v1.x);
        }
        u = nu;
    }
    if (acc == 12345.0) out[blockIdx.x] = acc;
}

int main() {
    const uint64_t n = 10000000;
    const int W = 4;
    double *x[W], *y[W], *out;
    for (int w = 0; w < W; w++) {
        CK(hipMalloc(&x[w], n * 8));
        CK(hipMalloc(&y[w], n * 8));
        CK(hipMemset(x[w], 0, n * 8));
        CK(hipMemset(y[w], 0, n * 8));
    }
    CK(hipMalloc(&out, 65536 * 8));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct G { int blocks, threads; } geo[] = {{256, 1024}, {256, 512}, {512, 512}, {512, 1024}, {1024, 256}, {1024, 512}, {2048, 256}, {4096, 256}};
    const int R = 40;
    unsigned* ctr;
    const size_t nctr = (size_t)(R + 4) * 16 * 8 * 8;
    CK(hipMalloc(&ctr, nctr * 4));
    for (int mode = 0; mode < 6; mode++) {
        for (auto g : geo) {
            CK(hipMemset(ctr, 0, nctr * 4));
            CK(hipDeviceSynchronize());
            const uint64_t iters = (n + 255) / 256;
            const uint64_t chunk = ((iters + g.blocks - 1) / g.blocks) * 256;
            float best = 1e9f, sum = 0.f;
            for (int r = 0; r < R + 4; r++) {
                const int w = r % W;
                CK(hipEventRecord(e0, s));
                if (mode == 0) empty_k<<<g.blocks, g.threads, 0, s>>>(out);
                else if (mode == 1) stream_k<<<g.blocks, g.threads, 0, s>>>(x[w], y[w], n, chunk, out);
                else if (mode == 2) stream_gs<<<g.blocks, g.threads, 0, s>>>(x[w], y[w], n, out);
                else if (mode == 3) stream_dyn<2><<<g.blocks, g.threads, 0, s>>>(x[w], y[w], n, ctr + (size_t)r * 16 * 8, out);
                else if (mode == 4) stream_dyn<4><<<g.blocks, g.threads, 0, s>>>(x[w], y[w], n, ctr + (size_t)r * 16 * 8, out);
                else stream_dyn<8><<<g.blocks, g.threads, 0, s>>>(x[w], y[w], n, ctr + (size_t)r * 16 * 8, out);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 4) {
                    sum += ms;
                    if (ms < best) best = ms;
                }
            }
            const double us = 1000.0 * sum / R;
            printf("%-10s blocks %5d threads %5d  avg %7.2f us  min %7.2f us  %6.2f TB/s\n",
                   mode == 0 ? "empty" : mode == 1 ? "chunked" : mode == 2 ? "gridstride" : mode == 3 ? "dyn2" : mode == 4 ? "dyn4" : "dyn8", g.blocks, g.threads, us, 1000.0 * best,
                   mode ? 16.0 * n / (us * 1e-6) / 1e12 : 0.0);
        }
    }
    return 0;
}
