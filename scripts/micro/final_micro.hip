// Microbenchmark (measurement only): costs of the kNN final's building blocks on one
// 1024-thread workgroup, timed in-kernel with s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(1024) void micro(unsigned long long* out, const unsigned long long* gsrc, int mode) {
    __shared__ __attribute__((aligned(16))) unsigned long long d[8192];
    __shared__ unsigned ix[8192];
    const unsigned t = threadIdx.x;
    for (unsigned i = t; i < 8192; i += 1024) { d[i] = (i * 2654435761u) & 0xffff; ix[i] = i; }
    __syncthreads();
    unsigned long long t0 = now();
    // 1: 16 barriers
    for (int i = 0; i < 16; i++) __syncthreads();
    unsigned long long t1 = now();
    // 2: 256-key rank (4 lanes per key, 64 slots per lane, 8-key batches)
    unsigned r = 0;
    {
        const unsigned k = t >> 2, g = t & 3;
        const unsigned long long kd = d[k];
#pragma unroll
        for (unsigned j = 64 * g; j < 64 * g + 64; j += 8) {
            ulonglong2 dd[4];
#pragma unroll
            for (int u = 0; u < 4; u++) dd[u] = *reinterpret_cast<const ulonglong2*>(d + j + 2 * u);
#pragma unroll
            for (int u = 0; u < 4; u++) r += (dd[u].x < kd) + (dd[u].y < kd);
        }
    }
    __syncthreads();
    unsigned long long t2 = now();
    // 3: 64 dependent LDS reads (pointer chase)
    unsigned p = t & 8191;
    for (int i = 0; i < 64; i++) p = ix[(p * 7 + 1) & 8191];
    __syncthreads();
    unsigned long long t3 = now();
    // 4: one global load round trip per thread
    unsigned long long v = gsrc[t * 17];
    __syncthreads();
    unsigned long long t4 = now();
    // 5: LDS atomics, all threads on one address
    atomicAdd(&ix[0], 1u);
    __syncthreads();
    unsigned long long t5 = now();
    if (t == 0) {
        out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = t5 - t4;
        out[5] = r + p + v;
    }
}

int main() {
    unsigned long long *out, *src;
    hipMalloc(&out, 64 * 8);
    hipMalloc(&src, 1 << 22);
    hipMemset(src, 1, 1 << 22);
    for (int rep = 0; rep < 3; rep++) {
        micro<<<1, 1024>>>(out, src, 0);
        hipDeviceSynchronize();
        unsigned long long h[8];
        hipMemcpy(h, out, 64, hipMemcpyDeviceToHost);
        printf("16 barriers %.2f us | rank256 %.2f us | 64 dep LDS reads %.2f us | global load %.2f us | 1024 same-addr LDS atomics %.2f us\n",
               h[0] / 100.0, h[1] / 100.0, h[2] / 100.0, h[3] / 100.0, h[4] / 100.0);
    }
    // the same with 255 other busy blocks streaming memory
    return 0;
}
