// Microbenchmark (measurement only): the HBM write rate of the join's pair-store shapes.  A
// 3.6 GB output (4.5e8 8-byte pairs, the C3 pair volume) written by waves that each store runs
// of R consecutive pairs (grid-stride over runs), per store width and cache policy.
//   hipcc -O3 --offload-arch=gfx950 store_micro.hip -o /tmp/store_micro && /tmp/store_micro
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

// W = 8: one pair per lane per store (512 B per wave-instruction); W = 16: two (1 KB)
template <int W, bool NT>
__global__ void store_runs(unsigned long long* __restrict__ out, uint64_t npairs, unsigned run) {
    const unsigned lane = threadIdx.x & 63;
    const uint64_t gw = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwt = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t nruns = npairs / run;
    for (uint64_t r = gw; r < nruns; r += nwt) {
        const uint64_t base = r * run;
        if (W == 8) {
            for (unsigned t = lane; t < run; t += 64) {
                const unsigned long long v = (base + t) * 0x9E3779B97F4A7C15ull;
                if (NT) __builtin_nontemporal_store(v, out + base + t);
                else out[base + t] = v;
            }
        } else {
            for (unsigned t = 2 * lane; t + 1 < run; t += 128) {
                const unsigned long long v = (base + t) * 0x9E3779B97F4A7C15ull;
                typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                u64x2* p = reinterpret_cast<u64x2*>(out + base + t);
                const u64x2 w = {v, v + 1};
                if (NT) __builtin_nontemporal_store(w, p);
                else *p = w;
            }
        }
    }
}

template <int W, bool NT>
static int run_case(const char* name, unsigned long long* out, uint64_t npairs, unsigned run, unsigned blocks,
                    unsigned threads) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f, sum = 0.f;
    const int reps = 6;
    for (int i = 0; i < reps + 1; i++) {
        CK(hipEventRecord(a));
        store_runs<W, NT><<<blocks, threads>>>(out, npairs, run);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (i == 0) continue;  // warmup
        sum += ms;
        if (ms < best) best = ms;
    }
    const double bytes = (double)(npairs / run) * run * 8.0;
    printf("%-10s run %4u  grid %5u x %4u  avg %.3f ms  %.2f TB/s (best %.2f)\n", name, run, blocks, threads,
           sum / reps, bytes / (sum / reps * 1e-3) / 1e12, bytes / (best * 1e-3) / 1e12);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

int main() {
    const uint64_t npairs = 450000000ull;
    unsigned long long* out;
    CK(hipMalloc(&out, npairs * 8));
    CK(hipMemset(out, 0, npairs * 8));
    int rc = 0;
    for (unsigned run : {64u, 448u, 4096u}) {
        rc |= run_case<8, true>("8B nt", out, npairs, run, 1280, 256);
        rc |= run_case<8, false>("8B plain", out, npairs, run, 1280, 256);
        rc |= run_case<16, true>("16B nt", out, npairs, run, 1280, 256);
        rc |= run_case<16, false>("16B plain", out, npairs, run, 1280, 256);
    }
    rc |= run_case<8, true>("8B nt", out, npairs, 448, 256, 1024);
    rc |= run_case<16, false>("16B plain", out, npairs, 448, 256, 1024);
    rc |= run_case<16, false>("16B plain", out, npairs, 448, 2560, 256);
    CK(hipFree(out));
    return rc;
}
