// sort.hip -- ascending (distance bits, index) order of a selected kNN set of any size.
//
// The large-k kNN paths (k above what one workgroup ranks in LDS: point kNN k > 1024, point-
// polygon kNN k > 256, rank merges of more than 8192 entries with k > 256) end with exactly the
// k smallest (dist, idx) keys, unordered.  Their order is the reference's output order
// (PointPointKNNQuery.java:125-191 + KNNQuery.java:204-272: ascending distance; the build breaks
// exact ties by index): two stable LSD radix passes -- by index, then by distance bits -- over
// the 96-bit key.  rocPRIM's onesweep radix sort does the passes; nothing here is on a per-window
// hot path (the large-k forms only).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <rocprim/device/device_radix_sort.hpp>

namespace geohip {

size_t sort_dist_idx_temp_bytes(unsigned n) {
    size_t a = 0, b = 0;
    if (rocprim::radix_sort_pairs(nullptr, a, (const unsigned*)nullptr, (unsigned*)nullptr,
                                  (const unsigned long long*)nullptr, (unsigned long long*)nullptr, n, 0, 32) !=
        hipSuccess)
        return 0;
    if (rocprim::radix_sort_pairs(nullptr, b, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                  (const unsigned*)nullptr, (unsigned*)nullptr, n, 0, 64) != hipSuccess)
        return 0;
    return std::max<size_t>(std::max(a, b), 16);
}

// (d_in[t], i_in[t]) for t < n sorted ascending by (d, i) into (d_out, i_out); d_tmp / i_tmp hold
// the intermediate order.  Inputs are not modified.
hipError_t sort_dist_idx(void* temp, size_t temp_bytes, const unsigned long long* d_in, const unsigned* i_in,
                         unsigned long long* d_tmp, unsigned* i_tmp, unsigned long long* d_out, unsigned* i_out,
                         unsigned n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    size_t tb = temp_bytes;
    hipError_t e = rocprim::radix_sort_pairs(temp, tb, i_in, i_tmp, d_in, d_tmp, n, 0, 32, st);
    if (e != hipSuccess) return e;
    tb = temp_bytes;
    return rocprim::radix_sort_pairs(temp, tb, d_tmp, d_out, i_tmp, i_out, n, 0, 64, st);
}

}  // namespace geohip
