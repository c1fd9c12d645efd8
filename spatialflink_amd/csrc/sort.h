// sort.h -- (distance bits, index) sort of the large-k kNN forms (sort.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace geohip {
// temporary storage sort_dist_idx needs for n entries (0: the query failed)
size_t sort_dist_idx_temp_bytes(unsigned n);
// (d_in, i_in)[0, n) ascending by (d, i) into (d_out, i_out); d_tmp / i_tmp: n entries each
hipError_t sort_dist_idx(void* temp, size_t temp_bytes, const unsigned long long* d_in, const unsigned* i_in,
                         unsigned long long* d_tmp, unsigned* i_tmp, unsigned long long* d_out, unsigned* i_out,
                         unsigned n, hipStream_t st);
}  // namespace geohip
