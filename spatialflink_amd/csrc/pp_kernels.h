// pp_kernels.h -- launch interface of the libgeohip kernels (host side).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "geohip_internal.h"

namespace geohip {

struct KnnArgs {
    Box u[kMaxPointBoxes + 1];  // G u C as boxes
    int32_t nu;
    uint32_t k;
    double qx, qy;
    int32_t hist_base;  // (biased exponent of the lowest histogram octave) << 4
    int32_t pad;
};

struct RangeArgs {
    Box g[kMaxPointBoxes];
    Box c;
    int32_t ng, nc;
    double qx, qy, r;
    double r2lo, r2hi;  // squared screens (device_common.h kSqLo/kSqHi); r2lo < 0 disables
};

// kNN scan over ceil(n / chunk) = nblocks blocks (chunk a multiple of 1024); its last-arriving
// block runs the final selection into out_* (spill_cnt[0] = spill count, spill_cnt[1] = arrival
// ticket; both zero between launches).  ev0/ev1 (optional) bracket the one scan launch.
hipError_t launch_knn(const double* x, const double* y, uint64_t n, const KnnArgs& args, int kpl,
                      unsigned long long* part_d, unsigned* part_i, unsigned nblocks, uint64_t chunk, double* out_d,
                      unsigned* out_i, unsigned* out_count, unsigned long long* spill_d, unsigned* spill_i,
                      unsigned* spill_cnt, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1);
hipError_t launch_knn_scan_variant(int mode, const double* x, const double* y, uint64_t n, const KnnArgs& args,
                                   unsigned long long* part_d, unsigned* part_i, unsigned nblocks, uint64_t chunk,
                                   unsigned long long* spill_d, unsigned* spill_i, unsigned* spill_cnt, double* out_d,
                                   unsigned* out_i, unsigned* out_count, hipStream_t st);
// 1: final selection in the scan's last-arriving block (default); 0: separate knn_final launch
void set_knn_fused(int fused);
// measurement hook: fused range pass ablation (0 full, 1 counts only, 2 loads only)
void set_range_mode(int mode);
// kNN scan launch shape: waves per block (4, 8, 16), load pipeline depth (1, 2), arrival
// ticket groups (1 .. 64).  Returns -1 for an unsupported shape.
struct KnnConfig {
    int nw, pf, groups, epi_sort, interleave;
};
int set_knn_config(int nw, int pf, int groups, int epi_sort, int interleave);
KnnConfig knn_config();
// trace buffer of knn_scan MODE 6 (8 * (nblocks + 1) u64, device)
hipError_t set_knn_trace(unsigned long long* buf);
// blocks and chunk (points per block) of a kNN scan over n points under the current shape
void knn_geometry(uint64_t n, unsigned* nblocks, uint64_t* chunk);
// spill_cnt scratch (zeroed once; every user re-zeroes what it used): word 0 = spill count,
// arrival tickets from word kTicketStride (128 B apart), the final selection's head
// histogram (512 words) from word kGhistWord
constexpr unsigned kTicketStride = 32;  // words between counters
constexpr unsigned kMaxTicketGroups = 64;
constexpr unsigned kGhistWord = kTicketStride * (kMaxTicketGroups + 2);
constexpr int kGhistCopies = 8;
constexpr size_t kKnnCounterBytes = 32768;
hipError_t launch_knn_merge(const unsigned long long* d, const unsigned* i, unsigned nlists, unsigned list_len,
                            unsigned k, double* out_d, unsigned* out_i, unsigned* out_count, hipStream_t st);
// range: bitmask (16 words / 1024 pts), unit_count (units), offs (units) scratch.
hipError_t launch_range(const double* x, const double* y, uint64_t n, const RangeArgs& a, int approximate,
                        unsigned long long* bitmask, unsigned* unit_count, uint64_t* offs, uint64_t* total,
                        unsigned* out, uint64_t cap, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1,
                        unsigned long long* lb_status, unsigned* lb_ticket, unsigned long long epoch);
hipError_t launch_synth_uniform(double* x, double* y, uint64_t n, uint64_t base, uint64_t seed, double min_x,
                                double max_x, double min_y, double max_y, hipStream_t st);
hipError_t launch_selftest_fp64(const double* a, const double* b, uint64_t n, double* o_sqrt, double* o_div,
                                double* o_hypot, double* o_mulsub, hipStream_t st);

constexpr uint64_t kRangeUnitPts = 1024;

}  // namespace geohip
