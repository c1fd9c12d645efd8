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
    uint32_t point_base;  // added to every hit index (mod 2^32): a pane's stream position
    uint32_t pad;
};

// kNN counter scratch (zeroed once; every launch re-arms what it used): word 0 = spill count,
// arrival tickets from word kTicketStride (128 B apart)
constexpr unsigned kTicketStride = 32;  // words between counters
constexpr unsigned kMaxTicketGroups = 64;
constexpr unsigned kGhistWord = kTicketStride * (kMaxTicketGroups + 2);
constexpr int kGhistCopies = 8;
constexpr size_t kKnnCounterBytes = 32768;
// kNN pass (one launch per window; k <= GEOHIP_KNN_MAX_K): list_d/list_i hold
// knn_pass_list_entries(nblocks) entries (block lists, packed heads, lengths), spill_d/spill_i
// n entries, ctr is the kKnnCounterBytes zeroed counter scratch (re-armed by every launch).
void knn_pass_geometry(uint64_t n, unsigned* nblocks, uint64_t* chunk);
size_t knn_pass_list_entries(unsigned nblocks);
// The range query of the same point fused into the pass (see knn_pass; status = kPassMaxBlocks
// epoch-tagged look-back words shared with the range pass).
struct PassRangeIo {
    RangeArgs a;
    int approximate;
    unsigned long long* status;
    unsigned long long epoch;
    unsigned* out;
    uint64_t cap;
    uint64_t* total;
    unsigned long long* trace;  // measurement only: look-back done / hits written at [8 b + 5, 6]
    unsigned* fault;            // set when the look-back wait gives up (poll_block_counts)
    unsigned spin_limit, inject;
    // unordered (geohip_ctx_set_range_order GEOHIP_ORDER_ANY): no look-back -- each block reserves
    // its hits on *cursor (zero before a launch; the kNN's last block writes the total and
    // re-arms it) and the pass sweeps the window in interleaved fronts as the kNN alone does
    int unordered;
    unsigned long long* cursor;
};
// whether a window of n points fits the fused kNN + range pass (block chunk <= 131072 points)
bool knn_pass_fuses_range(uint64_t n);
hipError_t launch_knn_pass(const double* x, const double* y, uint64_t n, const KnnArgs& args,
                           unsigned long long* list_d, unsigned* list_i, unsigned long long* spill_d, unsigned* spill_i,
                           unsigned* ctr, double* out_d, unsigned* out_i, unsigned* out_count, hipStream_t st,
                           hipEvent_t ev0, hipEvent_t ev1, unsigned long long* trace = nullptr, int abl = 0,
                           const PassRangeIo* range = nullptr);
// add chunk * chunk_pts to every valid index of nlists lists of k (host windows staged in chunks)
hipError_t launch_knn_rebase(unsigned* idx, unsigned nlists, unsigned k, uint64_t chunk_pts, hipStream_t st);
hipError_t launch_knn_merge(const unsigned long long* d, const unsigned* i, unsigned nlists, unsigned list_len,
                            unsigned k, double* out_d, unsigned* out_i, unsigned* out_count, hipStream_t st);
// pane merge: n lists of list_len in ring slots slot[0..n) (oldest first), indices + off[b]
constexpr unsigned kMaxPanes = 16;
struct PaneMerge {
    unsigned slot[kMaxPanes];
    unsigned off[kMaxPanes];
    unsigned n, list_len, k, pad;
};
hipError_t launch_knn_merge_panes(const unsigned long long* ring_d, const unsigned* ring_i, const PaneMerge& pm,
                                  double* out_d, unsigned* out_i, unsigned* out_count, hipStream_t st,
                                  hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);  // timed: the kernel's stamps
// range: bitmask (16 words / 1024 pts), unit_count (units), offs (units) scratch.
// the range runs as one fused kernel at this window size (else three launches)
bool range_is_one_kernel(uint64_t n);
hipError_t launch_range(const double* x, const double* y, uint64_t n, const RangeArgs& a, int approximate,
                        unsigned long long* bitmask, unsigned* unit_count, uint64_t* offs, uint64_t* total,
                        unsigned* out, uint64_t cap, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1,
                        unsigned long long* lb_status, unsigned* lb_ticket, unsigned long long epoch,
                        unsigned* lb_fault, unsigned lb_spins, unsigned lb_inject);
// range with unordered-set output: io.word = (hits reserved << 20) | blocks arrived, zero before
// the first launch (each launch's last block re-arms it); grid <= min(cus, 2^20 - 1) blocks
struct RangeSetIo {
    unsigned long long* word;
};
hipError_t launch_range_set(const double* x, const double* y, uint64_t n, const RangeArgs& a, int approximate,
                            const RangeSetIo& io, uint64_t* total, unsigned* out, uint64_t cap, unsigned cus,
                            hipStream_t st, hipEvent_t ev0, hipEvent_t ev1);
hipError_t launch_synth_uniform(double* x, double* y, uint64_t n, uint64_t base, uint64_t seed, double min_x,
                                double max_x, double min_y, double max_y, hipStream_t st);
hipError_t launch_selftest_fp64(const double* a, const double* b, uint64_t n, double* o_sqrt, double* o_div,
                                double* o_hypot, double* o_mulsub, hipStream_t st);

constexpr uint64_t kRangeUnitPts = 1024;

}  // namespace geohip
