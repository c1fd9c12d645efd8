// join.h -- point-point window join (PointPointJoinQuery.java:113-172).
#pragma once
#include <type_traits>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "geohip_internal.h"

namespace geohip {
// The ctx's device fault word (bits; read, reported and cleared by geohip_ctx_sync and by the
// synchronous calls): a device-side condition an enqueue-only call cannot return as a status.
constexpr unsigned kFaultLookback = 1u;       // a look-back wait gave up (GEOHIP_ERR_DEVICE)
constexpr unsigned kFaultQueryKey = 2u;       // join query key: NumberFormatException (GEOHIP_ERR_ARG)
constexpr unsigned kFaultQueryLoop = 4u;      // join query block: a loop that never ends (GEOHIP_ERR_ARG)
constexpr unsigned kFaultCandNeed = 8u;       // point-polygon: the candidate buffer was short (a hint, not an
                                              // error: the stream decided the rest; the size it needed)

// context services implemented in abi.cpp
int ctx_fail(geohip_ctx* ctx, int code, const std::string& msg);
int ctx_ensure(geohip_ctx* ctx, int slot, size_t bytes, void** out);  // slot 0..27 (JSlot, cell_kernels.hip)
int ctx_ensure_zeroed(geohip_ctx* ctx, int slot, size_t bytes, void** out);  // zeroed when (re)allocated
int ctx_ensure_ingest(geohip_ctx* ctx, int slot, size_t bytes, void** out);  // slot 0..11
int ctx_ensure_ingest_zeroed(geohip_ctx* ctx, int slot, size_t bytes, void** out);  // zeroed when (re)allocated
unsigned long long ctx_next_epoch(geohip_ctx* ctx);  // look-back epoch: 1 .. 2^22 - 1, new per call
// the ingest look-back status slot (zeroed on allocation and on epoch wrap) and this call's epoch
int ctx_lookback_status(geohip_ctx* ctx, int slot, size_t bytes, void** out, unsigned long long* epoch);
int ctx_cus(geohip_ctx* ctx);                       // compute units of the ctx's device
int ctx_begin(geohip_ctx* ctx);  // clears the error, selects the ctx's device
hipStream_t ctx_stream(geohip_ctx* ctx);
int ctx_mem(geohip_ctx* ctx);
uint64_t* ctx_pinned(geohip_ctx* ctx);
// the fault block on the device: word 0 = fault bits, words 2..3 = the u64 candidate count an
// overflowing async point-polygon call needed (atomicMax); allocated zeroed on first use
int ctx_fault_block(geohip_ctx* ctx, unsigned** out);
void ctx_timing_events(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1);      // a step of several launches
void ctx_kernel_events(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1);      // one kernel inside such a step
void ctx_kernel_step_events(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1); // a step that is one kernel

// A kernel of a timed step: while the ctx's timing is on, launched with a fresh event pair that
// its own dispatch stamps (begin / end, the durations rocprofv3 reports), so a step's kernel time
// is the sum of its kernels without the gaps between them.
// The arguments are packed as given (no conversion to the kernel's parameter types), so they must
// match those types in size and kind (a pointer may gain const): checked at compile time.
template <typename... P, typename... A>
inline void tlaunch(geohip_ctx* ctx, void (*kernel)(P...), dim3 grid, dim3 block, uint32_t shm, hipStream_t st, A... a) {
    static_assert(sizeof...(P) == sizeof...(A), "tlaunch: argument count");
    static_assert(((sizeof(typename std::decay<P>::type) == sizeof(A) &&
                    std::is_convertible<A, typename std::decay<P>::type>::value &&
                    std::is_floating_point<typename std::decay<P>::type>::value == std::is_floating_point<A>::value) && ...),
                  "tlaunch: argument types must match the kernel's (same size and kind)");
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (ctx) ctx_kernel_events(ctx, &e0, &e1);
    hipExtLaunchKernelGGL(kernel, grid, block, shm, st, e0, e1, 0, a...);
}
int ctx_stage_xy(geohip_ctx* ctx, const double* x, const double* y, uint64_t n, int which, const double** dx,
                 const double** dy);
void** ctx_pcache_slot(geohip_ctx* ctx);  // the ctx's point-polygon plan cache (owned by cell_kernels)
void** ctx_kcache_slot(geohip_ctx* ctx);  // the ctx's point-polygon kNN polygon cache

// squared-distance screen bounds for "dist <= r" (r2lo < 0 / r2hi = inf where they cannot hold)
void pp_screen_bounds(double r, double* r2lo, double* r2hi);

// count_dev (async, device window and outputs): the pair total goes there, nothing is read back
int join_pp_impl(geohip_ctx* ctx, const geohip_grid* grid_data, const geohip_grid* grid_query, const double* dx,
                 const double* dy, uint64_t nd, const double* qx, const double* qy, uint64_t nq, double r,
                 int approximate, uint32_t* out_pairs, uint64_t cap, uint64_t* out_count, bool count_only,
                 uint64_t* count_dev = nullptr);
// key-band owner partition of a window (band.hip; geohip_band_pack_async)
int band_pack_impl(geohip_ctx* ctx, const geohip_grid* grid, int32_t nb, uint32_t world, const double* x,
                   const double* y, uint64_t n, int64_t base, double* out_x, double* out_y, int64_t* out_idx,
                   uint64_t* out_counts, const PointPlan* filter = nullptr);
// point output codecs (format.hip; geohip_format_points, geohip_format_points_csv)
int format_points_impl(geohip_ctx* ctx, const geohip_text_out_spec* spec, const double* x, const double* y, uint64_t n,
                       const int64_t* ts, const uint8_t* oid_text, const uint64_t* oid_off, const uint32_t* idx,
                       uint64_t m, uint8_t* out, uint64_t cap, uint64_t* out_len, uint64_t* rec_off);
int format_csv_impl(geohip_ctx* ctx, const geohip_csv_out_spec* spec, const double* x, const double* y, uint64_t n,
                    const int64_t* ts, const uint8_t* oid_text, const uint64_t* oid_off, const uint32_t* idx,
                    uint64_t m, uint8_t* out, uint64_t cap, uint64_t* out_len, uint64_t* rec_off);
}  // namespace geohip
