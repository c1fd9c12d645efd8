// abi.cpp -- the extern "C" boundary of libgeohip.so (include/geohip.h).
//
// Owns contexts (device, stream, grow-on-demand device scratch, pinned readback words,
// optional per-launch event timing), validates arguments the way the reference fails
// (System.exit / exceptions -> status codes, never abort), plans each query on the host
// (plan.cpp) and launches the gfx950 kernels (pp_kernels.hip, join.hip, ppoly.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

#include "geohip_internal.h"
#include "join.h"
#include "pp_kernels.h"
#include "ppoly.h"

using namespace geohip;

enum Slot {
    S_X, S_Y, S_QX, S_QY, S_GTHR, S_PART_D, S_PART_I, S_OUT_D, S_OUT_I, S_OUT_CNT,
    S_MASK, S_UCNT, S_OFFS, S_TOTAL, S_OUT_IDX, S_OUT_PAIRS, S_SPILL_D, S_SPILL_I, S_SPILL_CNT, S_RLB, S_TRACE,
    S_J0, S_J1, S_J2, S_J3, S_J4, S_J5, S_J6, S_J7, S_J8, S_J9, S_J10, S_J11, S_J12, S_J13, S_J14, S_J15,
    S_J16, S_J17, S_J18, S_J19, S_J20, S_J21, S_J22, S_J23, S_J24, S_J25, S_J26, S_J27,
    S_I0, S_I1, S_I2, S_I3, S_I4, S_I5, S_I6, S_I7, S_I8, S_I9, S_I10, S_I11,
    S_COUNT
};

// Persistent copy workers of one ctx (host staging): a job is a list of (dst, src, bytes)
// slices, one per worker; the caller waits until every slice is done.
struct CopyPool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::vector<std::tuple<char*, const char*, size_t>> work;
    uint64_t gen = 0;
    unsigned pending = 0;
    bool stop = false;
    explicit CopyPool(unsigned n) {
        // fewer workers when thread creation fails (RLIMIT_NPROC, a container): std::system_error
        // must not cross the C ABI; stage_copy splits over the workers that exist (none: memcpy)
        for (unsigned t = 0; t < n; t++) try {
            th.emplace_back([this, t] {
                uint64_t seen = 0;
                for (;;) {
                    std::tuple<char*, const char*, size_t> w{nullptr, nullptr, 0};
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        if (t < work.size()) w = work[t];
                    }
                    if (std::get<2>(w)) memcpy(std::get<0>(w), std::get<1>(w), std::get<2>(w));
                    {
                        std::lock_guard<std::mutex> lk(mu);
                        if (--pending == 0) done_cv.notify_one();
                    }
                }
            });
        } catch (...) {
            break;
        }
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& h : th) h.join();
    }
    // copy the slices in parallel (at most one per worker) and wait
    void run(const std::vector<std::tuple<char*, const char*, size_t>>& slices) {
        std::unique_lock<std::mutex> lk(mu);
        work = slices;
        pending = (unsigned)th.size();
        gen++;
        cv.notify_all();
        done_cv.wait(lk, [&] { return pending == 0; });
    }
};

struct geohip_ctx {
    int device = 0;
    int cus = 256;               // compute units of the device (persistent grids)
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    int mem = GEOHIP_MEM_HOST;
    std::string err;
    void* buf[S_COUNT] = {};
    size_t cap[S_COUNT] = {};
    uint64_t* pinned = nullptr;  // 8 words of pinned host memory for count readback
    bool timing = false;
    // timed event pairs since the last readout: kind 0 = a step bracketed by hipEventRecord (its
    // kernels and the gaps between them), 1 = one kernel of such a step, 2 = a step that is one
    // kernel; kinds 1 and 2 are stamped by the kernel's own dispatch (hipExtLaunchKernel), the
    // begin/end timestamps rocprofv3 reports
    struct TimedPair {
        hipEvent_t a, b;
        int kind;
    };
    std::vector<TimedPair> pending;
    std::vector<hipEvent_t> pool;
    double acc_ms = 0.0;      // steps (kinds 0, 2)
    uint64_t launches = 0;    // steps
    double kern_ms = 0.0;     // kernels (kinds 1, 2)
    uint64_t kernels = 0;
    // last point plan: a continuous query plans the same (grid, q, r) for every window
    bool plan_valid = false;
    geohip_grid plan_grid{};
    double plan_q[3] = {0, 0, 0};
    PointPlan plan{};
    unsigned long long range_epoch = 0;  // fused range pass: status words of this launch carry it
    bool lb_inject = false;              // test knob: range look-back waits give up (geohip_debug_lookback_inject)
    int range_order = GEOHIP_ORDER_ASCENDING;  // geohip_ctx_set_range_order
    unsigned long long lb_epoch = 0;     // chunk look-backs (ingest, point-polygon stream): status words of a launch carry it
    // host windows (GEOHIP_MEM_HOST): two pinned staging slots; the DMA of one slot runs on the
    // copy stream while the host fills the other (host_stage)
    hipStream_t cstream = nullptr;
    char* stg[2] = {nullptr, nullptr};
    hipEvent_t stg_ev[2] = {nullptr, nullptr};
    bool stg_used[2] = {false, false};
    std::unique_ptr<CopyPool> copy_pool;
    hipEvent_t switch_ev = nullptr;  // orders a stream rebinding after the old stream's work
    void* pcache = nullptr;          // point-polygon plan cache (cell_kernels.hip owns the type)
    void* kcache = nullptr;          // point-polygon kNN polygon cache (cell_kernels.hip owns the type)
};

namespace {

int fail(geohip_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int hip_fail(geohip_ctx* c, hipError_t e, const char* where) {
    return fail(c, GEOHIP_ERR_DEVICE, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIPCHK(expr)                                          \
    do {                                                      \
        hipError_t e_ = (expr);                               \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr); \
    } while (0)

int ensure(geohip_ctx* ctx, Slot s, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (ctx->cap[s] >= bytes) return GEOHIP_OK;
    if (ctx->buf[s]) {
        hipStreamSynchronize(ctx->stream);
        hipFree(ctx->buf[s]);
        ctx->buf[s] = nullptr;
        ctx->cap[s] = 0;
    }
    size_t want = bytes + bytes / 4;
    want = (want + 255) & ~(size_t)255;
    void* p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) {
        (void)hipGetLastError();
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            return fail(ctx, GEOHIP_ERR_OOM, "device allocation of " + std::to_string(bytes) + " bytes failed");
        }
        want = bytes;
    }
    ctx->buf[s] = p;
    ctx->cap[s] = want;
    return GEOHIP_OK;
}

template <typename T>
T* B(geohip_ctx* ctx, Slot s) { return reinterpret_cast<T*>(ctx->buf[s]); }

int ensure_zeroed(geohip_ctx* ctx, Slot s, size_t bytes) {
    const bool fresh = ctx->cap[s] < (bytes ? bytes : 16);
    int rc = ensure(ctx, s, bytes);
    if (rc) return rc;
    if (fresh && hipMemsetAsync(ctx->buf[s], 0, ctx->cap[s], ctx->stream) != hipSuccess)
        return fail(ctx, GEOHIP_ERR_DEVICE, "memset failed");
    return GEOHIP_OK;
}

// The range look-back words (S_RLB): 256 block-count status words, then the arrival ticket, then
// the fault block (16 B), then the unordered range's reservation word (u64: hits << 20 | blocks
// arrived).  Zeroed on allocation; the status words again when the 24-bit epoch wraps (a word last
// written 2^24 - 1 launches ago must not read as ready); the reservation word is re-armed by the
// last block of each launch.
constexpr size_t kRlbBytes = 256 * 8 + 64;
struct RangeLb {
    unsigned long long* status;
    unsigned* ticket;
    unsigned* fault;
    unsigned long long epoch;
    unsigned spins, inject;
    RangeSetIo set;
};
int range_lookback(geohip_ctx* ctx, RangeLb* lb) {
    int rc = ensure_zeroed(ctx, S_RLB, kRlbBytes);
    if (rc) return rc;
    ctx->range_epoch = ctx->range_epoch % ((1ull << 24) - 1) + 1;
    char* base = B<char>(ctx, S_RLB);
    if (ctx->range_epoch == 1 && hipMemsetAsync(base, 0, 256 * 8, ctx->stream) != hipSuccess)
        return fail(ctx, GEOHIP_ERR_DEVICE, "look-back status reset failed");
    lb->status = reinterpret_cast<unsigned long long*>(base);
    lb->ticket = reinterpret_cast<unsigned*>(base + 256 * 8);
    lb->fault = reinterpret_cast<unsigned*>(base + 256 * 8 + 16);
    lb->set.word = reinterpret_cast<unsigned long long*>(base + 256 * 8 + 32);
    lb->epoch = ctx->range_epoch;
    lb->spins = ctx->lb_inject ? 4096u : (1u << 22);  // kLookbackSpins (device_common.h): seconds
    lb->inject = ctx->lb_inject ? 1u : 0u;
    return GEOHIP_OK;
}

// The fault block (the S_RLB tail, join.h kFault*): word 0 = fault bits, words 2..3 = the
// candidate count an overflowing async point-polygon call needed.
constexpr size_t kFaultOff = 256 * 8 + 16;
unsigned* fault_block(geohip_ctx* ctx) {
    return ctx->buf[S_RLB] ? reinterpret_cast<unsigned*>(B<char>(ctx, S_RLB) + kFaultOff) : nullptr;
}
constexpr int kPinFault = 6;  // pinned[6] = fault bits, pinned[7] = the candidate need

// Queue the fault block's read into pinned[6..7] behind the call's own readback (one
// synchronisation covers both; nothing to read before the block exists).
int queue_fault_read(geohip_ctx* ctx) {
    ctx->pinned[kPinFault] = 0;
    ctx->pinned[kPinFault + 1] = 0;
    unsigned* fw = fault_block(ctx);
    if (fw) HIPCHK(hipMemcpyAsync(ctx->pinned + kPinFault, fw, 16, hipMemcpyDeviceToHost, ctx->stream));
    return GEOHIP_OK;
}

// After the synchronisation that follows queue_fault_read: the faults since the last check as
// one status (the block cleared on the ctx's stream, the candidate need kept for the next call).
// `mask` = the fault bits this caller consumes: the synchronous range / kNN calls take only their
// own look-back bit and leave an earlier async call's faults for geohip_ctx_sync (geohip.h).
int report_faults(geohip_ctx* ctx, unsigned mask = ~0u) {
    const unsigned seen = (unsigned)(ctx->pinned[kPinFault] & 0xffffffffu);
    const unsigned bits = seen & mask;
    if (!bits) return GEOHIP_OK;
    const uint64_t need = ctx->pinned[kPinFault + 1];
    const unsigned rest = seen & ~mask;
    if (rest)  // keep the other calls' bits (and the candidate need) for their own check
        HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(fault_block(ctx)), (int)rest, 1, ctx->stream));
    else
        HIPCHK(hipMemsetAsync(fault_block(ctx), 0, 16, ctx->stream));
    if (bits & kFaultCandNeed) ppoly_note_cand_need(ctx, need);  // a sizing hint, not an error
    if (bits & kFaultLookback)
        return fail(ctx, GEOHIP_ERR_DEVICE, "range look-back wait gave up (a block count never arrived); results invalid");
    if (bits & kFaultQueryKey)
        return fail(ctx, GEOHIP_ERR_ARG, "async join: NumberFormatException in getIntCellIndices (query point key)");
    if (bits & kFaultQueryLoop)
        return fail(ctx, GEOHIP_ERR_ARG, "async join: reference neighbour loop does not terminate");
    return GEOHIP_OK;
}

int begin(geohip_ctx* ctx) {
    if (!ctx) return GEOHIP_ERR_ARG;
    ctx->err.clear();
    // switch the calling thread's device only when it differs (hipGetDevice reads thread state)
    int current = -1;
    if (hipGetDevice(&current) != hipSuccess || current != ctx->device) {
        hipError_t e = hipSetDevice(ctx->device);
        if (e != hipSuccess) return hip_fail(ctx, e, "hipSetDevice");
    }
    return GEOHIP_OK;
}

void timed_pair(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1, int kind) {
    *e0 = *e1 = nullptr;
    if (!ctx->timing) return;
    hipEvent_t ev[2] = {nullptr, nullptr};
    for (int t = 0; t < 2; t++) {
        if (!ctx->pool.empty()) {
            ev[t] = ctx->pool.back();
            ctx->pool.pop_back();
        } else if (hipEventCreate(&ev[t]) != hipSuccess) {
            if (t) ctx->pool.push_back(ev[0]);
            return;
        }
    }
    *e0 = ev[0];
    *e1 = ev[1];
    ctx->pending.push_back({ev[0], ev[1], kind});
}

// a step of several launches: the caller records e0 / e1 around them (hipEventRecord)
void timing_events(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1) { timed_pair(ctx, e0, e1, 0); }
// a step that is one kernel: e0 / e1 go to hipExtLaunchKernel (the kernel's own timestamps)
void kernel_step_events(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1) { timed_pair(ctx, e0, e1, 2); }

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Stage x/y for the kernels: host pointers are copied into ctx scratch, device pointers used.
// ---- host windows: chunked staging through ctx-owned pinned slots ------------------------
// A pageable host window reaches the device in chunks of kStagePts points: the host copies chunk
// c into pinned slot c % 2 (kStageThreads threads) while the DMA of chunk c - 1 runs on the copy
// stream; each chunk's arrival is an event the compute stream can wait on, so kernels over
// landed chunks overlap the copies of later ones (the kNN pipelines this way).
constexpr uint64_t kStagePts = 1ull << 20;      // 16 MB of x + y per slot
constexpr unsigned kStageThreads = 16;


int stage_init(geohip_ctx* ctx) {
    if (ctx->cstream) return GEOHIP_OK;
    HIPCHK(hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking));
    const unsigned hw = std::thread::hardware_concurrency();
    const unsigned nw = std::max(2u, std::min(kStageThreads, hw ? hw : 2u));
    try {
        ctx->copy_pool = std::make_unique<CopyPool>(nw);
    } catch (...) {
        return fail(ctx, GEOHIP_ERR_OOM, "host staging: copy worker pool");
    }
    for (int k = 0; k < 2; k++) {
        HIPCHK(hipHostMalloc((void**)&ctx->stg[k], kStagePts * 16, hipHostMallocDefault));
        HIPCHK(hipEventCreateWithFlags(&ctx->stg_ev[k], hipEventDisableTiming));
        ctx->stg_used[k] = false;
    }
    return GEOHIP_OK;
}

// x and y of one chunk into a pinned slot, split over the ctx's copy workers
void stage_copy(geohip_ctx* ctx, char* dx, const char* sx, char* dy, const char* sy, size_t bytes) {
    if (bytes < (1u << 18) || !ctx->copy_pool || ctx->copy_pool->th.empty()) {
        memcpy(dx, sx, bytes);
        memcpy(dy, sy, bytes);
        return;
    }
    const unsigned nw = (unsigned)ctx->copy_pool->th.size();
    const unsigned half = nw / 2 ? nw / 2 : 1;
    std::vector<std::tuple<char*, const char*, size_t>> sl;
    const size_t per = ((bytes + half - 1) / half + 63) & ~(size_t)63;
    for (int a = 0; a < 2; a++)
        for (unsigned t = 0; t < half; t++) {
            const size_t b = t * per, e = std::min(bytes, b + per);
            if (b < e) sl.emplace_back((a ? dy : dx) + b, (a ? sy : sx) + b, e - b);
        }
    ctx->copy_pool->run(sl);
}

// Copies host x/y[0, n) to device dx/dy; after chunk c is enqueued, on_chunk(c, first, count,
// arrival event) runs (it may make ctx->stream wait on the event and launch work on the chunk).
// On return ctx->stream is ordered after every chunk's DMA.
template <typename F>
int host_stage(geohip_ctx* ctx, const double* x, const double* y, uint64_t n, double* dx, double* dy, F&& on_chunk) {
    int rc = stage_init(ctx);
    if (rc) return rc;
    const uint64_t nch = (n + kStagePts - 1) / kStagePts;
    for (uint64_t c = 0; c < nch; c++) {
        const int slot = (int)(c & 1);
        const uint64_t b = c * kStagePts, m = std::min<uint64_t>(kStagePts, n - b);
        if (ctx->stg_used[slot]) HIPCHK(hipEventSynchronize(ctx->stg_ev[slot]));  // slot's last DMA done
        char* sp = ctx->stg[slot];
        stage_copy(ctx, sp, reinterpret_cast<const char*>(x + b), sp + kStagePts * 8, reinterpret_cast<const char*>(y + b),
                   m * 8);
        HIPCHK(hipMemcpyAsync(dx + b, sp, m * 8, hipMemcpyHostToDevice, ctx->cstream));
        HIPCHK(hipMemcpyAsync(dy + b, sp + kStagePts * 8, m * 8, hipMemcpyHostToDevice, ctx->cstream));
        HIPCHK(hipEventRecord(ctx->stg_ev[slot], ctx->cstream));
        ctx->stg_used[slot] = true;
        rc = on_chunk(c, b, m, ctx->stg_ev[slot]);
        if (rc) return rc;
    }
    for (int k = 0; k < 2; k++)
        if (ctx->stg_used[k]) HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->stg_ev[k], 0));
    return GEOHIP_OK;
}

int stage_xy(geohip_ctx* ctx, const double* x, const double* y, uint64_t n, Slot sx, Slot sy,
             const double** dx, const double** dy) {
    if (n == 0) {
        *dx = *dy = nullptr;
        return GEOHIP_OK;
    }
    if (!x || !y) return fail(ctx, GEOHIP_ERR_ARG, "null coordinate array");
    if (ctx->mem == GEOHIP_MEM_DEVICE) {
        if (!aligned16(x) || !aligned16(y)) return fail(ctx, GEOHIP_ERR_ARG, "device x/y must be 16-byte aligned");
        *dx = x;
        *dy = y;
        return GEOHIP_OK;
    }
    int rc = ensure(ctx, sx, n * 8);
    if (!rc) rc = ensure(ctx, sy, n * 8);
    if (rc) return rc;
    // the device buffers may still be read by work queued earlier on ctx->stream (the copy
    // stream does not follow it): order the copies after it
    hipEvent_t prior = nullptr;
    HIPCHK(hipEventCreateWithFlags(&prior, hipEventDisableTiming));
    hipError_t e = hipEventRecord(prior, ctx->stream);
    if (e == hipSuccess) e = stage_init(ctx) ? hipErrorUnknown : hipStreamWaitEvent(ctx->cstream, prior, 0);
    hipEventDestroy(prior);
    if (e != hipSuccess) return hip_fail(ctx, e, "staging order");
    rc = host_stage(ctx, x, y, n, B<double>(ctx, sx), B<double>(ctx, sy),
                    [](uint64_t, uint64_t, uint64_t, hipEvent_t) { return GEOHIP_OK; });
    if (rc) return rc;
    *dx = B<double>(ctx, sx);
    *dy = B<double>(ctx, sy);
    return GEOHIP_OK;
}

int plan_or_fail(geohip_ctx* ctx, const geohip_grid* grid, double qx, double qy, double r, PointPlan* plan) {
    if (!grid) return fail(ctx, GEOHIP_ERR_ARG, "null grid");
    const double q[3] = {qx, qy, r};
    if (ctx->plan_valid && memcmp(&ctx->plan_grid, grid, sizeof(geohip_grid)) == 0 && memcmp(ctx->plan_q, q, sizeof q) == 0) {
        *plan = ctx->plan;  // bitwise-identical inputs: the same plan
        return GEOHIP_OK;
    }
    std::string err;
    int rc = plan_point(*grid, qx, qy, r, plan, nullptr, nullptr, &err);
    if (rc) return fail(ctx, rc, err);
    ctx->plan_valid = true;
    memcpy(&ctx->plan_grid, grid, sizeof(geohip_grid));
    memcpy(ctx->plan_q, q, sizeof q);
    ctx->plan = *plan;
    return GEOHIP_OK;
}

KnnArgs make_knn_args(const PointPlan& plan, uint32_t k, double qx, double qy) {
    KnnArgs a;
    memset(&a, 0, sizeof a);
    for (int i = 0; i < plan.nu; i++) a.u[i] = plan.u[i];
    a.nu = plan.nu;
    a.k = k;
    a.qx = qx;
    a.qy = qy;
    // distance histogram: 32 octaves below 2^e_top, where every candidate distance is < 2^(e_top-1)
    double ex = 0.0, ey = 0.0;
    for (int i = 0; i < plan.nu; i++) {
        const Box& b = plan.u[i];
        ex = std::max(ex, std::max(std::fabs(b.xlo - qx), std::fabs(b.xhi - qx)));
        ey = std::max(ey, std::max(std::fabs(b.ylo - qy), std::fabs(b.yhi - qy)));
    }
    const double dmax = std::sqrt(ex * ex + ey * ey);
    int e_top = 1024;
    if (std::isfinite(dmax) && dmax > 0) e_top = std::ilogb(dmax) + 2;
    int E0 = e_top - 32 + 1023;
    if (E0 < 0) E0 = 0;
    if (E0 > 2047 - 32) E0 = 2047 - 32;
    a.hist_base = E0 << 4;
    return a;
}

RangeArgs make_range_args(const PointPlan& plan, double qx, double qy, double r) {
    RangeArgs a;
    memset(&a, 0, sizeof a);
    for (int i = 0; i < plan.ng; i++) a.g[i] = plan.g[i];
    a.ng = plan.ng;
    a.c = plan.c;
    a.nc = plan.nc;
    a.qx = qx;
    a.qy = qy;
    a.r = r;
    // squared screens for the candidate cells (see device_common.h): a 2^-40 margin
    pp_screen_bounds(r, &a.r2lo, &a.r2hi);
    return a;
}

// scratch that must start zeroed (the final kernel re-zeroes it after each use)
int ensure_zeroed(geohip_ctx* ctx, Slot s, size_t bytes);

// kNN enqueue shared by the sync and async forms.
int knn_enqueue(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                double qx, double qy, double r, uint32_t k, double* out_d, unsigned* out_i, unsigned* out_cnt) {
    if (k == 0) return fail(ctx, GEOHIP_ERR_ARG, "k must be > 0");
    if (n >= 0xffffffffull) return fail(ctx, GEOHIP_ERR_UNSUPPORTED, "window larger than 2^32-1 points");
    PointPlan plan;
    int rc = plan_or_fail(ctx, grid, qx, qy, r, &plan);
    if (rc) return rc;
    const double *dx, *dy;
    rc = stage_xy(ctx, x, y, n, S_X, S_Y, &dx, &dy);
    if (rc) return rc;
    // k beyond the one-pass selection: candidates, radix select and sort (any k)
    if (k > GEOHIP_KNN_MAX_K) return knn_pp_large_impl(ctx, plan, dx, dy, n, qx, qy, k, out_d, out_i, out_cnt);
    KnnArgs a = make_knn_args(plan, k, qx, qy);
    unsigned nb = 0;
    uint64_t ch = 0;
    knn_pass_geometry(n, &nb, &ch);
    const size_t ents = knn_pass_list_entries(nb ? nb : 1);
    rc = ensure(ctx, S_PART_D, ents * 8);
    if (!rc) rc = ensure(ctx, S_PART_I, ents * 4);
    if (!rc) rc = ensure(ctx, S_SPILL_D, n * 8);  // worst case: every point survives
    if (!rc) rc = ensure(ctx, S_SPILL_I, n * 4);
    if (!rc) rc = ensure_zeroed(ctx, S_SPILL_CNT, kKnnCounterBytes);
    if (rc) return rc;
    hipEvent_t e0, e1;
    kernel_step_events(ctx, &e0, &e1);
    hipError_t e = launch_knn_pass(dx, dy, n, a, B<unsigned long long>(ctx, S_PART_D), B<unsigned>(ctx, S_PART_I),
                                   B<unsigned long long>(ctx, S_SPILL_D), B<unsigned>(ctx, S_SPILL_I),
                                   B<unsigned>(ctx, S_SPILL_CNT), out_d, out_i, out_cnt, ctx->stream, e0, e1);
    if (e != hipSuccess) return hip_fail(ctx, e, "knn launch");
    return GEOHIP_OK;
}

// kNN of a host window staged in chunks (GEOHIP_MEM_HOST, >= 2 chunks): each chunk's pass
// starts as soon as its DMA has landed (overlapping the copies of the later chunks), the chunk
// lists are rebased to window indices and merged -- the k smallest of the union of per-chunk k
// smallest is the window's k smallest (PointPointKNNQuery.java:125-191's windowAll merge).
int knn_host_pipelined(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                       double qx, double qy, double r, uint32_t k, double* out_d, unsigned* out_i, unsigned* out_cnt,
                       bool* done) {
    *done = false;
    const uint64_t nch = (n + kStagePts - 1) / kStagePts;
    if (ctx->mem != GEOHIP_MEM_HOST || nch < 2 || n >= 0xffffffffull || k == 0 || k > GEOHIP_KNN_MAX_K ||
        (k > 256 && nch * k > 8192) || nch > 4096)
        return GEOHIP_OK;  // the one-pass path
    if (!x || !y) return fail(ctx, GEOHIP_ERR_ARG, "null coordinate array");
    PointPlan plan;
    int rc = plan_or_fail(ctx, grid, qx, qy, r, &plan);
    if (rc) return rc;
    KnnArgs a = make_knn_args(plan, k, qx, qy);
    unsigned nb = 0;
    uint64_t chp = 0;
    knn_pass_geometry(kStagePts, &nb, &chp);
    const size_t ents = knn_pass_list_entries(nb ? nb : 1);
    rc = ensure(ctx, S_X, n * 8);
    if (!rc) rc = ensure(ctx, S_Y, n * 8);
    if (!rc) rc = ensure(ctx, S_PART_D, ents * 8);
    if (!rc) rc = ensure(ctx, S_PART_I, ents * 4);
    if (!rc) rc = ensure(ctx, S_SPILL_D, kStagePts * 8);
    if (!rc) rc = ensure(ctx, S_SPILL_I, kStagePts * 4);
    if (!rc) rc = ensure_zeroed(ctx, S_SPILL_CNT, kKnnCounterBytes);
    if (!rc) rc = ensure(ctx, S_QX, nch * k * 8);   // chunk lists (distance bits)
    if (!rc) rc = ensure(ctx, S_QY, nch * k * 4);   // chunk lists (indices)
    if (!rc) rc = ensure(ctx, S_UCNT, nch * 4);     // chunk list counts
    if (!rc) rc = stage_init(ctx);
    if (rc) return rc;
    hipEvent_t prior = nullptr;
    HIPCHK(hipEventCreateWithFlags(&prior, hipEventDisableTiming));
    hipError_t e = hipEventRecord(prior, ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(ctx->cstream, prior, 0);
    hipEventDestroy(prior);
    if (e != hipSuccess) return hip_fail(ctx, e, "staging order");
    double* dx = B<double>(ctx, S_X);
    double* dy = B<double>(ctx, S_Y);
    double* ld = B<double>(ctx, S_QX);
    unsigned* li = B<unsigned>(ctx, S_QY);
    unsigned* lc = B<unsigned>(ctx, S_UCNT);
    hipEvent_t e0, e1;
    timing_events(ctx, &e0, &e1);  // timed: the first chunk's pass to the merge
    rc = host_stage(ctx, x, y, n, dx, dy, [&](uint64_t c, uint64_t b, uint64_t m, hipEvent_t ev) -> int {
        HIPCHK(hipStreamWaitEvent(ctx->stream, ev, 0));
        hipError_t le = launch_knn_pass(dx + b, dy + b, m, a, B<unsigned long long>(ctx, S_PART_D),
                                        B<unsigned>(ctx, S_PART_I), B<unsigned long long>(ctx, S_SPILL_D),
                                        B<unsigned>(ctx, S_SPILL_I), B<unsigned>(ctx, S_SPILL_CNT), ld + c * k,
                                        li + c * k, lc + c, ctx->stream, c == 0 ? e0 : nullptr, nullptr);
        if (le != hipSuccess) return hip_fail(ctx, le, "knn chunk launch");
        return GEOHIP_OK;
    });
    if (rc) return rc;
    e = launch_knn_rebase(li, (unsigned)nch, k, kStagePts, ctx->stream);
    if (e == hipSuccess)
        e = launch_knn_merge(reinterpret_cast<const unsigned long long*>(ld), li, (unsigned)nch, k, k, out_d, out_i,
                             out_cnt, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "knn merge launch");
    if (e1) HIPCHK(hipEventRecord(e1, ctx->stream));
    *done = true;
    return GEOHIP_OK;
}

int range_enqueue(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n, double qx,
                  double qy, double r, int approximate, unsigned* out, uint64_t cap, uint64_t* total,
                  uint32_t point_base = 0) {
    if (n >= 0xffffffffull) return fail(ctx, GEOHIP_ERR_UNSUPPORTED, "window larger than 2^32-1 points");
    PointPlan plan;
    int rc = plan_or_fail(ctx, grid, qx, qy, r, &plan);
    if (rc) return rc;
    RangeArgs a = make_range_args(plan, qx, qy, r);
    a.point_base = point_base;
    const double *dx, *dy;
    rc = stage_xy(ctx, x, y, n, S_X, S_Y, &dx, &dy);
    if (rc) return rc;
    const uint64_t units = (n + kRangeUnitPts - 1) / kRangeUnitPts;
    rc = ensure(ctx, S_MASK, units * 16 * 8);
    if (!rc) rc = ensure(ctx, S_UCNT, units * 4);
    if (!rc) rc = ensure(ctx, S_OFFS, units * 8);
    if (rc) return rc;
    // fused pass: 256 status words + the arrival ticket (zeroed once; re-armed by each launch)
    RangeLb lb;
    rc = range_lookback(ctx, &lb);
    if (rc) return rc;
    hipEvent_t e0, e1;
    if (ctx->range_order == GEOHIP_ORDER_ANY) {  // one kernel, no look-back, no ordered emission
        kernel_step_events(ctx, &e0, &e1);
        hipError_t e = launch_range_set(dx, dy, n, a, approximate, lb.set, total, out, cap, (unsigned)ctx->cus,
                                        ctx->stream, e0, e1);
        if (e != hipSuccess) return hip_fail(ctx, e, "range launch");
        return GEOHIP_OK;
    }
    if (range_is_one_kernel(n)) kernel_step_events(ctx, &e0, &e1);
    else timing_events(ctx, &e0, &e1);
    hipError_t e = launch_range(dx, dy, n, a, approximate, B<unsigned long long>(ctx, S_MASK), B<unsigned>(ctx, S_UCNT),
                                B<uint64_t>(ctx, S_OFFS), total, out, cap, ctx->stream, e0, e1, lb.status, lb.ticket,
                                lb.epoch, lb.fault, lb.spins, lb.inject);
    if (e != hipSuccess) return hip_fail(ctx, e, "range launch");
    return GEOHIP_OK;
}

// kNN (k) and range of the same point over one window: one fused pass when the window fits
// (knn_pass_fuses_range), else the two passes back to back.
int knn_range_enqueue(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                      double qx, double qy, double r, uint32_t k, int approximate, double* kd, unsigned* ki,
                      unsigned* kcnt, unsigned* rout, uint64_t rcap, uint64_t* rtotal) {
    if (k == 0) return fail(ctx, GEOHIP_ERR_ARG, "k must be > 0");
    PointPlan plan;
    int rc = plan_or_fail(ctx, grid, qx, qy, r, &plan);
    if (rc) return rc;
    if (n == 0 || plan.nu == 0 || !knn_pass_fuses_range(n) || k > GEOHIP_KNN_MAX_K) {
        rc = knn_enqueue(ctx, grid, x, y, n, qx, qy, r, k, kd, ki, kcnt);
        if (!rc) rc = range_enqueue(ctx, grid, x, y, n, qx, qy, r, approximate, rout, rcap, rtotal);
        return rc;
    }
    KnnArgs a = make_knn_args(plan, k, qx, qy);
    const double *dx, *dy;
    rc = stage_xy(ctx, x, y, n, S_X, S_Y, &dx, &dy);
    if (rc) return rc;
    unsigned nb = 0;
    uint64_t ch = 0;
    knn_pass_geometry(n, &nb, &ch);
    const size_t ents = knn_pass_list_entries(nb ? nb : 1);
    rc = ensure(ctx, S_PART_D, ents * 8);
    if (!rc) rc = ensure(ctx, S_PART_I, ents * 4);
    if (!rc) rc = ensure(ctx, S_SPILL_D, n * 8);
    if (!rc) rc = ensure(ctx, S_SPILL_I, n * 4);
    if (!rc) rc = ensure_zeroed(ctx, S_SPILL_CNT, kKnnCounterBytes);
    RangeLb lb;
    if (!rc) rc = range_lookback(ctx, &lb);
    if (rc) return rc;
    PassRangeIo rio;
    memset(&rio, 0, sizeof rio);
    rio.a = make_range_args(plan, qx, qy, r);
    rio.approximate = approximate;
    rio.status = lb.status;
    rio.epoch = lb.epoch;
    rio.fault = lb.fault;
    rio.spin_limit = lb.spins;
    rio.inject = lb.inject;
    rio.out = rout;
    rio.cap = rcap;
    rio.total = rtotal;
    rio.unordered = ctx->range_order == GEOHIP_ORDER_ANY ? 1 : 0;  // the set, no look-back
    rio.cursor = lb.set.word;
    hipEvent_t e0, e1;
    kernel_step_events(ctx, &e0, &e1);
    hipError_t e = launch_knn_pass(dx, dy, n, a, B<unsigned long long>(ctx, S_PART_D), B<unsigned>(ctx, S_PART_I),
                                   B<unsigned long long>(ctx, S_SPILL_D), B<unsigned>(ctx, S_SPILL_I),
                                   B<unsigned>(ctx, S_SPILL_CNT), kd, ki, kcnt, ctx->stream, e0, e1, nullptr, 0, &rio);
    if (e != hipSuccess) return hip_fail(ctx, e, "knn+range launch");
    return GEOHIP_OK;
}

}  // namespace

extern "C" {

const char* geohip_version(void) { return "geohip 0.2 (gfx950)"; }
int geohip_abi_version(void) { return GEOHIP_ABI_VERSION; }

int geohip_device_count(int* out_count) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) {
        (void)hipGetLastError();
        c = 0;
    }
    if (out_count) *out_count = c;
    return GEOHIP_OK;
}

int geohip_ctx_create(uint32_t device_mask, geohip_ctx** out_ctx) {
    if (!out_ctx) return GEOHIP_ERR_ARG;
    *out_ctx = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return GEOHIP_ERR_DEVICE;
    }
    int dev = 0;
    if (device_mask == 0) {
        if (hipGetDevice(&dev) != hipSuccess) return GEOHIP_ERR_DEVICE;
    } else {
        if (device_mask & (device_mask - 1)) return GEOHIP_ERR_UNSUPPORTED;  // one device per ctx
        dev = __builtin_ctz(device_mask);
        if (dev >= ndev) return GEOHIP_ERR_ARG;
    }
    geohip_ctx* ctx = new geohip_ctx();
    ctx->device = dev;
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0) ctx->cus = ncu;
    }
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&ctx->pinned, 64, hipHostMallocDefault) != hipSuccess) {
        delete ctx;
        return GEOHIP_ERR_DEVICE;
    }
    ctx->stream = ctx->own;
    *out_ctx = ctx;
    return GEOHIP_OK;
}

int geohip_ctx_destroy(geohip_ctx* ctx) {
    if (ctx) ppoly_cache_drop(ctx);
    if (ctx) knn_poly_cache_drop(ctx);
    if (!ctx) return GEOHIP_ERR_ARG;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    for (int s = 0; s < S_COUNT; s++)
        if (ctx->buf[s]) hipFree(ctx->buf[s]);
    for (auto& p : ctx->pending) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (auto ev : ctx->pool) hipEventDestroy(ev);
    if (ctx->pinned) hipHostFree(ctx->pinned);
    if (ctx->cstream) hipStreamSynchronize(ctx->cstream);
    for (int k = 0; k < 2; k++) {
        if (ctx->stg[k]) hipHostFree(ctx->stg[k]);
        if (ctx->stg_ev[k]) hipEventDestroy(ctx->stg_ev[k]);
    }
    if (ctx->cstream) hipStreamDestroy(ctx->cstream);
    if (ctx->switch_ev) hipEventDestroy(ctx->switch_ev);
    if (ctx->own) hipStreamDestroy(ctx->own);
    delete ctx;
    return GEOHIP_OK;
}

const char* geohip_last_error(const geohip_ctx* ctx) { return ctx ? ctx->err.c_str() : "null ctx"; }

int geohip_ctx_set_mem(geohip_ctx* ctx, int mem_kind) {
    if (!ctx || (mem_kind != GEOHIP_MEM_HOST && mem_kind != GEOHIP_MEM_DEVICE)) return GEOHIP_ERR_ARG;
    ctx->mem = mem_kind;
    return GEOHIP_OK;
}

// Rebinding the ctx to another stream: the ctx's scratch (block lists, spill counter, look-back
// words, staging slots) is shared by every call, so work still queued on the old stream must
// finish before the new stream's kernels touch it -- the new stream waits on an event recorded
// on the old one.
static int switch_stream(geohip_ctx* ctx, hipStream_t next) {
    if (next == ctx->stream) return GEOHIP_OK;
    int rc = begin(ctx);
    if (rc) return rc;
    if (!ctx->switch_ev) HIPCHK(hipEventCreateWithFlags(&ctx->switch_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ctx->switch_ev, ctx->stream));
    HIPCHK(hipStreamWaitEvent(next, ctx->switch_ev, 0));
    ctx->stream = next;
    return GEOHIP_OK;
}

int geohip_ctx_set_stream(geohip_ctx* ctx, void* hip_stream) {
    if (!ctx) return GEOHIP_ERR_ARG;
    return switch_stream(ctx, (hipStream_t)hip_stream);  // NULL: the HIP null stream (PyTorch's default)
}

int geohip_ctx_reset_stream(geohip_ctx* ctx) {
    if (!ctx) return GEOHIP_ERR_ARG;
    return switch_stream(ctx, ctx->own);
}

void* geohip_ctx_stream(geohip_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int geohip_ctx_set_range_order(geohip_ctx* ctx, int order) {
    if (!ctx) return GEOHIP_ERR_ARG;
    if (order != GEOHIP_ORDER_ASCENDING && order != GEOHIP_ORDER_ANY)
        return fail(ctx, GEOHIP_ERR_ARG, "range order must be GEOHIP_ORDER_ASCENDING or GEOHIP_ORDER_ANY");
    ctx->range_order = order;
    return GEOHIP_OK;
}

int geohip_ctx_set_timing(geohip_ctx* ctx, int enable) {
    if (!ctx) return GEOHIP_ERR_ARG;
    ctx->timing = enable != 0;
    return GEOHIP_OK;
}

int geohip_ctx_timing(geohip_ctx* ctx, double* total_ms, uint64_t* launches, int reset) {
    int rc = begin(ctx);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (auto& p : ctx->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            if (p.kind != 1) {
                ctx->acc_ms += ms;
                ctx->launches++;
            }
            if (p.kind != 0) {
                ctx->kern_ms += ms;
                ctx->kernels++;
            }
        } else {
            (void)hipGetLastError();
        }
        ctx->pool.push_back(p.a);
        ctx->pool.push_back(p.b);
    }
    ctx->pending.clear();
    if (total_ms) *total_ms = ctx->acc_ms;
    if (launches) *launches = ctx->launches;
    if (reset) {
        ctx->acc_ms = 0.0;
        ctx->launches = 0;
        ctx->kern_ms = 0.0;
        ctx->kernels = 0;
    }
    return GEOHIP_OK;
}

int geohip_ctx_sync(geohip_ctx* ctx) {
    int rc = begin(ctx);
    if (rc) return rc;
    rc = queue_fault_read(ctx);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return report_faults(ctx);
}

// Test knob: while on, the range look-back waits (range_fused, the kNN pass's fused range) wait
// for an epoch no block publishes and give up after 4096 polls -- the fault path, exercised.
int geohip_debug_lookback_inject(geohip_ctx* ctx, int on) {
    if (!ctx) return GEOHIP_ERR_ARG;
    ctx->lb_inject = on != 0;
    return GEOHIP_OK;
}

int geohip_ctx_timing_kernels(geohip_ctx* ctx, double* step_ms, uint64_t* steps, double* kernel_ms,
                              uint64_t* kernels, int reset) {
    double km = 0.0;
    uint64_t kn = 0;
    int rc = geohip_ctx_timing(ctx, step_ms, steps, 0);
    if (rc) return rc;
    km = ctx->kern_ms;
    kn = ctx->kernels;
    if (kernel_ms) *kernel_ms = km;
    if (kernels) *kernels = kn;
    if (reset) geohip_ctx_timing(ctx, nullptr, nullptr, 1);
    return GEOHIP_OK;
}

int geohip_range_pp(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                    double qx, double qy, double r, int approximate, uint32_t* out_idx, uint64_t cap,
                    uint64_t* out_count) {
    return geohip_range_pp_pane(ctx, grid, x, y, n, 0u, qx, qy, r, approximate, out_idx, cap, out_count);
}

int geohip_range_pp_pane(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                         uint32_t point_base, double qx, double qy, double r, int approximate, uint32_t* out_idx,
                         uint64_t cap, uint64_t* out_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (!out_count || (cap && !out_idx)) return fail(ctx, GEOHIP_ERR_ARG, "null output");
    unsigned* out = nullptr;
    if (ctx->mem == GEOHIP_MEM_DEVICE) {
        out = out_idx;
    } else {
        rc = ensure(ctx, S_OUT_IDX, cap * 4);
        if (rc) return rc;
        out = B<unsigned>(ctx, S_OUT_IDX);
    }
    rc = ensure(ctx, S_TOTAL, 8);
    if (rc) return rc;
    rc = range_enqueue(ctx, grid, x, y, n, qx, qy, r, approximate, out, cap, B<uint64_t>(ctx, S_TOTAL), point_base);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(ctx->pinned, ctx->buf[S_TOTAL], 8, hipMemcpyDeviceToHost, ctx->stream));
    rc = queue_fault_read(ctx);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    rc = report_faults(ctx, kFaultLookback);
    if (rc) return rc;
    const uint64_t total = ctx->pinned[0];
    *out_count = total;
    if (ctx->mem == GEOHIP_MEM_HOST) {
        const uint64_t m = total < cap ? total : cap;
        if (m) HIPCHK(hipMemcpy(out_idx, out, m * 4, hipMemcpyDeviceToHost));
    }
    if (total > cap) return fail(ctx, GEOHIP_ERR_CAPACITY, "output capacity too small; *out_count = required");
    return GEOHIP_OK;
}

int geohip_range_pp_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                          double qx, double qy, double r, int approximate, uint32_t* out_idx, uint64_t cap,
                          uint64_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (!out_count_dev || (cap && !out_idx)) return fail(ctx, GEOHIP_ERR_ARG, "null output");
    return range_enqueue(ctx, grid, x, y, n, qx, qy, r, approximate, out_idx, cap, out_count_dev);
}

int geohip_knn_pp(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                  double qx, double qy, double r, uint32_t k, uint32_t* out_idx, double* out_dist,
                  uint32_t* out_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (!out_idx || !out_dist || !out_count) return fail(ctx, GEOHIP_ERR_ARG, "null output");
    double* od;
    unsigned* oi;
    if (ctx->mem == GEOHIP_MEM_DEVICE) {
        od = out_dist;
        oi = out_idx;
    } else {
        rc = ensure(ctx, S_OUT_D, (size_t)k * 8);
        if (!rc) rc = ensure(ctx, S_OUT_I, (size_t)k * 4);
        if (rc) return rc;
        od = B<double>(ctx, S_OUT_D);
        oi = B<unsigned>(ctx, S_OUT_I);
    }
    rc = ensure(ctx, S_OUT_CNT, 8);
    if (rc) return rc;
    bool done = false;
    rc = knn_host_pipelined(ctx, grid, x, y, n, qx, qy, r, k, od, oi, B<unsigned>(ctx, S_OUT_CNT), &done);
    if (!rc && !done) rc = knn_enqueue(ctx, grid, x, y, n, qx, qy, r, k, od, oi, B<unsigned>(ctx, S_OUT_CNT));
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(ctx->pinned, ctx->buf[S_OUT_CNT], 4, hipMemcpyDeviceToHost, ctx->stream));
    if (ctx->mem == GEOHIP_MEM_HOST) {
        HIPCHK(hipMemcpyAsync(out_dist, od, (size_t)k * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(out_idx, oi, (size_t)k * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    *out_count = (uint32_t)(ctx->pinned[0] & 0xffffffffu);
    return GEOHIP_OK;
}

int geohip_knn_pp_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                        double qx, double qy, double r, uint32_t k, uint32_t* out_idx, double* out_dist,
                        uint32_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (!out_idx || !out_dist || !out_count_dev) return fail(ctx, GEOHIP_ERR_ARG, "null output");
    return knn_enqueue(ctx, grid, x, y, n, qx, qy, r, k, out_dist, out_idx, out_count_dev);
}

int geohip_format_points_csv(geohip_ctx* ctx, const geohip_csv_out_spec* spec, const double* x, const double* y,
                             uint64_t n, const int64_t* ts, const uint8_t* oid_text, const uint64_t* oid_off,
                             const uint32_t* idx, uint64_t m, uint8_t* out, uint64_t cap, uint64_t* out_len,
                             uint64_t* rec_off) {
    int rc = begin(ctx);
    if (rc) return rc;
    return format_csv_impl(ctx, spec, x, y, n, ts, oid_text, oid_off, idx, m, out, cap, out_len, rec_off);
}

int geohip_format_points(geohip_ctx* ctx, const geohip_text_out_spec* spec, const double* x, const double* y,
                         uint64_t n, const int64_t* ts, const uint8_t* oid_text, const uint64_t* oid_off,
                         const uint32_t* idx, uint64_t m, uint8_t* out, uint64_t cap, uint64_t* out_len,
                         uint64_t* rec_off) {
    int rc = begin(ctx);
    if (rc) return rc;
    return format_points_impl(ctx, spec, x, y, n, ts, oid_text, oid_off, idx, m, out, cap, out_len, rec_off);
}

int geohip_band_pack_async(geohip_ctx* ctx, const geohip_grid* grid_data, int32_t nb, uint32_t world,
                           const double* x, const double* y, uint64_t n, int64_t base, double* out_x,
                           double* out_y, int64_t* out_idx, uint64_t* out_counts_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    return band_pack_impl(ctx, grid_data, nb, world, x, y, n, base, out_x, out_y, out_idx, out_counts_dev);
}

int geohip_band_pack_query_async(geohip_ctx* ctx, const geohip_grid* grid_data, int32_t nb, uint32_t world, double qx,
                                 double qy, double r, const double* x, const double* y, uint64_t n, int64_t base,
                                 double* out_x, double* out_y, int64_t* out_idx, uint64_t* out_counts_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    PointPlan plan;
    rc = plan_or_fail(ctx, grid_data, qx, qy, r, &plan);
    if (rc) return rc;
    return band_pack_impl(ctx, grid_data, nb, world, x, y, n, base, out_x, out_y, out_idx, out_counts_dev, &plan);
}

int geohip_knn_merge_async(geohip_ctx* ctx, const double* dist, const uint32_t* idx, uint32_t nlists,
                           uint32_t list_len, uint32_t k, uint32_t* out_idx, double* out_dist,
                           uint32_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (k == 0) return fail(ctx, GEOHIP_ERR_ARG, "k must be > 0");
    if (!dist || !idx || !out_idx || !out_dist || !out_count_dev) return fail(ctx, GEOHIP_ERR_ARG, "null pointer");
    if (k > 256 && (uint64_t)nlists * list_len > 8192)  // beyond one workgroup's LDS sort
        return knn_merge_large_impl(ctx, reinterpret_cast<const unsigned long long*>(dist), idx, nlists, list_len, k,
                                    out_dist, out_idx, out_count_dev);
    hipError_t e = launch_knn_merge(reinterpret_cast<const unsigned long long*>(dist), idx, nlists, list_len, k,
                                    out_dist, out_idx, out_count_dev, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "knn merge launch");
    return GEOHIP_OK;
}

int geohip_knn_merge_panes_async(geohip_ctx* ctx, const double* ring_dist, const uint32_t* ring_idx, uint32_t list_len,
                                 const uint32_t* slots, const uint64_t* offsets, uint32_t npanes, uint32_t k,
                                 uint32_t* out_idx, double* out_dist, uint32_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (k == 0 || list_len == 0) return fail(ctx, GEOHIP_ERR_ARG, "k and list_len must be > 0");
    if (npanes == 0 || npanes > kMaxPanes) return fail(ctx, GEOHIP_ERR_UNSUPPORTED, "1..16 panes per window");
    if (!ring_dist || !ring_idx || !slots || !offsets || !out_idx || !out_dist || !out_count_dev)
        return fail(ctx, GEOHIP_ERR_ARG, "null pointer");
    if ((uint64_t)npanes * list_len > (1ull << 30)) return fail(ctx, GEOHIP_ERR_UNSUPPORTED, "panes too long");
    PaneMerge pm;
    memset(&pm, 0, sizeof pm);
    for (uint32_t b = 0; b < npanes; b++) {
        if (offsets[b] >= 0xffffffffull) return fail(ctx, GEOHIP_ERR_UNSUPPORTED, "window beyond 2^32-1 points");
        pm.slot[b] = slots[b];
        pm.off[b] = (unsigned)offsets[b];
    }
    pm.n = npanes;
    pm.list_len = list_len;
    pm.k = k;
    hipEvent_t ev0, ev1;
    timed_pair(ctx, &ev0, &ev1, 1);  // one kernel of the pane step (the pane's scan is the other)
    hipError_t e = launch_knn_merge_panes(reinterpret_cast<const unsigned long long*>(ring_dist), ring_idx, pm,
                                          out_dist, out_idx, out_count_dev, ctx->stream, ev0, ev1);
    if (e != hipSuccess) return hip_fail(ctx, e, "pane merge launch");
    return GEOHIP_OK;
}

int geohip_knn_range_pp(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                        double qx, double qy, double r, uint32_t k, int approximate, uint32_t* knn_idx,
                        double* knn_dist, uint32_t* knn_count, uint32_t* range_idx, uint64_t range_cap,
                        uint64_t* range_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (!knn_idx || !knn_dist || !knn_count || !range_count || (range_cap && !range_idx))
        return fail(ctx, GEOHIP_ERR_ARG, "null output");
    double* od;
    unsigned *oi, *ro;
    if (ctx->mem == GEOHIP_MEM_DEVICE) {
        od = knn_dist;
        oi = knn_idx;
        ro = range_idx;
    } else {
        rc = ensure(ctx, S_OUT_D, (size_t)k * 8);
        if (!rc) rc = ensure(ctx, S_OUT_I, (size_t)k * 4);
        if (!rc) rc = ensure(ctx, S_OUT_IDX, range_cap * 4);
        if (rc) return rc;
        od = B<double>(ctx, S_OUT_D);
        oi = B<unsigned>(ctx, S_OUT_I);
        ro = B<unsigned>(ctx, S_OUT_IDX);
    }
    rc = ensure(ctx, S_OUT_CNT, 8);
    if (!rc) rc = ensure(ctx, S_TOTAL, 8);
    if (rc) return rc;
    rc = knn_range_enqueue(ctx, grid, x, y, n, qx, qy, r, k, approximate, od, oi, B<unsigned>(ctx, S_OUT_CNT), ro,
                           range_cap, B<uint64_t>(ctx, S_TOTAL));
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(ctx->pinned, ctx->buf[S_OUT_CNT], 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->pinned + 1, ctx->buf[S_TOTAL], 8, hipMemcpyDeviceToHost, ctx->stream));
    if (ctx->mem == GEOHIP_MEM_HOST) {
        HIPCHK(hipMemcpyAsync(knn_dist, od, (size_t)k * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(knn_idx, oi, (size_t)k * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    rc = queue_fault_read(ctx);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    rc = report_faults(ctx, kFaultLookback);
    if (rc) return rc;
    *knn_count = (uint32_t)(ctx->pinned[0] & 0xffffffffu);
    const uint64_t total = ctx->pinned[1];
    *range_count = total;
    if (ctx->mem == GEOHIP_MEM_HOST) {
        const uint64_t m = total < range_cap ? total : range_cap;
        if (m) HIPCHK(hipMemcpy(range_idx, ro, m * 4, hipMemcpyDeviceToHost));
    }
    if (total > range_cap) return fail(ctx, GEOHIP_ERR_CAPACITY, "range capacity too small; *range_count = required");
    return GEOHIP_OK;
}

int geohip_knn_range_pp_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                              double qx, double qy, double r, uint32_t k, int approximate, uint32_t* knn_idx,
                              double* knn_dist, uint32_t* knn_count_dev, uint32_t* range_idx, uint64_t range_cap,
                              uint64_t* range_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (!knn_idx || !knn_dist || !knn_count_dev || !range_count_dev || (range_cap && !range_idx))
        return fail(ctx, GEOHIP_ERR_ARG, "null output");
    return knn_range_enqueue(ctx, grid, x, y, n, qx, qy, r, k, approximate, knn_dist, knn_idx, knn_count_dev, range_idx,
                             range_cap, range_count_dev);
}

int geohip_join_pp(geohip_ctx* ctx, const geohip_grid* grid_data, const geohip_grid* grid_query, const double* dx,
                   const double* dy, uint64_t nd, const double* qx, const double* qy, uint64_t nq, double r,
                   int approximate, uint32_t* out_pairs, uint64_t cap, uint64_t* out_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    return join_pp_impl(ctx, grid_data, grid_query, dx, dy, nd, qx, qy, nq, r, approximate, out_pairs, cap, out_count,
                        false);
}

int geohip_join_pp_count_only(geohip_ctx* ctx, const geohip_grid* grid_data, const geohip_grid* grid_query,
                              const double* dx, const double* dy, uint64_t nd, const double* qx, const double* qy,
                              uint64_t nq, double r, int approximate, uint64_t* out_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    return join_pp_impl(ctx, grid_data, grid_query, dx, dy, nd, qx, qy, nq, r, approximate, nullptr, 0, out_count,
                        true);
}

int geohip_join_pp_async(geohip_ctx* ctx, const geohip_grid* grid_data, const geohip_grid* grid_query,
                         const double* dx, const double* dy, uint64_t nd, const double* qx, const double* qy,
                         uint64_t nq, double r, int approximate, uint32_t* out_pairs, uint64_t cap,
                         uint64_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (!out_count_dev || (cap && !out_pairs)) return fail(ctx, GEOHIP_ERR_ARG, "null output");
    return join_pp_impl(ctx, grid_data, grid_query, dx, dy, nd, qx, qy, nq, r, approximate, out_pairs, cap, nullptr,
                        false, out_count_dev);
}

int geohip_range_ppoly_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                             const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx, const double* vy,
                             uint64_t nv, uint32_t npoly, double r, int approximate, uint32_t* out_pairs, uint64_t cap,
                             uint64_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (!out_count_dev) return fail(ctx, GEOHIP_ERR_ARG, "null output");
    return ppoly_impl(ctx, grid, nullptr, 0, x, y, n, poly_rings, ring_off, vx, vy, nv, npoly, r, approximate, out_pairs,
                      cap, nullptr, 0, out_count_dev);
}

int geohip_range_ppoly_pane_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                                  uint64_t n, uint32_t point_base, const uint32_t* poly_rings, const uint32_t* ring_off,
                                  const double* vx, const double* vy, uint64_t nv, uint32_t npoly, double r,
                                  int approximate, uint32_t* out_pairs, uint64_t cap, uint64_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (!out_count_dev) return fail(ctx, GEOHIP_ERR_ARG, "null output");
    return ppoly_impl(ctx, grid, nullptr, 0, x, y, n, poly_rings, ring_off, vx, vy, nv, npoly, r, approximate, out_pairs,
                      cap, nullptr, point_base, out_count_dev);
}

int geohip_join_ppoly_async(geohip_ctx* ctx, const geohip_grid* grid_points, const geohip_grid* grid_query,
                            const double* x, const double* y, uint64_t n, const uint32_t* poly_rings,
                            const uint32_t* ring_off, const double* vx, const double* vy, uint64_t nv, uint32_t npoly,
                            double r, int approximate, uint32_t* out_pairs, uint64_t cap, uint64_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    if (!out_count_dev) return fail(ctx, GEOHIP_ERR_ARG, "null output");
    return ppoly_impl(ctx, grid_points, grid_query, 1, x, y, n, poly_rings, ring_off, vx, vy, nv, npoly, r, approximate,
                      out_pairs, cap, nullptr, 0, out_count_dev);
}

int geohip_range_ppoly(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                       const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx, const double* vy,
                       uint64_t nv, uint32_t npoly, double r, int approximate, uint32_t* out_pairs, uint64_t cap,
                       uint64_t* out_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    return ppoly_impl(ctx, grid, nullptr, 0, x, y, n, poly_rings, ring_off, vx, vy, nv, npoly, r, approximate, out_pairs,
                      cap, out_count);
}

int geohip_range_ppoly_pane(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                            uint32_t point_base, const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
                            const double* vy, uint64_t nv, uint32_t npoly, double r, int approximate,
                            uint32_t* out_pairs, uint64_t cap, uint64_t* out_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    return ppoly_impl(ctx, grid, nullptr, 0, x, y, n, poly_rings, ring_off, vx, vy, nv, npoly, r, approximate, out_pairs,
                      cap, out_count, point_base);
}

int geohip_join_ppoly(geohip_ctx* ctx, const geohip_grid* grid_points, const geohip_grid* grid_query, const double* x,
                      const double* y, uint64_t n, const uint32_t* poly_rings, const uint32_t* ring_off,
                      const double* vx, const double* vy, uint64_t nv, uint32_t npoly, double r, int approximate,
                      uint32_t* out_pairs, uint64_t cap, uint64_t* out_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    return ppoly_impl(ctx, grid_points, grid_query, 1, x, y, n, poly_rings, ring_off, vx, vy, nv, npoly, r, approximate,
                      out_pairs, cap, out_count);
}

int geohip_knn_ppoly(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                     const uint32_t* ring_off, uint32_t nring, const double* vx, const double* vy, uint64_t nv,
                     double r, uint32_t k, int approximate, uint32_t* out_idx, double* out_dist, uint32_t* out_count) {
    int rc = begin(ctx);
    if (rc) return rc;
    return knn_ppoly_impl(ctx, grid, x, y, n, ring_off, nring, vx, vy, nv, r, k, approximate, out_idx, out_dist,
                          out_count, false);
}

int geohip_knn_ppoly_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                           const uint32_t* ring_off, uint32_t nring, const double* vx, const double* vy, uint64_t nv,
                           double r, uint32_t k, int approximate, uint32_t* out_idx, double* out_dist,
                           uint32_t* out_count_dev) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (ctx->mem != GEOHIP_MEM_DEVICE) return fail(ctx, GEOHIP_ERR_ARG, "async forms need GEOHIP_MEM_DEVICE");
    return knn_ppoly_impl(ctx, grid, x, y, n, ring_off, nring, vx, vy, nv, r, k, approximate, out_idx, out_dist,
                          out_count_dev, true);
}

int geohip_plan_point(const geohip_grid* grid, double qx, double qy, double r, geohip_rect* g_rects, uint32_t* n_g,
                      geohip_rect* c_rect, uint32_t* n_c, int32_t* layers_g, int32_t* layers_c) {
    if (!grid || !n_g || !n_c) return GEOHIP_ERR_ARG;
    PointPlan plan;
    std::vector<geohip_rect> gr, cr;
    std::string err;
    int rc = plan_point(*grid, qx, qy, r, &plan, &gr, &cr, &err);
    if (rc) return rc;
    *n_g = (uint32_t)gr.size();
    *n_c = (uint32_t)cr.size();
    for (size_t i = 0; i < gr.size() && g_rects; i++) g_rects[i] = gr[i];
    if (c_rect && !cr.empty()) *c_rect = cr[0];
    if (layers_g) *layers_g = plan.layers_g;
    if (layers_c) *layers_c = plan.layers_c;
    return GEOHIP_OK;
}

int geohip_plan_cell(const geohip_grid* grid, double x, double y, int32_t* cx, int32_t* cy) {
    if (!grid || !cx || !cy) return GEOHIP_ERR_ARG;
    return cell_of(*grid, x, y, cx, cy);
}

int geohip_synth_uniform_async(geohip_ctx* ctx, double* x, double* y, uint64_t n, uint64_t base, uint64_t seed,
                               double min_x, double max_x, double min_y, double max_y) {
    int rc = begin(ctx);
    if (rc) return rc;
    hipError_t e = launch_synth_uniform(x, y, n, base, seed, min_x, max_x, min_y, max_y, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "synth launch");
    return GEOHIP_OK;
}

// Test hook (host only): classify points with the planner's exact boxes, exactly as the
// kernels do: out[i] = inG | inC << 1 | inU << 2.
static inline bool host_in_box(const Box& b, double x, double y) {
    bool bx = (x >= b.xlo) && (x <= b.xhi);
    bool by = (y >= b.ylo) && (y <= b.yhi);
    if (b.nan_x) bx = bx || (x != x);
    if (b.nan_y) by = by || (y != y);
    return bx && by;
}
int geohip_debug_classify(const geohip_grid* grid, double qx, double qy, double r, const double* x, const double* y,
                          uint64_t n, uint8_t* out) {
    if (!grid) return GEOHIP_ERR_ARG;
    PointPlan plan;
    std::string err;
    int rc = plan_point(*grid, qx, qy, r, &plan, nullptr, nullptr, &err);
    if (rc) return rc;
    for (uint64_t i = 0; i < n; i++) {
        bool g = false, u = false;
        for (int b = 0; b < plan.ng; b++) g = g || host_in_box(plan.g[b], x[i], y[i]);
        for (int b = 0; b < plan.nu; b++) u = u || host_in_box(plan.u[b], x[i], y[i]);
        const bool c = !g && plan.nc && host_in_box(plan.c, x[i], y[i]);
        out[i] = (uint8_t)(g | (c << 1) | (u << 2));
    }
    return GEOHIP_OK;
}

// Test hook (not part of the operator surface): fp64 primitive bits on the device.
int geohip_debug_selftest_fp64(geohip_ctx* ctx, const double* a, const double* b, uint64_t n, double* o_sqrt,
                               double* o_div, double* o_hypot, double* o_mulsub) {
    int rc = begin(ctx);
    if (rc) return rc;
    hipError_t e = launch_selftest_fp64(a, b, n, o_sqrt, o_div, o_hypot, o_mulsub, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "selftest launch");
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return GEOHIP_OK;
}

// Measurement hook: counters of the last kNN pass's final selection (entries gathered, spilled,
// kept at or below the k-th bin), read back after a synchronise.
int geohip_debug_knn_pass_stats(geohip_ctx* ctx, uint32_t* out3) {
    int rc = begin(ctx);
    if (rc) return rc;
    if (!ctx->buf[S_SPILL_CNT]) return fail(ctx, GEOHIP_ERR_ARG, "no kNN pass ran");
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(out3, B<char>(ctx, S_SPILL_CNT) + kKnnCounterBytes - 64, 12, hipMemcpyDeviceToHost));
    return GEOHIP_OK;
}

// Measurement hook: one kNN pass (device memory) with per-block phase timestamps (100 MHz):
// host[16 b + s], s = start, stream end, flush, stores drained, arrived; the last block also
// acquired, gathered, written.  *nblocks = blocks of the launch.
int geohip_debug_knn_pass_trace(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                                uint64_t n, double qx, double qy, double r, uint32_t k, int ablation, uint64_t* host,
                                uint64_t cap_words, unsigned* nblocks) {
    const bool with_range = ablation < 0;  // measurement of the fused kNN + range pass
    if (with_range) ablation = 0;
    int rc = begin(ctx);
    if (rc) return rc;
    PointPlan plan;
    rc = plan_or_fail(ctx, grid, qx, qy, r, &plan);
    if (rc) return rc;
    KnnArgs a = make_knn_args(plan, k, qx, qy);
    unsigned nb = 0;
    uint64_t ch = 0;
    knn_pass_geometry(n, &nb, &ch);
    if (cap_words < 16ull * nb) return fail(ctx, GEOHIP_ERR_CAPACITY, "trace buffer too small");
    const size_t ents = knn_pass_list_entries(nb ? nb : 1);
    rc = ensure(ctx, S_PART_D, ents * 8);
    if (!rc) rc = ensure(ctx, S_PART_I, ents * 4);
    if (!rc) rc = ensure(ctx, S_SPILL_D, n * 8);
    if (!rc) rc = ensure(ctx, S_SPILL_I, n * 4);
    if (!rc) rc = ensure_zeroed(ctx, S_SPILL_CNT, kKnnCounterBytes);
    if (!rc) rc = ensure(ctx, S_OUT_D, (size_t)k * 8);
    if (!rc) rc = ensure(ctx, S_OUT_I, (size_t)k * 4);
    if (!rc) rc = ensure(ctx, S_OUT_CNT, 8);
    if (!rc) rc = ensure(ctx, S_TRACE, 16ull * nb * 8);
    if (rc) return rc;
    unsigned long long* tr = B<unsigned long long>(ctx, S_TRACE);
    HIPCHK(hipMemsetAsync(tr, 0, 16ull * nb * 8, ctx->stream));
    PassRangeIo rio;
    memset(&rio, 0, sizeof rio);
    if (with_range) {
        RangeLb lb;
        rc = range_lookback(ctx, &lb);
        if (!rc) rc = ensure(ctx, S_OUT_IDX, n * 4);
        if (!rc) rc = ensure(ctx, S_TOTAL, 8);
        if (rc) return rc;
        rio.a = make_range_args(plan, qx, qy, r);
        rio.status = lb.status;
        rio.epoch = lb.epoch;
        rio.fault = lb.fault;
        rio.spin_limit = lb.spins;
        rio.inject = lb.inject;
        rio.out = B<unsigned>(ctx, S_OUT_IDX);
        rio.cap = n;
        rio.total = B<uint64_t>(ctx, S_TOTAL);
        rio.trace = tr;
    }
    hipError_t e = launch_knn_pass(x, y, n, a, B<unsigned long long>(ctx, S_PART_D), B<unsigned>(ctx, S_PART_I),
                                   B<unsigned long long>(ctx, S_SPILL_D), B<unsigned>(ctx, S_SPILL_I),
                                   B<unsigned>(ctx, S_SPILL_CNT), B<double>(ctx, S_OUT_D), B<unsigned>(ctx, S_OUT_I),
                                   B<unsigned>(ctx, S_OUT_CNT), ctx->stream, nullptr, nullptr, tr, ablation,
                                   with_range ? &rio : nullptr);
    if (e != hipSuccess) return hip_fail(ctx, e, "knn pass launch");
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(host, tr, 16ull * nb * 8, hipMemcpyDeviceToHost));
    *nblocks = nb;
    return GEOHIP_OK;
}

// Test hook: byte budget of this ctx's join hit masks (beyond it the write pass recomputes).
}  // extern "C"

// ------------------------------------------------------------------ shared with join/ppoly --
namespace geohip {
int ctx_fail(geohip_ctx* ctx, int code, const std::string& msg) { return fail(ctx, code, msg); }
int ctx_ensure(geohip_ctx* ctx, int slot, size_t bytes, void** out) {
    if (slot < 0 || S_J0 + slot > S_J27) return fail(ctx, GEOHIP_ERR_DEVICE, "internal: scratch slot out of range");
    int rc = ensure(ctx, (Slot)(S_J0 + slot), bytes);
    if (!rc) *out = ctx->buf[S_J0 + slot];
    return rc;
}
int ctx_ensure_zeroed(geohip_ctx* ctx, int slot, size_t bytes, void** out) {
    if (slot < 0 || S_J0 + slot > S_J27) return fail(ctx, GEOHIP_ERR_DEVICE, "internal: scratch slot out of range");
    int rc = ensure_zeroed(ctx, (Slot)(S_J0 + slot), bytes);
    if (!rc) *out = ctx->buf[S_J0 + slot];
    return rc;
}
int ctx_ensure_ingest(geohip_ctx* ctx, int slot, size_t bytes, void** out) {
    if (slot < 0 || S_I0 + slot >= S_COUNT) return fail(ctx, GEOHIP_ERR_DEVICE, "internal: scratch slot out of range");
    int rc = ensure(ctx, (Slot)(S_I0 + slot), bytes);
    if (!rc) *out = ctx->buf[S_I0 + slot];
    return rc;
}
int ctx_ensure_ingest_zeroed(geohip_ctx* ctx, int slot, size_t bytes, void** out) {
    if (slot < 0 || S_I0 + slot >= S_COUNT) return fail(ctx, GEOHIP_ERR_DEVICE, "internal: scratch slot out of range");
    int rc = ensure_zeroed(ctx, (Slot)(S_I0 + slot), bytes);
    if (!rc) *out = ctx->buf[S_I0 + slot];
    return rc;
}
unsigned long long ctx_next_epoch(geohip_ctx* ctx) {
    ctx->lb_epoch = ctx->lb_epoch % ((1ull << 22) - 1) + 1;
    return ctx->lb_epoch;
}
// Look-back status words of a launch carry its epoch in their top bits, so they need no reset
// between launches -- provided no word can hold the epoch of the current launch unless this
// launch wrote it: the slot is zeroed whenever it is (re)allocated (epoch 0 is never issued), and
// all of it again when the epoch counter wraps (a word last written 2^22 - 1 launches ago by a
// larger batch would otherwise read as ready).
int ctx_lookback_status(geohip_ctx* ctx, int slot, size_t bytes, void** out, unsigned long long* epoch) {
    if (slot < 0 || S_I0 + slot >= S_COUNT) return fail(ctx, GEOHIP_ERR_DEVICE, "internal: scratch slot out of range");
    const Slot s = (Slot)(S_I0 + slot);
    int rc = ensure_zeroed(ctx, s, bytes);
    if (rc) return rc;
    *epoch = ctx_next_epoch(ctx);
    if (*epoch == 1 && hipMemsetAsync(ctx->buf[s], 0, ctx->cap[s], ctx->stream) != hipSuccess)
        return fail(ctx, GEOHIP_ERR_DEVICE, "look-back status reset failed");
    *out = ctx->buf[s];
    return GEOHIP_OK;
}
int ctx_cus(geohip_ctx* ctx) { return ctx->cus; }

int ctx_begin(geohip_ctx* ctx) { return begin(ctx); }
hipStream_t ctx_stream(geohip_ctx* ctx) { return ctx->stream; }
int ctx_mem(geohip_ctx* ctx) { return ctx->mem; }
uint64_t* ctx_pinned(geohip_ctx* ctx) { return ctx->pinned; }
int ctx_fault_block(geohip_ctx* ctx, unsigned** out) {
    int rc = ensure_zeroed(ctx, S_RLB, kRlbBytes);
    if (rc) return rc;
    *out = fault_block(ctx);
    return GEOHIP_OK;
}
void** ctx_pcache_slot(geohip_ctx* ctx) { return &ctx->pcache; }
void** ctx_kcache_slot(geohip_ctx* ctx) { return &ctx->kcache; }
void ctx_timing_events(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1) { timing_events(ctx, e0, e1); }
void ctx_kernel_events(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1) { timed_pair(ctx, e0, e1, 1); }
void ctx_kernel_step_events(geohip_ctx* ctx, hipEvent_t* e0, hipEvent_t* e1) { timed_pair(ctx, e0, e1, 2); }
int ctx_stage_xy(geohip_ctx* ctx, const double* x, const double* y, uint64_t n, int which, const double** dx,
                 const double** dy) {
    return which == 0 ? stage_xy(ctx, x, y, n, S_X, S_Y, dx, dy) : stage_xy(ctx, x, y, n, S_QX, S_QY, dx, dy);
}
}  // namespace geohip
