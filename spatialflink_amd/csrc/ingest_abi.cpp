// ingest_abi.cpp -- geohip_ingest_points (include/geohip.h): argument checks the way the
// reference fails, scratch, the ingest launch (ingest.hip) and the count readback.
// Also the CPU test hook geohip_debug_ingest_record, which runs the very parser the kernels run
// (ingest_parse.h, host-compiled) on one record so the CPU suite can check its decisions.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>

#include "geohip_internal.h"
#include "ingest.h"
#include <cstdlib>
#include "join.h"

using namespace geohip;

namespace {

#define ICHK(expr)                                                                                  \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

enum { I_TEXT, I_STATUS, I_WORDS, I_X, I_Y, I_TS, I_CELL, I_LIST, I_OID, I_OIDLEN, I_OIDSEG };

// java.util.regex metacharacters: "\\s*" + delimiter + "\\s*" would not be a literal split
bool delim_ok(int32_t d) {
    if (d <= 0 || d >= 0x80 || d == '"' || d == '\n') return false;
    return strchr("\\^$.|?*+()[]{}", d) == nullptr;
}

int check_spec(geohip_ctx* ctx, const geohip_ingest_spec* sp, ingest::Spec* out) {
    if (!sp) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null spec");
    if (sp->format < GEOHIP_FMT_CSV || sp->format > GEOHIP_FMT_WKT) return ctx_fail(ctx, GEOHIP_ERR_ARG, "unknown format");
    memset(out, 0, sizeof *out);
    out->format = sp->format;
    out->delim = sp->delim;
    out->fx = sp->attr_x;
    out->fy = sp->attr_y;
    out->fts = sp->attr_ts;
    out->foid = -1;
    if (sp->format == GEOHIP_FMT_CSV) {
        if (!delim_ok(sp->delim)) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "delimiter must be one literal byte");
        if (sp->attr_x < 0 || sp->attr_y < 0 || sp->attr_ts < -1)
            return ctx_fail(ctx, GEOHIP_ERR_ARG, "negative csvTsvSchemaAttr index");  // List.get(-1) throws
        if (sp->attr_x > 4095 || sp->attr_y > 4095 || sp->attr_ts > 4095)
            return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "field index > 4095");
    } else {
        out->fts = -1;
    }
    return GEOHIP_OK;
}

struct HostReader {
    const uint8_t* b;
    uint64_t n;
    uint8_t operator()(uint64_t p) const { return p < n ? b[p] : (uint8_t)'\n'; }
};

// The TrajectoryStream parts of the spec: the CSV objID field, the GeoJSON property names and
// the DateFormat (GeoJSONToTSpatial, Deserialization.java:149-208).
int check_traj(geohip_ctx* ctx, const geohip_ingest_spec* sp, const geohip_traj_spec* tr, bool want_oid,
               ingest::Spec* out) {
    if (sp->format == GEOHIP_FMT_CSV && want_oid) {
        if (sp->attr_oid < 0) return ctx_fail(ctx, GEOHIP_ERR_ARG, "negative csvTsvSchemaAttr index");
        if (sp->attr_oid > 4095) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "field index > 4095");
        out->foid = sp->attr_oid;
    }
    if (sp->format != GEOHIP_FMT_GEOJSON) return GEOHIP_OK;
    if (!tr) return ctx_fail(ctx, GEOHIP_ERR_ARG, "GeoJSON trajectories need a geohip_traj_spec");
    if (tr->date_format != GEOHIP_DATE_NONE && tr->date_format != GEOHIP_DATE_YMD_HMS)
        return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "date format not restated (GEOHIP_DATE_YMD_HMS only)");
    if (tr->utc_offset_min < -24 * 60 || tr->utc_offset_min > 24 * 60)
        return ctx_fail(ctx, GEOHIP_ERR_ARG, "utc_offset_min out of range");
    const size_t lt = strnlen(tr->prop_ts, sizeof tr->prop_ts), lo = strnlen(tr->prop_oid, sizeof tr->prop_oid);
    if (lt >= sizeof tr->prop_ts || lo >= sizeof tr->prop_oid) return ctx_fail(ctx, GEOHIP_ERR_ARG, "property name not NUL-terminated");
    for (size_t i = 0; i < lt; i++)
        if (tr->prop_ts[i] == '"' || tr->prop_ts[i] == '\\' || (unsigned char)tr->prop_ts[i] < 0x20)
            return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "property names with JSON escapes are not restated");
    for (size_t i = 0; i < lo; i++)
        if (tr->prop_oid[i] == '"' || tr->prop_oid[i] == '\\' || (unsigned char)tr->prop_oid[i] < 0x20)
            return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "property names with JSON escapes are not restated");
    out->traj = 1;
    out->date_fmt = tr->date_format;
    out->utc_off_min = tr->utc_offset_min;
    out->kts_len = (int32_t)lt;
    out->koid_len = (int32_t)lo;
    memcpy(out->kts, tr->prop_ts, lt);
    memcpy(out->koid, tr->prop_oid, lo);
    return GEOHIP_OK;
}

int ingest_impl(geohip_ctx* ctx, const geohip_grid* grid, const geohip_ingest_spec* spec, const geohip_traj_spec* traj,
                bool trajectory, const char* text, uint64_t nbytes, double* out_x, double* out_y, int64_t* out_ts,
                uint32_t* out_cell, uint64_t* out_oid, uint64_t cap, uint64_t* out_count, uint64_t* out_bad) {
    int rc = ctx_begin(ctx);
    if (rc) return rc;
    if (!out_count || !out_bad) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null count output");
    *out_count = 0;
    *out_bad = UINT64_MAX;
    if (cap && (!out_x || !out_y)) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null coordinate output");
    if (out_cell && !grid) return ctx_fail(ctx, GEOHIP_ERR_ARG, "cell output needs a grid");
    if (nbytes && !text) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null text");
    IngestArgs a;
    memset(&a, 0, sizeof a);
    rc = check_spec(ctx, spec, &a.spec);
    if (!rc && trajectory) rc = check_traj(ctx, spec, traj, out_oid != nullptr, &a.spec);
    if (rc) return rc;
    if (nbytes >= (1ull << 40)) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "batch larger than 1 TiB");
    if (grid) {
        a.min_x = grid->min_x;
        a.min_y = grid->min_y;
        a.cell_len = grid->cell_len;
        a.n = grid->n;
    }
    a.pad = 0;
    const uint64_t nchunks = ingest_chunks(nbytes);
    if (nchunks >= (1ull << 31)) return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED, "batch too large");
    hipStream_t st = ctx_stream(ctx);
    const bool dev = ctx_mem(ctx) == GEOHIP_MEM_DEVICE;
    void *status, *words, *list;
    unsigned long long epoch = 0;
    rc = ctx_lookback_status(ctx, I_STATUS, nchunks * 8, &status, &epoch);
    if (!rc) rc = ctx_ensure_ingest(ctx, I_LIST, nchunks * 16, &list);
    if (!rc) rc = ctx_ensure_ingest_zeroed(ctx, I_WORDS, 64, &words);  // the ticket word starts at zero
    if (rc) return rc;
    const uint8_t* dtext = reinterpret_cast<const uint8_t*>(text);
    double *dx = out_x, *dy = out_y;
    int64_t* dts = out_ts;
    uint32_t* dcell = out_cell;
    uint64_t* doid = out_oid;
    if (dev) {
        if (((uintptr_t)text & 15u) != 0) return ctx_fail(ctx, GEOHIP_ERR_ARG, "device text must be 16-byte aligned");
    } else {
        void *t, *px, *py, *pts = nullptr, *pc = nullptr, *po = nullptr;
        rc = ctx_ensure_ingest(ctx, I_TEXT, nbytes, &t);
        if (!rc) rc = ctx_ensure_ingest(ctx, I_X, cap * 8, &px);
        if (!rc) rc = ctx_ensure_ingest(ctx, I_Y, cap * 8, &py);
        if (!rc && out_ts) rc = ctx_ensure_ingest(ctx, I_TS, cap * 8, &pts);
        if (!rc && out_cell) rc = ctx_ensure_ingest(ctx, I_CELL, cap * 4, &pc);
        if (!rc && out_oid) rc = ctx_ensure_ingest(ctx, I_OID, cap * 8, &po);
        if (rc) return rc;
        if (nbytes) ICHK(hipMemcpyAsync(t, text, nbytes, hipMemcpyHostToDevice, st));
        dtext = static_cast<const uint8_t*>(t);
        dx = static_cast<double*>(px);
        dy = static_cast<double*>(py);
        dts = static_cast<int64_t*>(pts);
        dcell = static_cast<uint32_t*>(pc);
        doid = static_cast<uint64_t*>(po);
    }
    a.oid = doid;
    // [0] total, [1] ticket (re-armed by the kernel), [2] ~first rejected record, [3] listed chunks
    unsigned long long* w = static_cast<unsigned long long*>(words);
    ICHK(hipMemsetAsync(w + 2, 0, 16, st));
    const IngestLookback lb{static_cast<unsigned long long*>(status), reinterpret_cast<unsigned*>(w + 1),
                            epoch, static_cast<ulonglong2*>(list), reinterpret_cast<unsigned*>(w + 3)};
    hipError_t e = launch_ingest(ctx, dtext, nbytes, a, lb, w, dx, dy, dts, dcell, cap, w + 2, st);
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("ingest launch: ") + hipGetErrorString(e));
    uint64_t* pinned = ctx_pinned(ctx);
    ICHK(hipMemcpyAsync(pinned, w, 32, hipMemcpyDeviceToHost, st));
    ICHK(hipStreamSynchronize(st));
    if (pinned[3] >> 32) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, "ingest: record-base look-back gave up");
    const uint64_t total = pinned[0], bad = pinned[2] ? ~pinned[2] : UINT64_MAX;
    *out_count = total;
    *out_bad = bad;
    if (!dev) {
        const uint64_t m = total < cap ? total : cap;
        if (m) {
            ICHK(hipMemcpy(out_x, dx, m * 8, hipMemcpyDeviceToHost));
            ICHK(hipMemcpy(out_y, dy, m * 8, hipMemcpyDeviceToHost));
            if (out_ts) ICHK(hipMemcpy(out_ts, dts, m * 8, hipMemcpyDeviceToHost));
            if (out_cell) ICHK(hipMemcpy(out_cell, dcell, m * 4, hipMemcpyDeviceToHost));
            if (out_oid) ICHK(hipMemcpy(out_oid, doid, m * 8, hipMemcpyDeviceToHost));
        }
    }
    if (bad != UINT64_MAX)
        return ctx_fail(ctx, GEOHIP_ERR_UNSUPPORTED,
                        "record " + std::to_string(bad) + " is malformed or outside the device grammar");
    if (total > cap) return ctx_fail(ctx, GEOHIP_ERR_CAPACITY, "output capacity too small; *out_count = required");
    return GEOHIP_OK;
}

}  // namespace

extern "C" {

int geohip_ingest_points(geohip_ctx* ctx, const geohip_grid* grid, const geohip_ingest_spec* spec, const char* text,
                         uint64_t nbytes, double* out_x, double* out_y, int64_t* out_ts, uint32_t* out_cell,
                         uint64_t cap, uint64_t* out_count, uint64_t* out_bad) {
    return ingest_impl(ctx, grid, spec, nullptr, false, text, nbytes, out_x, out_y, out_ts, out_cell, nullptr, cap,
                       out_count, out_bad);
}

int geohip_ingest_trajectory(geohip_ctx* ctx, const geohip_grid* grid, const geohip_ingest_spec* spec,
                             const geohip_traj_spec* traj, const char* text, uint64_t nbytes, double* out_x,
                             double* out_y, int64_t* out_ts, uint32_t* out_cell, uint64_t* out_oid, uint64_t cap,
                             uint64_t* out_count, uint64_t* out_bad) {
    return ingest_impl(ctx, grid, spec, traj, true, text, nbytes, out_x, out_y, out_ts, out_cell, out_oid, cap,
                       out_count, out_bad);
}

int geohip_ingest_oid_compact(geohip_ctx* ctx, const char* text, uint64_t nbytes, const uint64_t* oid_spans,
                              uint64_t m, uint8_t* out_text, uint64_t cap, uint64_t* out_off, uint64_t* out_len) {
    int rc = ctx_begin(ctx);
    if (rc) return rc;
    if (!out_len) return ctx_fail(ctx, GEOHIP_ERR_ARG, "null out_len");
    *out_len = 0;
    if (ctx_mem(ctx) != GEOHIP_MEM_DEVICE) return ctx_fail(ctx, GEOHIP_ERR_ARG, "geohip_ingest_oid_compact takes device memory");
    if (!out_off || (m && !oid_spans) || (nbytes && !text) || (cap && !out_text))
        return ctx_fail(ctx, GEOHIP_ERR_ARG, "null argument");
    hipStream_t st = ctx_stream(ctx);
    const uint64_t nseg = oid_segments(m);
    void *len, *seg;
    rc = ctx_ensure_ingest(ctx, I_OIDLEN, m * 8 + 8, &len);
    if (!rc) rc = ctx_ensure_ingest(ctx, I_OIDSEG, nseg * 8 + 64, &seg);
    if (rc) return rc;
    hipError_t e = launch_oid_compact(ctx, reinterpret_cast<const uint8_t*>(text), nbytes, oid_spans, m,
                                      static_cast<uint64_t*>(len), static_cast<uint64_t*>(seg), out_off, nullptr, 0, st);
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("oid compact launch: ") + hipGetErrorString(e));
    uint64_t* pinned = ctx_pinned(ctx);
    ICHK(hipMemcpyAsync(pinned, static_cast<uint64_t*>(seg) + nseg, 16, hipMemcpyDeviceToHost, st));
    ICHK(hipStreamSynchronize(st));
    if (pinned[1]) return ctx_fail(ctx, GEOHIP_ERR_ARG, "an objID span lies outside the text");
    *out_len = pinned[0];
    if (pinned[0] > cap) return ctx_fail(ctx, GEOHIP_ERR_CAPACITY, "output capacity too small; *out_len = required");
    e = launch_oid_compact(ctx, reinterpret_cast<const uint8_t*>(text), nbytes, oid_spans, m, static_cast<uint64_t*>(len),
                           static_cast<uint64_t*>(seg), out_off, out_text, cap, st);
    if (e != hipSuccess) return ctx_fail(ctx, GEOHIP_ERR_DEVICE, std::string("oid compact launch: ") + hipGetErrorString(e));
    ICHK(hipStreamSynchronize(st));
    return GEOHIP_OK;
}

// Test hook: the device parser (ingest_parse.h) compiled for the host, on one record
// (rec[0..len), no '\n' inside).  Returns GEOHIP_OK, GEOHIP_ERR_UNSUPPORTED (rejected) or
// GEOHIP_ERR_ARG (bad spec).
int geohip_debug_ingest_record(const geohip_ingest_spec* spec, const char* rec, uint64_t len, double* x, double* y,
                               int64_t* ts) {
    ingest::Spec sp;
    if (!spec || spec->format < 0 || spec->format > 2) return GEOHIP_ERR_ARG;
    memset(&sp, 0, sizeof sp);  // no trajectory fields: point records only
    sp.foid = -1;
    sp.format = spec->format;
    sp.delim = spec->delim;
    sp.fx = spec->attr_x;
    sp.fy = spec->attr_y;
    sp.fts = spec->format == GEOHIP_FMT_CSV ? spec->attr_ts : -1;
    if (spec->format == GEOHIP_FMT_CSV && (!delim_ok(spec->delim) || sp.fx < 0 || sp.fy < 0 || sp.fts < -1))
        return GEOHIP_ERR_ARG;
    const HostReader rd{reinterpret_cast<const uint8_t*>(rec), len};
    ingest::Parsed o;
    o.x = o.y = 0.0;
    o.ts = 0;
    if (ingest::parse_record(rd, 0, sp, &o) != ingest::kOk) return GEOHIP_ERR_UNSUPPORTED;
    *x = o.x;
    *y = o.y;
    *ts = o.ts;
    return GEOHIP_OK;
}

// Test hook: the trajectory parse (CSV objID, GeoJSON properties) of one record on the host;
// *oid = the objID span relative to rec (0xffffff length: null).
int geohip_debug_ingest_traj_record(const geohip_ingest_spec* spec, const geohip_traj_spec* traj, const char* rec,
                                    uint64_t len, double* x, double* y, int64_t* ts, uint64_t* oid) {
    ingest::Spec sp;
    if (!spec || check_spec(nullptr, spec, &sp) != GEOHIP_OK || check_traj(nullptr, spec, traj, true, &sp) != GEOHIP_OK)
        return GEOHIP_ERR_ARG;
    if (spec->format == GEOHIP_FMT_CSV && (!delim_ok(spec->delim) || sp.fx < 0 || sp.fy < 0 || sp.fts < -1))
        return GEOHIP_ERR_ARG;
    const HostReader rd{reinterpret_cast<const uint8_t*>(rec), len};
    ingest::Parsed o;
    o.x = o.y = 0.0;
    o.ts = 0;
    if (ingest::parse_record(rd, 0, sp, &o) != ingest::kOk) return GEOHIP_ERR_UNSUPPORTED;
    *x = o.x;
    *y = o.y;
    *ts = o.ts;
    *oid = o.oid;
    return GEOHIP_OK;
}

}  // extern "C"
