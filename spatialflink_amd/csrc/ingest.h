// ingest.h -- launch interface of the ingest codec kernels (ingest.hip).
//
// A batch of '\n'-separated text records (the Strings a Flink source hands to
// Deserialization.PointStream's map functions, Deserialization.java:47-62) becomes SoA
// x[], y[] (+ Long timestamps, + the HelperClass.assignGridCellID cell as cx * n + cy).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ingest_parse.h"

namespace geohip {

// Bytes of text owned by one block (its records are those whose preceding '\n' lies in the
// chunk), and the LDS bytes staged past the chunk for the record that straddles its end (a
// longer record reads its remaining bytes from global memory through the general parser).
// 48 text bytes per thread of the 512-thread block (16-byte multiple): 24 KB chunks, ~430 CSV
// records for 512 threads (16 KB: ~290, 44 % of the lanes idle in the parse); same box: 32 B
// 494 us, 48 B 422 us, 64 B 466 us
constexpr uint32_t kIngestChunk = 512u * 48u;
constexpr uint32_t kIngestTail = 512;

struct IngestArgs {
    ingest::Spec spec;
    double min_x, min_y, cell_len;
    int32_t n;
    int32_t pad;
    uint64_t* oid;  // nullable: per-record objID spans (ingest::kOidLenBits packing)
};

inline uint64_t ingest_chunks(uint64_t nbytes) { return (nbytes + kIngestChunk - 1) / kIngestChunk; }

// Chunk-order look-back state: status[nchunks] words (any content before the first launch),
// a ticket word (zero before the first launch; the last chunk re-arms it), the launch's epoch
// (1 .. 2^22 - 1, new per launch); the chunks left to the general grammar: listed[nchunks]
// (chunk, record base) and their count *nlisted (zero before the launch); nlisted[1] = 1 when a
// look-back gave up (zero before the launch).
struct IngestLookback {
    unsigned long long* status;
    unsigned* ticket;
    unsigned long long epoch;
    ulonglong2* listed;
    unsigned* nlisted;
};

// Two launches: ingest_fused (per chunk record split + look-back record base + CSV fast-path
// parse; *total = records in the batch) and ingest_general (the full grammar over the chunks the
// first left undecided).  bad[0] = ~(first rejected record index), 0 if none (must hold 0
// before the launch).
hipError_t launch_ingest(geohip_ctx* ctx, const uint8_t* text, uint64_t nbytes, const IngestArgs& a,
                         const IngestLookback& lb, unsigned long long* total, double* x, double* y, int64_t* ts,
                         uint32_t* cell, uint64_t cap, unsigned long long* bad, hipStream_t st);

// objID spans -> strings: launch_oid_compact without out_text writes the lengths, the scan and
// out_off (seg[nseg] = the total bytes, seg[nseg + 1] != 0: a span outside the text); with
// out_text, the bytes (the same len / seg / out_off).  seg holds oid_segments(m) + 2 words.
uint64_t oid_segments(uint64_t m);
hipError_t launch_oid_compact(geohip_ctx* ctx, const uint8_t* text, uint64_t nbytes, const uint64_t* spans, uint64_t m,
                              uint64_t* len, uint64_t* seg, uint64_t* out_off, uint8_t* out_text, uint64_t cap,
                              hipStream_t st);

}  // namespace geohip
