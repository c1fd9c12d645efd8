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
// chunk), and the LDS bytes staged past the chunk for records that straddle its end.
constexpr uint32_t kIngestChunk = 16384;
constexpr uint32_t kIngestTail = 4096;

struct IngestArgs {
    ingest::Spec spec;
    double min_x, min_y, cell_len;
    int32_t n;
    int32_t pad;
};

inline uint64_t ingest_chunks(uint64_t nbytes) { return (nbytes + kIngestChunk - 1) / kIngestChunk; }

// Pass 1: records per chunk (chunk_cnt[nchunks]); pass 2: exclusive scan into chunk_base and
// the record total (*total); pass 3: per-block record split + parse.  bad[0] = first rejected
// record index (UINT64_MAX if none; must hold UINT64_MAX before the launch).
hipError_t launch_ingest(const uint8_t* text, uint64_t nbytes, const IngestArgs& a, unsigned* chunk_cnt,
                         unsigned long long* chunk_base, unsigned long long* total, double* x, double* y,
                         int64_t* ts, uint32_t* cell, uint64_t cap, unsigned long long* bad, hipStream_t st,
                         hipEvent_t ev0, hipEvent_t ev1);

}  // namespace geohip
