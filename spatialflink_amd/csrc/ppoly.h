// ppoly.h -- point-polygon window range query (PointPolygonRangeQuery.java:76-124).
#pragma once
#include <stdint.h>

#include "geohip_internal.h"

namespace geohip {
// drop the ctx's cached polygon plan (geohip_ctx_destroy)
void ppoly_cache_drop(geohip_ctx* ctx);

// range (join = 0: gq ignored, pairs (polygon, point)) or join (join = 1: polygons planned on gq,
// point cells on grid, pairs (point, polygon), PointPolygonJoinQuery.java:162-201)
int ppoly_impl(geohip_ctx* ctx, const geohip_grid* grid, const geohip_grid* gq, int join, const double* x,
               const double* y, uint64_t n, const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
               const double* vy, uint64_t nv, uint32_t npoly, double r, int approximate, uint32_t* out_pairs,
               uint64_t cap, uint64_t* out_count, uint32_t point_base = 0, uint64_t* count_dev = nullptr);
// geohip_ctx_sync found an async call's candidate overflow: the next call sizes its buffer for need
void ppoly_note_cand_need(geohip_ctx* ctx, uint64_t need);
// point-polygon kNN of one polygon (PointPolygonKNNQuery.java:162-236); async: device outputs and
// count, no host synchronisation
int knn_ppoly_impl(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y, uint64_t n,
                   const uint32_t* ring_off, uint32_t nring, const double* vx, const double* vy, uint64_t nv, double r,
                   uint32_t k, int approximate, uint32_t* out_idx, double* out_dist, uint32_t* out_count, bool async);
void knn_poly_cache_drop(geohip_ctx* ctx);
// point kNN with k > GEOHIP_KNN_MAX_K: candidate scan, keys, radix select, sort (device outputs)
int knn_pp_large_impl(geohip_ctx* ctx, const PointPlan& plan, const double* dx, const double* dy, uint64_t n,
                      double qx, double qy, uint32_t k, double* od, unsigned* oi, unsigned* ocnt);
// rank merge of nlists * list_len (> 8192) entries with k > 256 (device pointers)
int knn_merge_large_impl(geohip_ctx* ctx, const unsigned long long* d, const unsigned* i, unsigned nlists,
                         unsigned list_len, unsigned k, double* od, unsigned* oi, unsigned* ocnt);
}  // namespace geohip
