/*
 * geohip.h -- C ABI of libgeohip.so: MI355X (gfx950) evaluation of GeoFlink windowed
 * spatial queries.  One call evaluates one window's contents; window assembly (Flink's
 * SlidingProcessingTimeWindows, keyBy(gridID)) stays in the caller.
 *
 * Each entry point replaces the per-cell window-function body of one reference operator
 * (paths relative to /root/reference/src/main/java/GeoFlink):
 *
 *   geohip_range_pp    <- PointPointRangeQuery.run, window branch     spatialOperators/range/PointPointRangeQuery.java:86-137
 *                         (filter :102-107, keyBy :111-116, apply :117-136; RealTime :43-83 has the same predicate)
 *   geohip_knn_pp      <- PointPointKNNQuery.windowBased + merge      spatialOperators/knn/PointPointKNNQuery.java:125-191,
 *                                                                      spatialOperators/knn/KNNQuery.java:204-272
 *   geohip_join_pp     <- PointPointJoinQuery.windowBased             spatialOperators/join/PointPointJoinQuery.java:113-172
 *                         + JoinQuery.getReplicatedPointQueryStream    spatialOperators/join/JoinQuery.java:73-90
 *   geohip_range_ppoly <- PointPolygonRangeQuery.run, window branch   spatialOperators/range/PointPolygonRangeQuery.java:76-124
 *   geohip_join_ppoly  <- PointPolygonJoinQuery.windowBased            spatialOperators/join/PointPolygonJoinQuery.java:162-201
 *                         + JoinQuery.getReplicatedPolygonQueryStream  spatialOperators/join/JoinQuery.java:93-115
 *   geohip_knn_ppoly   <- PointPolygonKNNQuery.windowBased + merge     spatialOperators/knn/PointPolygonKNNQuery.java:162-236,
 *                                                                      spatialOperators/knn/KNNQuery.java:204-272
 *                         (one independent query per polygon)
 *   geohip_ingest_points <- Deserialization.PointStream / TrajectoryStream map functions
 *                         spatialStreams/Deserialization.java:47-80, 132-146, 223-228, 248-254, 306-321
 *   geohip_grid        <- UniformGrid getters                         spatialIndices/UniformGrid.java:136-146
 *                         (values copied from the Java object, so both constructors :47-85 are covered)
 *
 * Semantics (bit-exact contract, DESIGN.md "Parity"):
 *   - cell of a point  = (int)Math.floor((x - minX)/cellLength) per axis  (utils/HelperClass.java:104-116)
 *   - guaranteed cells = square of Lg=(int)floor(r/(l*sqrt2)-1) layers, candidate = Lc=(int)ceil(r/l)
 *     layers minus guaranteed, clipped by validKey               (UniformGrid.java:165-190, 224-229, 367-444)
 *   - distances: JTS 1.16.1 Geometry.distance (fdlibm hypot, DistanceOp MAX_VALUE start)
 *   - range: guaranteed cells emitted without a distance check; candidate cells need dist <= r
 *   - kNN: no radius filter; k smallest (dist, idx) over guaranteed u candidate cells, ascending
 *   - join: pairs (p, q) with cell_uGrid(p) in Nbr_qGrid(q) and dist <= r; r == 0 -> all cells
 *
 * Indices are window-local (0-based position in the caller's arrays) and map back to the
 * caller's Point objects.  Range output is in ascending index order; join and point-polygon
 * outputs are sets (unordered, like the reference's output streams); kNN is ascending
 * (dist, idx).
 *
 * Memory: the caller owns every buffer; nothing is retained after a call returns.  With
 * GEOHIP_MEM_HOST (default) input/output pointers are host memory; with GEOHIP_MEM_DEVICE
 * they are device pointers on the ctx's device (x/y 16-byte aligned).  Scalars
 * (out_count) are always host memory for the synchronous calls.
 *
 * Threading: one ctx per calling thread (Flink task slot); distinct ctxs may run
 * concurrently.  Synchronous calls return after the results are in place.  *_async calls
 * enqueue on the ctx stream and return immediately (device memory only).
 *
 * Errors: int status; never aborts.  GEOHIP_ERR_ARG covers the reference's System.exit(1)
 * (UniformGrid.java:237-241, 272-276: join with r < 0 or NaN) and NumberFormatException in
 * getIntCellIndices.  GEOHIP_ERR_CAPACITY reports the required size in *out_count.
 */
#ifndef GEOHIP_H
#define GEOHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GEOHIP_OK 0
#define GEOHIP_ERR_ARG 1
#define GEOHIP_ERR_CAPACITY 2
#define GEOHIP_ERR_DEVICE 3
#define GEOHIP_ERR_OOM 4
#define GEOHIP_ERR_UNSUPPORTED 5

#define GEOHIP_MEM_HOST 0
#define GEOHIP_MEM_DEVICE 1

/* Every k >= 1 is served (PointPointKNNQuery.java:33 / PointPolygonKNNQuery.java:34 take any
   Integer k).  Up to these values one pass selects the k nearest in one workgroup's LDS; above
   them the candidates are compacted, radix-selected and sorted (the large-k form). */
#define GEOHIP_KNN_MAX_K 1024
#define GEOHIP_KNN_PPOLY_MAX_K 256

typedef struct geohip_ctx geohip_ctx;

/* UniformGrid state: getMinX(), getMinY(), getCellLength(), getNumGridPartitions(). */
typedef struct geohip_grid {
    double min_x;
    double min_y;
    double cell_len;
    int32_t n;
    int32_t reserved;
} geohip_grid;

/* Inclusive cell-index rectangle (planning introspection). */
typedef struct geohip_rect {
    int32_t x0, x1, y0, y1;
} geohip_rect;

/* ---- context ---------------------------------------------------------------------- */
/* device_mask: bit i selects HIP device i (exactly one bit; 0 = current device). */
int geohip_ctx_create(uint32_t device_mask, geohip_ctx** out_ctx);
int geohip_ctx_destroy(geohip_ctx* ctx);
const char* geohip_last_error(const geohip_ctx* ctx);
int geohip_ctx_set_mem(geohip_ctx* ctx, int mem_kind);
/* Enqueue on the caller's hipStream_t from now on (NULL = the HIP null stream, e.g. PyTorch's
   default stream): work the caller queued on that stream before a call is ordered before the
   call's kernels, and the *_async results are ordered before later work on it. */
int geohip_ctx_set_stream(geohip_ctx* ctx, void* hip_stream);
/* Rebinding (set_stream / reset_stream) orders the new stream after the work already queued on
   the previously bound one (an event recorded on it at the switch), so a caller's stream must stay
   alive until the ctx is bound to another stream or destroyed. */
/* Back to the ctx's own (non-blocking) stream, the state after geohip_ctx_create. */
int geohip_ctx_reset_stream(geohip_ctx* ctx);
void* geohip_ctx_stream(geohip_ctx* ctx);
/* Output order of the point-point range calls (geohip_range_pp, _pane, _async):
   GEOHIP_ORDER_ASCENDING (the default after geohip_ctx_create) -- hit indices ascending;
   GEOHIP_ORDER_ANY -- the same set in an unspecified order, as the reference's window function
   emits it (PointPointRangeQuery.java:117-136 collects the filter's hits as they arrive), from
   one pass with no ordered emission (faster); geohip_knn_range_pp's range part likewise (its
   pass then sweeps the window in interleaved fronts as the kNN alone does). */
#define GEOHIP_ORDER_ASCENDING 0
#define GEOHIP_ORDER_ANY 1
int geohip_ctx_set_range_order(geohip_ctx* ctx, int order);
/* Device timing of each call's step (measurement): while enabled, every query call's device work
   is timed with HIP events on the ctx stream. */
int geohip_ctx_set_timing(geohip_ctx* ctx, int enable);
/* Synchronises, then reports the summed step duration and step count since the last reset (a
   one-kernel step: the kernel's own dispatch timestamps; a multi-launch step: first launch to
   last, gaps included). */
int geohip_ctx_timing(geohip_ctx* ctx, double* total_ms, uint64_t* launches, int reset);
/* As geohip_ctx_timing, plus the summed duration and count of the steps' kernels, each stamped by
   its own dispatch (hipExtLaunchKernel: the begin / end timestamps rocprofv3 reports), so
   kernel_ms / steps is a step's kernel time without the gaps between its launches. */
int geohip_ctx_timing_kernels(geohip_ctx* ctx, double* step_ms, uint64_t* steps, double* kernel_ms,
                              uint64_t* kernels, int reset);
/* Waits for the ctx's enqueued work, then reports what its *_async calls since the last check
   could not return as a status (the first that applies; all are cleared):
     GEOHIP_ERR_DEVICE    a kernel gave up a look-back wait (a device-side invariant broken: the
                          results of those calls are invalid),
     GEOHIP_ERR_ARG       geohip_join_pp_async: a query key the reference cannot parse back
                          (NumberFormatException) or whose neighbour loop never ends
                          (UniformGrid.java:261-293) -- its results are incomplete,
   (The point-polygon forms report no error for a short candidate buffer: the chunks whose
   candidates pass it are decided by a redo pass in the same call, and the count they needed
   sizes the next call's buffer.)
   The synchronous calls check the look-back themselves. */
int geohip_ctx_sync(geohip_ctx* ctx);
int geohip_device_count(int* out_count);
/* "geohip 0.2 (gfx950)".  GEOHIP_ABI_VERSION / geohip_abi_version() change whenever an existing
   entry point's signature changes, so a binding built against another header can refuse to run:
     1  round 1-3 signatures
     2  the polygon entry points take nv (the vertex count) after vy; the *_async join and
        point-polygon forms and geohip_abi_version added */
#define GEOHIP_ABI_VERSION 2
const char* geohip_version(void);
int geohip_abi_version(void);

/* ---- queries (synchronous) ------------------------------------------------------------ */
int geohip_range_pp(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                    uint64_t n, double qx, double qy, double r, int approximate,
                    uint32_t* out_idx, uint64_t cap, uint64_t* out_count);
/* geohip_range_pp over one pane of a sliding window (pane reuse): the hit
   indices are point_base + the position in the pane (mod 2^32) -- stream positions when
   point_base is the pane's first one, ascending -- so a pane's hits serve every window that
   holds it with no pass over them (PointPointRangeQuery.queryIncremental, :144-245). */
int geohip_range_pp_pane(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                         uint64_t n, uint32_t point_base, double qx, double qy, double r, int approximate,
                         uint32_t* out_idx, uint64_t cap, uint64_t* out_count);

int geohip_knn_pp(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                  uint64_t n, double qx, double qy, double r, uint32_t k,
                  uint32_t* out_idx, double* out_dist, uint32_t* out_count);

/* The kNN (k) and the range (radius r) of the same query point over one window -- two GeoFlink
   continuous queries (PointPointKNNQuery.java:125-191 and PointPointRangeQuery.java:86-137) with
   the same q and r over the same stream, as BASELINE.json configs[4] runs them -- evaluated in
   one pass over the window: results identical to geohip_knn_pp and geohip_range_pp. */
int geohip_knn_range_pp(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                        uint64_t n, double qx, double qy, double r, uint32_t k, int approximate,
                        uint32_t* knn_idx, double* knn_dist, uint32_t* knn_count,
                        uint32_t* range_idx, uint64_t range_cap, uint64_t* range_count);

/* out_pairs: 2*cap uint32 (p_idx, q_idx) pairs. */
int geohip_join_pp(geohip_ctx* ctx, const geohip_grid* grid_data, const geohip_grid* grid_query,
                   const double* dx, const double* dy, uint64_t nd,
                   const double* qx, const double* qy, uint64_t nq, double r, int approximate,
                   uint32_t* out_pairs, uint64_t cap, uint64_t* out_count);
int geohip_join_pp_count_only(geohip_ctx* ctx, const geohip_grid* grid_data, const geohip_grid* grid_query,
                              const double* dx, const double* dy, uint64_t nd,
                              const double* qx, const double* qy, uint64_t nq, double r,
                              int approximate, uint64_t* out_count);

/* Query polygons, always in HOST memory (whatever the ctx's mem kind: they are planned on the
   host and cached per ctx; only the points and the outputs follow GEOHIP_MEM_DEVICE).
   Polygon i = rings [poly_rings[i], poly_rings[i+1]) (poly_rings NULL: ring i alone), ring j =
   vertices vx/vy[ring_off[j] .. ring_off[j+1]) -- the List<List<Coordinate>> given to
   Polygon(List<List<Coordinate>>, UniformGrid) (Polygon.java:52-66, 115-165): one ring is closed
   here if open and needs > 3 coords; several rings are padded and closed each, the largest JTS
   area becomes the shell and the others its holes, in createPolygonArray's order.  Up to 65535
   rings per polygon.  Where the reference throws (an empty ring, a ring
   whose first coordinate is NaN: LinearRing not closed) or leaves the polygon null (first ring
   with <= 3 coords): GEOHIP_ERR_ARG.  npoly == 0: no pairs, the polygon arrays may be NULL.
   Distances: JTS point.distance(polygon) -- 0 inside the shell and outside every hole, or on any
   ring; else the minimum over every ring's segments.
   nv = the length of vx / vy: every ring offset the polygons use must be <= nv (GEOHIP_ERR_ARG
   otherwise -- the library reads no vertex past it).
   out_pairs: 2*cap uint32 (poly_idx, point_idx), unordered. */
int geohip_range_ppoly(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                       uint64_t n, const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
                       const double* vy, uint64_t nv, uint32_t npoly, double r, int approximate,
                       uint32_t* out_pairs, uint64_t cap, uint64_t* out_count);

/* geohip_range_ppoly over one pane of a sliding window (pane reuse): point
   indices are point_base + the position in the pane (mod 2^32), i.e. stream positions when
   point_base is the pane's first one -- a pane is evaluated once and its pairs serve every window
   that holds it unchanged (a window's local index = stream position - its first position). */
int geohip_range_ppoly_pane(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                            uint64_t n, uint32_t point_base, const uint32_t* poly_rings, const uint32_t* ring_off,
                            const double* vx, const double* vy, uint64_t nv, uint32_t npoly, double r,
                            int approximate, uint32_t* out_pairs, uint64_t cap, uint64_t* out_count);

/* Point-polygon window join: the polygon stream replicated to its guaranteed and candidate
   cells on grid_query (UniformGrid.java:193-206, 398-410), joined with the points' gridIDs on
   grid_points; emits (point_idx, poly_idx) iff approximate or JTS point.distance(polygon) <= r
   (no guaranteed-cell shortcut, PointPolygonJoinQuery.java:183-195).  Polygons as for
   geohip_range_ppoly (host arrays).  out_pairs: 2*cap uint32 (point_idx, poly_idx), unordered. */
int geohip_join_ppoly(geohip_ctx* ctx, const geohip_grid* grid_points, const geohip_grid* grid_query,
                      const double* x, const double* y, uint64_t n, const uint32_t* poly_rings,
                      const uint32_t* ring_off, const double* vx, const double* vy, uint64_t nv,
                      uint32_t npoly, double r, int approximate, uint32_t* out_pairs, uint64_t cap,
                      uint64_t* out_count);

/* Point-polygon kNN of one query polygon of nring rings (ring j = vx/vy[ring_off[j] ..
   ring_off[j+1]), host arrays of nv vertices, built as for geohip_range_ppoly): candidates are the points of
   the polygon's G u C cells (no radius filter); distance = JTS point.distance(polygon), or the
   bbox distance (DistanceFunctions.java:150-200) when approximate.  Output: the
   min(k, candidates) smallest (distance, idx) ascending by distance bits then idx (a NaN bbox
   distance ranks after +Infinity); any k >= 1. */
int geohip_knn_ppoly(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                     uint64_t n, const uint32_t* ring_off, uint32_t nring, const double* vx,
                     const double* vy, uint64_t nv, double r, uint32_t k, int approximate,
                     uint32_t* out_idx, double* out_dist, uint32_t* out_count);
/* Enqueue-only form of geohip_knn_ppoly (GEOHIP_MEM_DEVICE window and outputs; the polygon stays
   host memory and is planned once per ctx): k (dist, idx) ascending, entries past the candidate
   count are (+inf-bits sentinel, 0xffffffff); *out_count_dev = number of valid entries.  No host
   round trip: the selection path is chosen from the previous call's candidate count. */
int geohip_knn_ppoly_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                           uint64_t n, const uint32_t* ring_off, uint32_t nring, const double* vx,
                           const double* vy, uint64_t nv, double r, uint32_t k, int approximate,
                           uint32_t* out_idx, double* out_dist, uint32_t* out_count_dev);

/* ---- device-resident pipeline forms (GEOHIP_MEM_DEVICE pointers; enqueue only) -------- */
/* Writes k (dist, idx) ascending to out_dist/out_idx (device), entries past the candidate
   count are (+inf-bits sentinel, 0xffffffff); *out_count_dev = number of valid entries. */
int geohip_knn_pp_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                        uint64_t n, double qx, double qy, double r, uint32_t k,
                        uint32_t* out_idx, double* out_dist, uint32_t* out_count_dev);
/* Merge nlists sorted (dist, idx) lists of list_len entries (e.g. the all-gathered per-shard
   kNN results) into the k smallest; same output convention as geohip_knn_pp_async.
   idx values are taken as global ids (shards add their base offset before the gather).
   Any k >= 1 and list count (fewer than 2^32 entries in all). */
int geohip_knn_merge_async(geohip_ctx* ctx, const double* dist, const uint32_t* idx, uint32_t nlists,
                           uint32_t list_len, uint32_t k, uint32_t* out_idx, double* out_dist,
                           uint32_t* out_count_dev);
/* Sliding-window kNN with pane reuse (the window = the last npanes panes,
   PointPointKNNQuery's SlidingProcessingTimeWindows with size a multiple of the slide): the
   window's k smallest from the panes' top-k lists (each ascending, sentinel-padded, as
   geohip_knn_pp_async writes them) kept in a ring of list_len-entry slots (ring_dist/ring_idx,
   device); slots[b] (host) names the slot of the b-th pane, oldest first, offsets[b] (host) its
   first point's position in the window (indices are rebased by it).  One launch; output as
   geohip_knn_merge_async.  1 <= npanes <= 16. */
int geohip_knn_merge_panes_async(geohip_ctx* ctx, const double* ring_dist, const uint32_t* ring_idx,
                                 uint32_t list_len, const uint32_t* slots, const uint64_t* offsets,
                                 uint32_t npanes, uint32_t k, uint32_t* out_idx, double* out_dist,
                                 uint32_t* out_count_dev);
/* geohip_knn_range_pp into device buffers (counts on the device). */
int geohip_knn_range_pp_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                              uint64_t n, double qx, double qy, double r, uint32_t k, int approximate,
                              uint32_t* knn_idx, double* knn_dist, uint32_t* knn_count_dev,
                              uint32_t* range_idx, uint64_t range_cap, uint64_t* range_count_dev);
/* Range into device buffers: out_idx (cap entries), *out_count_dev = total hits. */
int geohip_range_pp_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                          uint64_t n, double qx, double qy, double r, int approximate,
                          uint32_t* out_idx, uint64_t cap, uint64_t* out_count_dev);
/* geohip_join_pp into device buffers with no host round trip: out_pairs (cap pairs),
   *out_count_dev (device uint64) = the window's pair total; pairs past cap are not written (the
   caller compares the count with cap).  Query-key errors surface at geohip_ctx_sync. */
int geohip_join_pp_async(geohip_ctx* ctx, const geohip_grid* grid_data, const geohip_grid* grid_query,
                         const double* dx, const double* dy, uint64_t nd, const double* qx, const double* qy,
                         uint64_t nq, double r, int approximate, uint32_t* out_pairs, uint64_t cap,
                         uint64_t* out_count_dev);
/* geohip_range_ppoly / geohip_join_ppoly into device buffers with no host round trip (points and
   outputs in device memory, polygons host arrays as for the synchronous forms):
   *out_count_dev = the pair total, pairs past cap not written.  The candidate buffer is sized
   from the previous call on this ctx (or n / 16); an overflow surfaces at geohip_ctx_sync.  A
   grid or polygon set the streaming path cannot take (n > 4096 cells per side, > 16384
   polygons) runs the tile-binned path, which synchronises inside the call. */
int geohip_range_ppoly_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                             uint64_t n, const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
                             const double* vy, uint64_t nv, uint32_t npoly, double r, int approximate,
                             uint32_t* out_pairs, uint64_t cap, uint64_t* out_count_dev);
/* geohip_range_ppoly_pane as an enqueue-only call (point indices point_base + position). */
int geohip_range_ppoly_pane_async(geohip_ctx* ctx, const geohip_grid* grid, const double* x, const double* y,
                                  uint64_t n, uint32_t point_base, const uint32_t* poly_rings,
                                  const uint32_t* ring_off, const double* vx, const double* vy, uint64_t nv,
                                  uint32_t npoly, double r, int approximate, uint32_t* out_pairs, uint64_t cap,
                                  uint64_t* out_count_dev);
int geohip_join_ppoly_async(geohip_ctx* ctx, const geohip_grid* grid_points, const geohip_grid* grid_query,
                            const double* x, const double* y, uint64_t n, const uint32_t* poly_rings,
                            const uint32_t* ring_off, const double* vx, const double* vy, uint64_t nv,
                            uint32_t npoly, double r, int approximate, uint32_t* out_pairs, uint64_t cap,
                            uint64_t* out_count_dev);

/* Key-band partition of one window shard for the multi-GPU join (the device form of the
   reference's keyBy(gridID) shuffle, PointPointJoinQuery.java:137-150): a point whose key
   (HelperClass.java:104-116 on grid_data) is a cell (cx, cy) of the nb x nb key space belongs to
   rank cx * world / nb; other points match no neighbour block and are dropped.  Writes the kept
   points grouped by owner rank, in arrival order inside a group -- out_x / out_y and out_idx =
   base + window position -- and out_counts_dev[world] = points per owner (device uint64), ready
   for one all-to-all.  Outputs need n entries.  1 <= world <= 64; device memory only. */
int geohip_band_pack_async(geohip_ctx* ctx, const geohip_grid* grid_data, int32_t nb, uint32_t world,
                           const double* x, const double* y, uint64_t n, int64_t base, double* out_x,
                           double* out_y, int64_t* out_idx, uint64_t* out_counts_dev);

/* The partition for a single point query (kNN / range of (qx, qy) with radius r on grid_data):
   only the points of the query's guaranteed and candidate cells are kept -- the reference filters
   them before its keyBy(gridID) (PointPointKNNQuery.java:137-151, PointPointRangeQuery.java:
   102-116) -- then grouped by owner rank, where column cx belongs to rank (cx / bw) mod world,
   bw = max(1, (2 Lc + 1) / (8 world)) with Lc = getCandidateNeighboringLayers(r)
   (UniformGrid.java:440-444): the query's 2 Lc + 1 candidate columns are dealt round-robin in
   blocks, as keyBy's key hashing spreads them (contiguous bands put one query's whole box on one
   rank).  Otherwise as geohip_band_pack_async. */
int geohip_band_pack_query_async(geohip_ctx* ctx, const geohip_grid* grid_data, int32_t nb, uint32_t world,
                                 double qx, double qy, double r, const double* x, const double* y, uint64_t n,
                                 int64_t base, double* out_x, double* out_y, int64_t* out_idx,
                                 uint64_t* out_counts_dev);

/* ---- output codecs ----------------------------------------------- */
/* The point output schemas of spatialStreams/Serialization.java for m result points, as one text
   buffer: record j is point p = idx[j] (or j when idx is NULL; p >= n is GEOHIP_ERR_ARG, e.g. a
   padded kNN list's 0xffffffff sentinel), each record followed by '\n'.  The Point's fields:
   objID = bytes oid_text[oid_off[p] .. oid_off[p+1]) (UTF-8; oid_text NULL: objID == null; bit 63
   of oid_off[p] set: point p's objID is null, offsets are the low 63 bits),
   timeStampMillisec = ts[p] (ts NULL: 0), point.getX()/getY() = x[p]/y[p], doubles through JDK 8
   Double.toString (FloatingDecimal).
     GEOHIP_FMT_CSV     <- PointToCSVTSVOutputSchema.serialize  Serialization.java:125-150: the
                           fields at positions 0..max(attr) (objID as "null" when null, Long.toString
                           of the timestamp, "0" where no field is), each followed by delim, then
                           deleteCharAt(length - 1) (one UTF-16 unit of the delimiter).
     GEOHIP_FMT_WKT     <- PointToWKTOutputSchema.serialize     Serialization.java:72-92:
                           "<objID><delim> POINT(<x> <y>)<delim> <date>"<delim>  (objID part only
                           when not null, date part only when the timestamp is not 0).
     GEOHIP_FMT_GEOJSON <- PointToGeoJSONOutputSchema.serialize Serialization.java:28-50: org.json
                           20200518 (pom.xml:87-89) JSONObject.toString -- Java 8 HashMap key order,
                           numberToString, quote -- i.e.
                           {"geometry":{"coordinates":[x,y],"type":"Point"},"type":"Feature",
                            "properties":{"oID":"..","timestamp":".."}}  (properties only when
                           objID is not null or the timestamp is not 0).  A NaN / infinite
                           coordinate is GEOHIP_ERR_ARG (JSONObject.toString returns null there).
   The WKT / GeoJSON date is the caller's DateFormat: GEOHIP_DATE_YMD_HMS restates
   SimpleDateFormat("yyyy-MM-dd HH:mm:ss") (conf/geoflink-conf.yml:15) in a zone of fixed offset
   utc_offset_min; GEOHIP_DATE_NONE, or a year outside 1583..9999, makes a nonzero timestamp
   GEOHIP_ERR_UNSUPPORTED.  The delimiter is the schema's effective SEPARATION (the `\\t` config
   string is already mapped to the two characters `\t`, Serialization.java:62-66).
   rec_off (nullable, m + 1 entries) receives the record offsets.  Device memory only; *out_len
   (host) = the total bytes; GEOHIP_ERR_CAPACITY when above cap (records that do not fit entirely
   are not written). */
#define GEOHIP_DATE_NONE 0
#define GEOHIP_DATE_YMD_HMS 1
typedef struct geohip_text_out_spec {
    int32_t format;                            /* GEOHIP_FMT_CSV / _WKT / _GEOJSON */
    int32_t attr_oid, attr_ts, attr_x, attr_y; /* CSV: csvTsvSchemaAttr[0..3], each 0..63 */
    int32_t delim_len;                         /* CSV / WKT: 1..8 bytes (UTF-8) */
    char delim[8];
    int32_t date_format;                       /* GEOHIP_DATE_* (WKT / GeoJSON) */
    int32_t utc_offset_min;                    /* the DateFormat's zone: minutes east of UTC */
} geohip_text_out_spec;
int geohip_format_points(geohip_ctx* ctx, const geohip_text_out_spec* spec, const double* x,
                         const double* y, uint64_t n, const int64_t* ts, const uint8_t* oid_text,
                         const uint64_t* oid_off, const uint32_t* idx, uint64_t m, uint8_t* out,
                         uint64_t cap, uint64_t* out_len, uint64_t* rec_off);
/* The CSV/TSV schema alone (geohip_format_points with format GEOHIP_FMT_CSV). */
typedef struct geohip_csv_out_spec {
    int32_t attr_oid, attr_ts, attr_x, attr_y; /* csvTsvSchemaAttr[0..3], each 0..63 */
    int32_t delim_len;                         /* 1..8 */
    char delim[8];
    int32_t reserved;
} geohip_csv_out_spec;
int geohip_format_points_csv(geohip_ctx* ctx, const geohip_csv_out_spec* spec, const double* x,
                             const double* y, uint64_t n, const int64_t* ts, const uint8_t* oid_text,
                             const uint64_t* oid_off, const uint32_t* idx, uint64_t m, uint8_t* out,
                             uint64_t cap, uint64_t* out_len, uint64_t* rec_off);

/* ---- ingest codec ---------------------------------------------- */
/* A batch of '\n'-separated text records, as a Flink source hands them to the map functions of
   Deserialization.PointStream / TrajectoryStream (spatialStreams/Deserialization.java:47-80),
   parsed on the device into SoA coordinates:
     GEOHIP_FMT_CSV     <- CSVTSVToSpatial.map   Deserialization.java:248-254 (attr_ts = -1)
                           CSVTSVToTSpatial.map  Deserialization.java:306-321 (attr_ts = csvTsvSchemaAttr.get(1))
     GEOHIP_FMT_GEOJSON <- GeoJSONToSpatial.map  Deserialization.java:132-146 (one Kafka message value per line)
     GEOHIP_FMT_WKT     <- WKTToSpatial.map      Deserialization.java:223-228, getCoordinate :1510-1514
   and the Point constructor's cell (spatialObjects/Point.java:60-66 -> HelperClass.java:104-116)
   as out_cell[i] = cx * grid->n + cy for a valid key (0 <= cx, cy < n), else 0xffffffff.
   Record i is the i-th line; a final empty line (text ending in '\n') is not a record.
   Every parsed value is the double Double.parseDouble / the JSON and WKT readers produce
   (correctly rounded), for the whole Java grammar: decimal and hex significands, exponents of any
   length, type suffixes, quotes inside CSV tokens, 19-digit longs, a third WKT ordinate, NaN
   words.  Records the device does not decide -- malformed ones, where the reference throws, and
   forms whose Java behaviour is not restated (tokens of 100000+ characters, Z / M tags, POINT
   EMPTY) -- make the call return GEOHIP_ERR_UNSUPPORTED with *out_bad = the first such record;
   the caller hands that batch to the reference deserializer.
   GEOHIP_MEM_DEVICE: text (16-byte aligned) and outputs are device pointers.
   *out_count = number of records (GEOHIP_ERR_CAPACITY if > cap; outputs hold the first cap). */
#define GEOHIP_FMT_CSV 0
#define GEOHIP_FMT_GEOJSON 1
#define GEOHIP_FMT_WKT 2
typedef struct geohip_ingest_spec {
    int32_t format;  /* GEOHIP_FMT_* */
    int32_t delim;   /* CSV/TSV: the one-byte `delimiter` string (not a regex metacharacter) */
    int32_t attr_x;  /* csvTsvSchemaAttr.get(2) */
    int32_t attr_y;  /* csvTsvSchemaAttr.get(3) */
    int32_t attr_ts; /* csvTsvSchemaAttr.get(1) for CSVTSVToTSpatial (Long.valueOf), -1: none */
    int32_t attr_oid; /* csvTsvSchemaAttr.get(0), the objID field: read only by geohip_ingest_trajectory
                         with out_oid (geohip_ingest_points ignores it) */
} geohip_ingest_spec;
int geohip_ingest_points(geohip_ctx* ctx, const geohip_grid* grid, const geohip_ingest_spec* spec,
                         const char* text, uint64_t nbytes, double* out_x, double* out_y,
                         int64_t* out_ts /* nullable */, uint32_t* out_cell /* nullable */,
                         uint64_t cap, uint64_t* out_count, uint64_t* out_bad);

/* TrajectoryStream (Deserialization.java:64-80): every field of the Point the reference builds,
   Point(objID, x, y, timeStampMillisec, uGrid) (spatialObjects/Point.java:91-100):
     GEOHIP_FMT_CSV     <- CSVTSVToTSpatial.map Deserialization.java:306-321: objID = field attr_oid,
                           timestamp = Long.valueOf(field attr_ts) (attr_ts -1: 0);
     GEOHIP_FMT_GEOJSON <- GeoJSONToTSpatial.map Deserialization.java:149-208: timestamp =
                           traj->date_format's parse of properties[prop_ts] (GEOHIP_DATE_YMD_HMS:
                           SimpleDateFormat("yyyy-MM-dd HH:mm:ss"), conf/geoflink-conf.yml, in a zone
                           of fixed offset utc_offset_min; GEOHIP_DATE_NONE: 0), 0 where the reference
                           catches a ParseException; objID = properties[prop_oid].toString() with every
                           '"' deleted, null where properties or the key are absent;
     GEOHIP_FMT_WKT     <- WKTToTSpatial.map Deserialization.java:258-284: objID null, timestamp 0.
   out_oid[i] = record i's objID as a span of the text: (offset << 24) | length -- the bytes of the
   reference's String once the '"' among them are deleted -- or 0xffffff (length field all ones)
   for a null objID; geohip_ingest_oid_compact turns the spans into the (oid_text, oid_off) form
   the output codecs take.  Records whose objID or date form is not restated here (non-ASCII or
   escaped JSON strings, JSON numbers with fractions, lenient date forms such as one-digit
   fields, empty or control-character CSV objIDs) are GEOHIP_ERR_UNSUPPORTED like any record the
   device does not decide.  Other arguments and errors as geohip_ingest_points. */
typedef struct geohip_traj_spec {
    int32_t date_format;    /* GEOHIP_DATE_NONE / GEOHIP_DATE_YMD_HMS (GeoJSON) */
    int32_t utc_offset_min; /* the DateFormat's zone: minutes east of UTC */
    char prop_ts[60];       /* propertyTimeStamp (GeoJSON), NUL-terminated, <= 59 bytes */
    char prop_oid[60];      /* propertyObjID (GeoJSON), NUL-terminated, <= 59 bytes */
} geohip_traj_spec;
int geohip_ingest_trajectory(geohip_ctx* ctx, const geohip_grid* grid, const geohip_ingest_spec* spec,
                             const geohip_traj_spec* traj /* nullable for CSV / WKT */, const char* text,
                             uint64_t nbytes, double* out_x, double* out_y, int64_t* out_ts /* nullable */,
                             uint32_t* out_cell /* nullable */, uint64_t* out_oid /* nullable */,
                             uint64_t cap, uint64_t* out_count, uint64_t* out_bad);
/* objID spans (geohip_ingest_trajectory's out_oid, m records) over the same text -> the strings:
   out_text = their bytes with every '"' deleted, concatenated; out_off[0..m] = each record's start
   in out_text (out_off[m] = the total), bit 63 of out_off[i] set where record i's objID is null.
   The layout geohip_format_points / _csv take as (oid_text, oid_off).  Device memory only;
   *out_len (host) = total bytes, GEOHIP_ERR_CAPACITY when above cap (out_off written, out_text
   untouched). */
int geohip_ingest_oid_compact(geohip_ctx* ctx, const char* text, uint64_t nbytes, const uint64_t* oid_spans,
                              uint64_t m, uint8_t* out_text, uint64_t cap, uint64_t* out_off, uint64_t* out_len);

/* ---- host-side planning introspection (no device needed) ------------------------------ */
/* Query-cell sets of a point query as rectangles: point in G iff in any g rect; point in C
   iff in the c rect and not in G.  Returns GEOHIP_ERR_ARG where the reference throws. */
int geohip_plan_point(const geohip_grid* grid, double qx, double qy, double r,
                      geohip_rect* g_rects, uint32_t* n_g, geohip_rect* c_rect, uint32_t* n_c,
                      int32_t* layers_g, int32_t* layers_c);
/* Cell of a coordinate (HelperClass.assignGridCellID) computed by the planner. */
int geohip_plan_cell(const geohip_grid* grid, double x, double y, int32_t* cx, int32_t* cy);

/* ---- synthetic window generators (bench / tests), device pointers --------------------- */
/* x[i] = min_x + u(seed, 2(base+i)) * (max_x - min_x), y likewise with 2(base+i)+1, where
   u = (splitmix64(seed ^ k) >> 11) * 2^-53.  Bit-identical to spatialflink_amd.synth. */
int geohip_synth_uniform_async(geohip_ctx* ctx, double* x, double* y, uint64_t n, uint64_t base,
                               uint64_t seed, double min_x, double max_x, double min_y, double max_y);

#ifdef __cplusplus
}
#endif
#endif /* GEOHIP_H */
