/*
 * geohip_oracle.c -- CPU restatement of GeoFlink's windowed spatial query evaluation.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (libgeohip.so) never links or calls it.
 *
 * Independent of the product on purpose: cell sets are explicit hash sets filled by the
 * same loops as the Java code (UniformGrid.java:165-206, 261-293, 367-444 with Java int
 * wrap-around and validKey), cell keys are reasoned about as the "%05d%05d" strings of
 * HelperClass.java:54-63,104-120,263-276 (snprintf + a Java Integer.parseInt restatement),
 * the exact orientation sign uses __float128 (the product uses an fma expansion), and
 * kNN uses a bounded max-heap (the product uses wave-level bitonic selection).
 *
 * Third-party arithmetic (jts-core 1.16.1, pom.xml:60-64, not vendored) is restated from
 * its published algorithm: Coordinate.distance = Math.hypot = fdlibm e_hypot.c (JDK 8
 * StrictMath), DistanceOp min with Double.MAX_VALUE start, Distance.pointToSegment,
 * RayCrossingCounter.countSegment with RobustDeterminant.signOfDet2x2.
 * Parity: see DESIGN.md "Parity" -- grid/cell semantics pinned by known answers derived from
 * the Java source; distance bits "parity unpinned" (no JVM / JTS jar reachable).
 *
 * Build: gcc -O2 -std=c11 -ffp-contract=off -fPIC -shared (oracle/Makefile).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define OR_OK 0
#define OR_ERR_ARG -1       /* System.exit(1) / NumberFormatException in the reference */
#define OR_ERR_CAPACITY -2  /* output larger than cap (count still reported) */
#define OR_ERR_HANG -3      /* reference loop would not terminate (i <= INT_MAX) */
#define OR_ERR_OOM -4

typedef struct {
    double min_x, min_y, cell_len;
    int32_t n;
} or_grid;

/* ------------------------------------------------------------------------------------ */
/* Java scalar semantics                                                                 */
/* ------------------------------------------------------------------------------------ */
static int32_t j_d2i(double v) { /* JLS 5.1.3 */
    if (v != v) return 0;
    if (v >= 2147483647.0) return INT32_MAX;
    if (v <= -2147483648.0) return INT32_MIN;
    return (int32_t)v;
}
static int32_t wrap32(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }

int32_t geohip_oracle_d2i(double v) { return j_d2i(v); }

/* HelperClass.assignGridCellID(Coordinate, UniformGrid) (HelperClass.java:104-116) */
void geohip_oracle_cell(const or_grid* g, double x, double y, int32_t* cx, int32_t* cy) {
    *cx = j_d2i(floor((x - g->min_x) / g->cell_len));
    *cy = j_d2i(floor((y - g->min_y) / g->cell_len));
}

/* UniformGrid.getGuaranteedNeighboringLayers / getCandidateNeighboringLayers (:427-444) */
int32_t geohip_oracle_layers_guaranteed(const or_grid* g, double r) {
    double diag = g->cell_len * sqrt(2.0);
    return j_d2i(floor((r / diag) - 1));
}
int32_t geohip_oracle_layers_candidate(const or_grid* g, double r) {
    return j_d2i(ceil(r / g->cell_len));
}

/* Integer.parseInt(str.replaceFirst("^0+(?!$)", "")) (HelperClass.java:60-63). */
static int java_parse_int(const char* s0, int len, int32_t* out) {
    int i = 0;
    while (i < len - 1 && s0[i] == '0') i++; /* ^0+ but never the last char: (?!$) */
    const char* s = s0 + i;
    int n = len - i;
    if (n <= 0) return -1;
    int neg = 0, p = 0;
    if (s[0] == '-' || s[0] == '+') {
        if (n == 1) return -1;
        neg = s[0] == '-';
        p = 1;
    }
    int64_t v = 0;
    for (; p < n; p++) {
        if (s[p] < '0' || s[p] > '9') return -1;
        v = v * 10 + (s[p] - '0');
        if (v > 2147483648LL) return -1;
    }
    if (neg) v = -v;
    if (v < INT32_MIN || v > INT32_MAX) return -1;
    *out = (int32_t)v;
    return 0;
}

static int key_str(int32_t cx, int32_t cy, char* buf) {
    return snprintf(buf, 32, "%05d%05d", cx, cy);
}

/* HelperClass.getIntCellIndices(assignGridCellID(...)) round trip (HelperClass.java:263-276) */
int geohip_oracle_key_roundtrip(int32_t cx, int32_t cy, int32_t* px, int32_t* py) {
    char buf[32];
    int L = key_str(cx, cy, buf);
    if (java_parse_int(buf, 5, px) != 0) return OR_ERR_ARG;
    if (java_parse_int(buf + 5, L - 5, py) != 0) return OR_ERR_ARG;
    return OR_OK;
}

/* canonical "%05d" rendering check: is s[0..len) == fmt05(v) for some int v? */
static int canonical05(const char* s, int len, int32_t* v) {
    char tmp[32];
    if (len <= 0 || len > 11) return 0;
    int64_t acc = 0;
    int p = 0, neg = 0;
    if (s[0] == '-') { neg = 1; p = 1; }
    if (p >= len) return 0;
    for (int i = p; i < len; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        acc = acc * 10 + (s[i] - '0');
        if (acc > 2147483648LL) return 0;
    }
    if (neg) acc = -acc;
    if (acc < INT32_MIN || acc > INT32_MAX) return 0;
    snprintf(tmp, sizeof tmp, "%05d", (int32_t)acc);
    if ((int)strlen(tmp) != len || memcmp(tmp, s, (size_t)len) != 0) return 0;
    *v = (int32_t)acc;
    return 1;
}

/* All (cx,cy) whose "%05d%05d" key equals the key of (kx,ky).  Returns count (<= 13). */
int geohip_oracle_key_matches(int32_t kx, int32_t ky, int32_t* pairs, int max_pairs) {
    char buf[32];
    int L = key_str(kx, ky, buf), cnt = 0;
    for (int s = 5; s <= L - 5; s++) {
        int32_t a, b;
        if (canonical05(buf, s, &a) && canonical05(buf + s, L - s, &b)) {
            if (cnt < max_pairs) { pairs[2 * cnt] = a; pairs[2 * cnt + 1] = b; }
            cnt++;
        }
    }
    return cnt;
}

/* ------------------------------------------------------------------------------------ */
/* fdlibm e_hypot.c (JDK 8 StrictMath.hypot); JTS Coordinate.distance                   */
/* ------------------------------------------------------------------------------------ */
static inline int32_t HI(double d) { uint64_t u; memcpy(&u, &d, 8); return (int32_t)(u >> 32); }
static inline uint32_t LO(double d) { uint64_t u; memcpy(&u, &d, 8); return (uint32_t)u; }
static inline double SETHI(double d, int32_t hi) {
    uint64_t u; memcpy(&u, &d, 8);
    u = ((uint64_t)(uint32_t)hi << 32) | (u & 0xffffffffull);
    memcpy(&d, &u, 8); return d;
}
static inline double HIONLY(int32_t hi) { return SETHI(0.0, hi); }

double geohip_oracle_hypot(double x, double y) {
    double a, b, t1, t2, y1, y2, w;
    int32_t j, k, ha, hb;
    ha = HI(x) & 0x7fffffff;
    hb = HI(y) & 0x7fffffff;
    if (hb > ha) { a = y; b = x; j = ha; ha = hb; hb = j; } else { a = x; b = y; }
    a = SETHI(a, ha);
    b = SETHI(b, hb);
    if ((ha - hb) > 0x3c00000) return a + b;
    k = 0;
    if (ha > 0x5f300000) {
        if (ha >= 0x7ff00000) {
            w = a + b;
            if (((ha & 0xfffff) | LO(a)) == 0) w = a;
            if (((hb ^ 0x7ff00000) | LO(b)) == 0) w = b;
            return w;
        }
        ha -= 0x25800000; hb -= 0x25800000; k += 600;
        a = SETHI(a, ha);
        b = SETHI(b, hb);
    }
    if (hb < 0x20b00000) {
        if (hb <= 0x000fffff) {
            if ((hb | LO(b)) == 0) return a;
            t1 = HIONLY(0x7fd00000);
            b *= t1; a *= t1; k -= 1022;
        } else {
            ha += 0x25800000; hb += 0x25800000; k -= 600;
            a = SETHI(a, ha);
            b = SETHI(b, hb);
        }
    }
    w = a - b;
    if (w > b) {
        t1 = HIONLY(ha);
        t2 = a - t1;
        w = sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)));
    } else {
        a = a + a;
        y1 = HIONLY(hb);
        y2 = b - y1;
        t1 = HIONLY(ha + 0x00100000);
        t2 = a - t1;
        w = sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)));
    }
    if (k != 0) return HIONLY(0x3ff00000 + (k << 20)) * w;
    return w;
}

static inline double coord_dist(double ax, double ay, double bx, double by) {
    return geohip_oracle_hypot(ax - bx, ay - by);
}
/* DistanceOp.computeMinDistancePoints: minDistance = MAX_VALUE, replaced only if strictly less */
double geohip_oracle_pp_distance(double ax, double ay, double bx, double by) {
    double d = coord_dist(ax, ay, bx, by);
    return d < DBL_MAX ? d : DBL_MAX;
}

/* JTS Distance.pointToSegment */
double geohip_oracle_point_segment(double px, double py, double ax, double ay, double bx, double by) {
    if (ax == bx && ay == by) return coord_dist(px, py, ax, ay);
    double len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay);
    double r = ((px - ax) * (bx - ax) + (py - ay) * (by - ay)) / len2;
    if (r <= 0.0) return coord_dist(px, py, ax, ay);
    if (r >= 1.0) return coord_dist(px, py, bx, by);
    double s = ((ay - py) * (bx - ax) - (ax - px) * (by - ay)) / len2;
    return fabs(s) * sqrt(len2);
}

/* exact sign of x1*y2 - y1*x2 (RobustDeterminant.signOfDet2x2) via binary128 */
static int sign_det(double x1, double y1, double x2, double y2) {
    __float128 p = (__float128)x1 * (__float128)y2;
    __float128 q = (__float128)y1 * (__float128)x2;
    __float128 d = p - q;
    return (d > 0) - (d < 0);
}

/* RayCrossingCounter.locatePointInRing: 0 interior, 1 boundary, 2 exterior */
static int locate_in_ring(double px, double py, const double* vx, const double* vy, int nv) {
    int crossings = 0;
    for (int i = 1; i < nv; i++) {
        double p1x = vx[i], p1y = vy[i], p2x = vx[i - 1], p2y = vy[i - 1];
        if (p1x < px && p2x < px) continue;
        if (px == p2x && py == p2y) return 1;
        if (p1y == py && p2y == py) {
            double mn = p1x, mx = p2x;
            if (mn > mx) { mn = p2x; mx = p1x; }
            if (px >= mn && px <= mx) return 1;
            continue;
        }
        if ((p1y > py && p2y <= py) || (p2y > py && p1y <= py)) {
            double x1 = p1x - px, y1 = p1y - py, x2 = p2x - px, y2 = p2y - py;
            int s = sign_det(x1, y1, x2, y2);
            if (s == 0) return 1;
            if (y2 < y1) s = -s;
            if (s > 0) crossings++;
        }
    }
    return (crossings & 1) ? 0 : 2;
}

typedef struct { double minx, miny, maxx, maxy; } or_env;

static or_env ring_env(const double* vx, const double* vy, int nv) {
    or_env e = {0, 0, -1, 0};
    for (int i = 0; i < nv; i++) {
        if (i == 0) { e.minx = e.maxx = vx[i]; e.miny = e.maxy = vy[i]; continue; }
        if (vx[i] < e.minx) e.minx = vx[i];
        if (vx[i] > e.maxx) e.maxx = vx[i];
        if (vy[i] < e.miny) e.miny = vy[i];
        if (vy[i] > e.maxy) e.maxy = vy[i];
    }
    return e;
}

/* point.distance(polygon) through JTS DistanceOp (shell only) */
double geohip_oracle_point_polygon(double px, double py, const double* vx, const double* vy, int nv) {
    or_env e = ring_env(vx, vy, nv);
    int inside_env = !(px > e.maxx || px < e.minx || py > e.maxy || py < e.miny);
    if (inside_env && locate_in_ring(px, py, vx, vy, nv) != 2) return 0.0;
    double md = DBL_MAX;
    for (int i = 0; i < nv - 1; i++) {
        double d = geohip_oracle_point_segment(px, py, vx[i], vy[i], vx[i + 1], vy[i + 1]);
        if (d < md) md = d;
        if (md <= 0.0) return md;
    }
    return md;
}

/* DistanceFunctions.getPointPointEuclideanDistance (:60-63) and bbox distance (:134-200) */
static double pp_euclid(double lon, double lat, double lon1, double lat1) {
    double dy = lat1 - lat, dx = lon1 - lon;
    return sqrt(dy * dy + dx * dx);
}
static double bbox_border(double x, double y, double x1, double y1, double x2, double y2) {
    if (x1 == x2) return pp_euclid(x, y, x1, y);
    else if (y1 == y2) return pp_euclid(x, y, x, y1);
    return 4.9e-324;
}
double geohip_oracle_bbox_distance(double x, double y, double x1, double y1, double x2, double y2) {
    if (x <= x1) {
        if (y <= y1) return pp_euclid(x, y, x1, y1);
        else if (y >= y2) return pp_euclid(x, y, x1, y2);
        return bbox_border(x, y, x1, y1, x1, y2);
    } else if (x >= x2) {
        if (y <= y1) return pp_euclid(x, y, x2, y1);
        else if (y >= y2) return pp_euclid(x, y, x2, y2);
        return bbox_border(x, y, x2, y1, x2, y2);
    } else {
        if (y <= y1) return bbox_border(x, y, x1, y1, x2, y1);
        else if (y >= y2) return bbox_border(x, y, x1, y2, x2, y2);
        return 0.0;
    }
}

/* ------------------------------------------------------------------------------------ */
/* cell sets (open addressing over packed (cx,cy))                                       */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint64_t* slot; uint64_t cap, cnt; } cset;
#define EMPTY_SLOT 0xffffffffffffffffull /* (-1,-1) packed is never inserted as EMPTY */

static uint64_t pack(int32_t x, int32_t y) { return ((uint64_t)(uint32_t)x << 32) | (uint32_t)y; }
static uint64_t hmix(uint64_t k) { k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; return k; }

static int cs_init(cset* s) {
    s->cap = 64; s->cnt = 0;
    s->slot = (uint64_t*)malloc(s->cap * 8);
    if (!s->slot) return -1;
    memset(s->slot, 0xff, s->cap * 8);
    return 0;
}
static void cs_free(cset* s) { free(s->slot); s->slot = NULL; }
static int cs_has_packed(const cset* s, uint64_t k) {
    if (k == EMPTY_SLOT) { /* (-1,-1) stored out of band in bit 0 of cnt? keep simple: linear */ }
    uint64_t m = s->cap - 1, h = hmix(k) & m;
    while (s->slot[h] != EMPTY_SLOT) {
        if (s->slot[h] == k) return 1;
        h = (h + 1) & m;
    }
    return 0;
}
static int cs_add_packed(cset* s, uint64_t k);
static int cs_grow(cset* s) {
    cset n; n.cap = s->cap * 2; n.cnt = 0;
    n.slot = (uint64_t*)malloc(n.cap * 8);
    if (!n.slot) return -1;
    memset(n.slot, 0xff, n.cap * 8);
    for (uint64_t i = 0; i < s->cap; i++) if (s->slot[i] != EMPTY_SLOT) cs_add_packed(&n, s->slot[i]);
    free(s->slot); *s = n;
    return 0;
}
static int cs_add_packed(cset* s, uint64_t k) {
    if ((s->cnt + 1) * 2 > s->cap && cs_grow(s)) return -1;
    uint64_t m = s->cap - 1, h = hmix(k) & m;
    while (s->slot[h] != EMPTY_SLOT) {
        if (s->slot[h] == k) return 0;
        h = (h + 1) & m;
    }
    s->slot[h] = k; s->cnt++;
    return 0;
}
/* (-1,-1) packs to EMPTY_SLOT; such a key can only come from a Lg==0 query key and only
   matches points in cell (-1,-1); track it with a flag */
typedef struct { cset s; int has_m1m1; } cellset;
static int cl_init(cellset* c) { c->has_m1m1 = 0; return cs_init(&c->s); }
static void cl_free(cellset* c) { cs_free(&c->s); }
static int cl_add(cellset* c, int32_t x, int32_t y) {
    uint64_t k = pack(x, y);
    if (k == EMPTY_SLOT) { c->has_m1m1 = 1; return 0; }
    return cs_add_packed(&c->s, k);
}
static int cl_has(const cellset* c, int32_t x, int32_t y) {
    uint64_t k = pack(x, y);
    if (k == EMPTY_SLOT) return c->has_m1m1;
    return cs_has_packed(&c->s, k);
}
/* add the cells whose key string equals the key of (kx,ky) */
static int cl_add_key(cellset* c, int32_t kx, int32_t ky) {
    int32_t pairs[2 * 16];
    int n = geohip_oracle_key_matches(kx, ky, pairs, 16);
    for (int i = 0; i < n && i < 16; i++)
        if (cl_add(c, pairs[2 * i], pairs[2 * i + 1])) return -1;
    return 0;
}

/* square of `layers` around (ci,cj) with Java int wrap; validKey; optional exclusion */
static int add_square(const or_grid* g, cellset* out, int32_t ci, int32_t cj, int32_t layers,
                      const cellset* excl) {
    int32_t lo_i = wrap32((int64_t)ci - layers), hi_i = wrap32((int64_t)ci + layers);
    int32_t lo_j = wrap32((int64_t)cj - layers), hi_j = wrap32((int64_t)cj + layers);
    if (lo_i > hi_i || lo_j > hi_j) return 0;
    if (hi_i == INT32_MAX || hi_j == INT32_MAX) return OR_ERR_HANG;
    /* the Java loops visit all (i,j) and keep validKey(i,j); same set */
    int64_t a0 = lo_i > 0 ? lo_i : 0, a1 = hi_i < g->n - 1 ? hi_i : g->n - 1;
    int64_t b0 = lo_j > 0 ? lo_j : 0, b1 = hi_j < g->n - 1 ? hi_j : g->n - 1;
    for (int64_t i = a0; i <= a1; i++)
        for (int64_t j = b0; j <= b1; j++) {
            if (excl && cl_has(excl, (int32_t)i, (int32_t)j)) continue;
            if (cl_add(out, (int32_t)i, (int32_t)j)) return OR_ERR_OOM;
        }
    return 0;
}

/* getGuaranteedNeighboringCells(r, key(kx,ky)) (UniformGrid.java:165-190) */
static int add_guaranteed(const or_grid* g, cellset* G, double r, int32_t kx, int32_t ky) {
    int32_t lg = geohip_oracle_layers_guaranteed(g, r);
    if (lg == 0) return cl_add_key(G, kx, ky) ? OR_ERR_OOM : 0;
    if (lg > 0) {
        int32_t ci, cj;
        if (geohip_oracle_key_roundtrip(kx, ky, &ci, &cj)) return OR_ERR_ARG;
        return add_square(g, G, ci, cj, lg, NULL);
    }
    return 0;
}
/* getCandidateNeighboringCells(r, key(kx,ky), G) (UniformGrid.java:367-394) */
static int add_candidate(const or_grid* g, cellset* C, const cellset* G, double r, int32_t kx, int32_t ky) {
    int32_t lc = geohip_oracle_layers_candidate(g, r);
    if (lc > 0) {
        int32_t ci, cj;
        if (geohip_oracle_key_roundtrip(kx, ky, &ci, &cj)) return OR_ERR_ARG;
        return add_square(g, C, ci, cj, lc, G);
    }
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* window queries                                                                        */
/* ------------------------------------------------------------------------------------ */
/* PointPointRangeQuery window body (PointPointRangeQuery.java:86-137). */
int64_t geohip_oracle_range_pp(const or_grid* g, const double* x, const double* y, uint64_t n,
                               double qx, double qy, double r, int approximate,
                               uint32_t* out_idx, uint64_t cap) {
    cellset G, C;
    int32_t qcx, qcy;
    if (g->n <= 0 || g->n > 99999 || !(g->cell_len > 0)) return OR_ERR_ARG;
    geohip_oracle_cell(g, qx, qy, &qcx, &qcy);
    cl_init(&G); cl_init(&C);
    int rc = add_guaranteed(g, &G, r, qcx, qcy);
    if (!rc) rc = add_candidate(g, &C, &G, r, qcx, qcy);
    if (rc) { cl_free(&G); cl_free(&C); return rc; }
    uint64_t cnt = 0;
    for (uint64_t i = 0; i < n; i++) {
        int32_t cx, cy;
        geohip_oracle_cell(g, x[i], y[i], &cx, &cy);
        int inG = cl_has(&G, cx, cy);
        if (!inG && !cl_has(&C, cx, cy)) continue;
        int emit = inG || approximate || geohip_oracle_pp_distance(qx, qy, x[i], y[i]) <= r;
        if (emit) { if (cnt < cap) out_idx[cnt] = (uint32_t)i; cnt++; }
    }
    cl_free(&G); cl_free(&C);
    return (int64_t)cnt;
}

typedef struct { double d; uint32_t i; } kent;
static int kless(kent a, kent b) { return a.d < b.d || (a.d == b.d && a.i < b.i); }
static void heap_down(kent* h, int n, int k) { /* max-heap on (d,i) */
    for (;;) {
        int l = 2 * k + 1, r = l + 1, m = k;
        if (l < n && kless(h[m], h[l])) m = l;
        if (r < n && kless(h[m], h[r])) m = r;
        if (m == k) return;
        kent t = h[k]; h[k] = h[m]; h[m] = t; k = m;
    }
}
static void heap_up(kent* h, int k) {
    while (k > 0) {
        int p = (k - 1) / 2;
        if (!kless(h[p], h[k])) return;
        kent t = h[k]; h[k] = h[p]; h[p] = t; k = p;
    }
}
static int kcmp(const void* a, const void* b) {
    kent x = *(const kent*)a, y = *(const kent*)b;
    return kless(x, y) ? -1 : kless(y, x) ? 1 : 0;
}

/* kNN build contract: k smallest (dist, idx) over G u C, ascending;
   per-cell heaps + windowAll merge (PointPointKNNQuery.java:125-191, KNNQuery.java:214-271)
   yield the same set for unique ids with no exact tie straddling rank k. */
int geohip_oracle_knn_pp(const or_grid* g, const double* x, const double* y, uint64_t n,
                         double qx, double qy, double r, uint32_t k,
                         uint32_t* out_idx, double* out_dist, uint32_t* out_count) {
    cellset G, C;
    int32_t qcx, qcy;
    *out_count = 0;
    if (g->n <= 0 || g->n > 99999 || !(g->cell_len > 0) || k == 0) return OR_ERR_ARG;
    geohip_oracle_cell(g, qx, qy, &qcx, &qcy);
    cl_init(&G); cl_init(&C);
    int rc = add_guaranteed(g, &G, r, qcx, qcy);
    if (!rc) rc = add_candidate(g, &C, &G, r, qcx, qcy);
    if (rc) { cl_free(&G); cl_free(&C); return rc; }
    kent* h = (kent*)malloc(sizeof(kent) * k);
    int hn = 0;
    for (uint64_t i = 0; i < n; i++) {
        int32_t cx, cy;
        geohip_oracle_cell(g, x[i], y[i], &cx, &cy);
        if (!cl_has(&G, cx, cy) && !cl_has(&C, cx, cy)) continue;
        kent e = {geohip_oracle_pp_distance(qx, qy, x[i], y[i]), (uint32_t)i};
        if (hn < (int)k) { h[hn] = e; heap_up(h, hn); hn++; }
        else if (kless(e, h[0])) { h[0] = e; heap_down(h, hn, 0); }
    }
    qsort(h, (size_t)hn, sizeof(kent), kcmp);
    for (int i = 0; i < hn; i++) { out_idx[i] = h[i].i; out_dist[i] = h[i].d; }
    *out_count = (uint32_t)hn;
    free(h); cl_free(&G); cl_free(&C);
    return OR_OK;
}

/* PointPointJoinQuery window join (PointPointJoinQuery.java:113-172) with
   JoinQuery.getReplicatedPointQueryStream (JoinQuery.java:73-90) and
   UniformGrid.getNeighboringCells (UniformGrid.java:261-293).  Pairs (p_idx, q_idx). */
int64_t geohip_oracle_join_pp(const or_grid* gd, const or_grid* gq, const double* dx, const double* dy,
                              uint64_t nd, const double* qx, const double* qy, uint64_t nq, double r,
                              int approximate, uint32_t* out_pairs, uint64_t cap) {
    if (gd->n <= 0 || gq->n <= 0 || gq->n > 99999 || gd->n > 99999) return OR_ERR_ARG;
    int32_t lc = geohip_oracle_layers_candidate(gq, r);
    int all = (r == 0);
    if (!all && lc <= 0) return OR_ERR_ARG; /* System.exit(1) at UniformGrid.java:272-276 */
    int64_t ncell = (int64_t)gq->n * gq->n;
    /* CSR: valid q-grid cell -> queries replicated there */
    uint32_t* cnt = (uint32_t*)calloc((size_t)ncell + 1, 4);
    if (!cnt) return OR_ERR_OOM;
    uint32_t* list = NULL;
    uint32_t* fill = NULL;
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 1) {
            for (int64_t c = 0, acc = 0; c <= ncell; c++) { uint32_t t = cnt[c]; cnt[c] = (uint32_t)acc; acc += t; }
            list = (uint32_t*)malloc(sizeof(uint32_t) * (cnt[ncell] + 1));
            fill = (uint32_t*)calloc((size_t)ncell, 4);
        }
        for (uint64_t q = 0; q < nq; q++) {
            int32_t ci, cj, a0, a1, b0, b1;
            if (all) { a0 = 0; a1 = gq->n - 1; b0 = 0; b1 = gq->n - 1; }
            else {
                int32_t kx, ky;
                geohip_oracle_cell(gq, qx[q], qy[q], &kx, &ky);
                if (geohip_oracle_key_roundtrip(kx, ky, &ci, &cj)) { free(cnt); free(list); free(fill); return OR_ERR_ARG; }
                int32_t lo_i = wrap32((int64_t)ci - lc), hi_i = wrap32((int64_t)ci + lc);
                int32_t lo_j = wrap32((int64_t)cj - lc), hi_j = wrap32((int64_t)cj + lc);
                if (lo_i > hi_i || lo_j > hi_j) continue;
                if (hi_i == INT32_MAX || hi_j == INT32_MAX) { free(cnt); free(list); free(fill); return OR_ERR_HANG; }
                a0 = lo_i > 0 ? lo_i : 0; a1 = hi_i < gq->n - 1 ? hi_i : gq->n - 1;
                b0 = lo_j > 0 ? lo_j : 0; b1 = hi_j < gq->n - 1 ? hi_j : gq->n - 1;
            }
            for (int64_t i = a0; i <= a1; i++)
                for (int64_t j = b0; j <= b1; j++) {
                    int64_t c = i * gq->n + j;
                    if (pass == 0) cnt[c]++;
                    else list[cnt[c] + fill[c]++] = (uint32_t)q;
                }
        }
        if (pass == 1) {
            uint64_t out = 0;
            for (uint64_t p = 0; p < nd; p++) {
                int32_t cx, cy;
                geohip_oracle_cell(gd, dx[p], dy[p], &cx, &cy);
                /* data key (uGrid) must equal a replicated key (valid in qGrid) */
                if (cx < 0 || cy < 0 || cx >= gq->n || cy >= gq->n) continue;
                int64_t c = (int64_t)cx * gq->n + cy;
                for (uint32_t t = cnt[c]; t < cnt[c + 1]; t++) {
                    uint32_t q = list[t];
                    if (approximate || geohip_oracle_pp_distance(dx[p], dy[p], qx[q], qy[q]) <= r) {
                        if (out < cap) { out_pairs[2 * out] = (uint32_t)p; out_pairs[2 * out + 1] = q; }
                        out++;
                    }
                }
            }
            free(list); free(fill); free(cnt);
            return (int64_t)out;
        }
    }
    free(cnt);
    return OR_ERR_ARG;
}

/* One query polygon as the reference builds it: ring closed (Polygon.java:147-155), JTS
   envelope, gridIDsSet = bbox cells on grid g unclipped (HelperClass.java:123-143), then
   G = union of guaranteed squares, C = union of candidate squares minus G
   (UniformGrid.java:193-206, 398-410).  rx/ry get nv+1 slots; returns OR_OK or an error. */
typedef struct { double* rx; double* ry; int nv; or_env env; cellset G, C; } or_poly;
static void poly_free(or_poly* P) { cl_free(&P->G); cl_free(&P->C); free(P->rx); free(P->ry); }
static int poly_prep(const or_grid* g, const double* vx, const double* vy, int nv, double r, or_poly* P) {
    if (nv <= 3) return OR_ERR_ARG; /* Polygon.java:53 */
    P->rx = (double*)malloc(sizeof(double) * (nv + 1));
    P->ry = (double*)malloc(sizeof(double) * (nv + 1));
    memcpy(P->rx, vx, sizeof(double) * nv);
    memcpy(P->ry, vy, sizeof(double) * nv);
    if (!(P->rx[0] == P->rx[nv - 1] && P->ry[0] == P->ry[nv - 1])) { P->rx[nv] = P->rx[0]; P->ry[nv] = P->ry[0]; nv++; }
    P->nv = nv;
    P->env = ring_env(P->rx, P->ry, nv);
    cl_init(&P->G); cl_init(&P->C);
    int32_t x1 = j_d2i(floor((P->env.minx - g->min_x) / g->cell_len));
    int32_t y1 = j_d2i(floor((P->env.miny - g->min_y) / g->cell_len));
    int32_t x2 = j_d2i(floor((P->env.maxx - g->min_x) / g->cell_len));
    int32_t y2 = j_d2i(floor((P->env.maxy - g->min_y) / g->cell_len));
    if (x2 == INT32_MAX || y2 == INT32_MAX) { poly_free(P); return OR_ERR_HANG; }
    int rc = 0;
    for (int64_t a = x1; a <= x2 && !rc; a++)
        for (int64_t c = y1; c <= y2 && !rc; c++) rc = add_guaranteed(g, &P->G, r, (int32_t)a, (int32_t)c);
    for (int64_t a = x1; a <= x2 && !rc; a++)
        for (int64_t c = y1; c <= y2 && !rc; c++) rc = add_candidate(g, &P->C, &P->G, r, (int32_t)a, (int32_t)c);
    if (rc) poly_free(P);
    return rc;
}

/* PointPolygonRangeQuery window body (PointPolygonRangeQuery.java:76-124) for npoly
   independent single-ring polygons (ring_off[npoly+1] into vx/vy; rings given as the
   caller's coordinate list, closed here per Polygon.java:147-155).  Pairs (poly, pt). */
int64_t geohip_oracle_range_ppoly(const or_grid* g, const double* x, const double* y, uint64_t n,
                                  const uint32_t* ring_off, const double* vx, const double* vy,
                                  uint32_t npoly, double r, int approximate,
                                  uint32_t* out_pairs, uint64_t cap) {
    if (g->n <= 0 || g->n > 99999 || !(g->cell_len > 0)) return OR_ERR_ARG;
    uint64_t out = 0;
    for (uint32_t pi = 0; pi < npoly; pi++) {
        or_poly P;
        int rc = poly_prep(g, vx + ring_off[pi], vy + ring_off[pi], (int)(ring_off[pi + 1] - ring_off[pi]), r, &P);
        if (rc) return rc;
        for (uint64_t i = 0; i < n; i++) {
            int32_t cx, cy;
            geohip_oracle_cell(g, x[i], y[i], &cx, &cy);
            int inG = cl_has(&P.G, cx, cy);
            if (!inG && !cl_has(&P.C, cx, cy)) continue;
            int emit = inG;
            if (!emit) {
                double d = approximate
                    ? geohip_oracle_bbox_distance(x[i], y[i], P.env.minx, P.env.miny, P.env.maxx, P.env.maxy)
                    : geohip_oracle_point_polygon(x[i], y[i], P.rx, P.ry, P.nv);
                emit = d <= r;
            }
            if (emit) {
                if (out < cap) { out_pairs[2 * out] = pi; out_pairs[2 * out + 1] = (uint32_t)i; }
                out++;
            }
        }
        poly_free(&P);
    }
    return (int64_t)out;
}

/* PointPolygonJoinQuery window join (PointPolygonJoinQuery.java:162-201) with the polygon
   stream replicated to its G and C cells on the query grid (JoinQuery.getReplicatedPolygonQueryStream,
   JoinQuery.java:93-115): a point joins a polygon iff its gridID (point grid) equals one of
   them, and approximate or JTS distance <= r.  No guaranteed-cell shortcut.  Pairs (pt, poly). */
int64_t geohip_oracle_join_ppoly(const or_grid* gp, const or_grid* gq, const double* x, const double* y, uint64_t n,
                                 const uint32_t* ring_off, const double* vx, const double* vy,
                                 uint32_t npoly, double r, int approximate,
                                 uint32_t* out_pairs, uint64_t cap) {
    if (gp->n <= 0 || gp->n > 99999 || !(gp->cell_len > 0)) return OR_ERR_ARG;
    if (gq->n <= 0 || gq->n > 99999 || !(gq->cell_len > 0)) return OR_ERR_ARG;
    uint64_t out = 0;
    int32_t* pc = (int32_t*)malloc(sizeof(int32_t) * 2 * (n ? n : 1));
    if (!pc) return OR_ERR_OOM;
    for (uint64_t i = 0; i < n; i++) geohip_oracle_cell(gp, x[i], y[i], &pc[2 * i], &pc[2 * i + 1]);
    for (uint32_t pi = 0; pi < npoly; pi++) {
        or_poly P;
        int rc = poly_prep(gq, vx + ring_off[pi], vy + ring_off[pi], (int)(ring_off[pi + 1] - ring_off[pi]), r, &P);
        if (rc) { free(pc); return rc; }
        for (uint64_t i = 0; i < n; i++) {
            int32_t cx = pc[2 * i], cy = pc[2 * i + 1];
            if (!cl_has(&P.G, cx, cy) && !cl_has(&P.C, cx, cy)) continue;
            if (approximate || geohip_oracle_point_polygon(x[i], y[i], P.rx, P.ry, P.nv) <= r) {
                if (out < cap) { out_pairs[2 * out] = (uint32_t)i; out_pairs[2 * out + 1] = pi; }
                out++;
            }
        }
        poly_free(&P);
    }
    free(pc);
    return (int64_t)out;
}

/* PointPolygonKNNQuery window body (PointPolygonKNNQuery.java:162-236): candidates are the
   points of G u C of the query polygon, distance = JTS point.distance(polygon) (or the bbox
   distance, DistanceFunctions.java:150-200, when approximate); no radius filter; same
   build contract as geohip_oracle_knn_pp: the k smallest (dist, idx), ascending. */
/* (distance bits, idx) keys: for the non-negative distances of this path the bit order is the
   value order; a NaN (the approximate bbox distance of a NaN coordinate) is canonicalised to
   0x7ff8000000000000 and so ranks after +Infinity -- the total order the device selects by. */
typedef struct { uint64_t d; uint32_t i; } kbent;
static int kbless(kbent a, kbent b) { return a.d < b.d || (a.d == b.d && a.i < b.i); }
static void kb_down(kbent* h, int n, int k) {
    for (;;) {
        int l = 2 * k + 1, r = l + 1, m = k;
        if (l < n && kbless(h[m], h[l])) m = l;
        if (r < n && kbless(h[m], h[r])) m = r;
        if (m == k) return;
        kbent t = h[k]; h[k] = h[m]; h[m] = t; k = m;
    }
}
static void kb_up(kbent* h, int k) {
    while (k > 0) {
        int p = (k - 1) / 2;
        if (!kbless(h[p], h[k])) return;
        kbent t = h[k]; h[k] = h[p]; h[p] = t; k = p;
    }
}
static int kbcmp(const void* a, const void* b) {
    kbent x = *(const kbent*)a, y = *(const kbent*)b;
    return kbless(x, y) ? -1 : kbless(y, x) ? 1 : 0;
}

int geohip_oracle_knn_ppoly(const or_grid* g, const double* x, const double* y, uint64_t n,
                            const double* vx, const double* vy, uint32_t nv, double r, uint32_t k,
                            int approximate, uint32_t* out_idx, double* out_dist, uint32_t* out_count) {
    *out_count = 0;
    if (g->n <= 0 || g->n > 99999 || !(g->cell_len > 0) || k == 0) return OR_ERR_ARG;
    or_poly P;
    int rc = poly_prep(g, vx, vy, (int)nv, r, &P);
    if (rc) return rc;
    kbent* h = (kbent*)malloc(sizeof(kbent) * k);
    int hn = 0;
    for (uint64_t i = 0; i < n; i++) {
        int32_t cx, cy;
        geohip_oracle_cell(g, x[i], y[i], &cx, &cy);
        if (!cl_has(&P.G, cx, cy) && !cl_has(&P.C, cx, cy)) continue;
        double d = approximate
            ? geohip_oracle_bbox_distance(x[i], y[i], P.env.minx, P.env.miny, P.env.maxx, P.env.maxy)
            : geohip_oracle_point_polygon(x[i], y[i], P.rx, P.ry, P.nv);
        uint64_t bits;
        memcpy(&bits, &d, 8);
        if (d != d) bits = 0x7ff8000000000000ull;
        kbent e = {bits, (uint32_t)i};
        if (hn < (int)k) { h[hn] = e; kb_up(h, hn); hn++; }
        else if (kbless(e, h[0])) { h[0] = e; kb_down(h, hn, 0); }
    }
    qsort(h, (size_t)hn, sizeof(kbent), kbcmp);
    for (int i = 0; i < hn; i++) { out_idx[i] = h[i].i; memcpy(&out_dist[i], &h[i].d, 8); }
    *out_count = (uint32_t)hn;
    free(h);
    poly_free(&P);
    return OR_OK;
}
