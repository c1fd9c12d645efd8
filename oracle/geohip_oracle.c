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
#ifdef _OPENMP
#include <omp.h>
#endif

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

/* Envelope.distance(Envelope) of a ring envelope to a point's (JTS 1.16.1): the ring skip test
   of DistanceOp.computeMinDistance(LineString, Point). */
static double env_point_distance(or_env e, double px, double py) {
    if (!(px > e.maxx || px < e.minx || py > e.maxy || py < e.miny)) return 0.0;
    double dx = 0.0, dy = 0.0;
    if (e.maxx < px) dx = px - e.maxx;
    else if (e.minx > px) dx = e.minx - px;
    if (e.maxy < py) dy = py - e.maxy;
    else if (e.miny > py) dy = e.miny - py;
    if (dx == 0.0) return dy;
    if (dy == 0.0) return dx;
    return sqrt(dx * dx + dy * dy);
}

/* PointLocator.locateInPolygonRing: envelope test, then the ray-crossing count */
static int ring_location(double px, double py, const double* vx, const double* vy, int nv, or_env e) {
    if (px > e.maxx || px < e.minx || py > e.maxy || py < e.miny) return 2;
    return locate_in_ring(px, py, vx, vy, nv);
}

/* point.distance(polygon) through JTS DistanceOp for a polygon of nring closed rings (ring 0 =
   shell, then holes; ring j = [roff[j], roff[j+1]) of vx/vy, envelopes renv[j]):
   PointLocator.locateInPolygon (shell EXTERIOR -> exterior, BOUNDARY -> boundary; each hole in
   order: INTERIOR -> exterior, BOUNDARY -> boundary), not exterior -> 0; else the minimum over
   the rings' segments (shell first), a ring skipped when its envelope is farther than the
   current minimum, MAX_VALUE start, strict <, stop at 0. */
static double poly_rings_distance(double px, double py, const double* vx, const double* vy, const int* roff,
                                  const or_env* renv, int nring) {
    int loc = ring_location(px, py, vx + roff[0], vy + roff[0], roff[1] - roff[0], renv[0]);
    if (loc == 1) return 0.0;
    if (loc == 0) {
        for (int h = 1; h < nring; h++) {
            int lh = ring_location(px, py, vx + roff[h], vy + roff[h], roff[h + 1] - roff[h], renv[h]);
            if (lh == 0) { loc = 2; break; }
            if (lh == 1) return 0.0;
        }
        if (loc == 0) return 0.0;
    }
    double md = DBL_MAX;
    for (int j = 0; j < nring; j++) {
        if (env_point_distance(renv[j], px, py) > md) continue;
        for (int i = roff[j]; i < roff[j + 1] - 1; i++) {
            double d = geohip_oracle_point_segment(px, py, vx[i], vy[i], vx[i + 1], vy[i + 1]);
            if (d < md) md = d;
            if (md <= 0.0) return md;
        }
    }
    return md;
}

/* point.distance(polygon) of a shell-only polygon (one closed ring) */
double geohip_oracle_point_polygon(double px, double py, const double* vx, const double* vy, int nv) {
    int roff[2] = {0, nv};
    or_env e = ring_env(vx, vy, nv);
    return poly_rings_distance(px, py, vx, vy, roff, &e, 1);
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
/* Order-independent 64-bit digest of an output set: sum over elements of mix64(element). */
static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t geohip_oracle_mix64(uint64_t z) { return mix64(z); }

static int g_threads = 0; /* 0: OpenMP default (OMP_NUM_THREADS) */
void geohip_oracle_set_threads(int t) { g_threads = t > 0 ? t : 0; }
static int nthreads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}
int geohip_oracle_threads(void) { return nthreads(); }

/* PointPointRangeQuery window body (PointPointRangeQuery.java:86-137): the per-point predicate
   evaluated over the window (points in parallel), hits in ascending index order.
   hash (nullable): sum of mix64(idx) over the hits. */
int64_t geohip_oracle_range_pp(const or_grid* g, const double* x, const double* y, uint64_t n,
                               double qx, double qy, double r, int approximate,
                               uint32_t* out_idx, uint64_t cap, uint64_t* hash) {
    cellset G, C;
    int32_t qcx, qcy;
    if (g->n <= 0 || g->n > 99999 || !(g->cell_len > 0)) return OR_ERR_ARG;
    geohip_oracle_cell(g, qx, qy, &qcx, &qcy);
    cl_init(&G); cl_init(&C);
    int rc = add_guaranteed(g, &G, r, qcx, qcy);
    if (!rc) rc = add_candidate(g, &C, &G, r, qcx, qcy);
    if (rc) { cl_free(&G); cl_free(&C); return rc; }
    uint8_t* hit = (uint8_t*)malloc(n ? n : 1);
    if (!hit) { cl_free(&G); cl_free(&C); return OR_ERR_OOM; }
    uint64_t h = 0;
#pragma omp parallel for schedule(static) num_threads(nthreads()) reduction(+ : h)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        int32_t cx, cy;
        geohip_oracle_cell(g, x[i], y[i], &cx, &cy);
        int inG = cl_has(&G, cx, cy);
        int emit = 0;
        if (inG || cl_has(&C, cx, cy))  /* filter :102-107 */
            emit = inG || approximate || geohip_oracle_pp_distance(qx, qy, x[i], y[i]) <= r;
        hit[i] = (uint8_t)emit;
        if (emit) h += mix64((uint64_t)i);
    }
    uint64_t cnt = 0;
    for (uint64_t i = 0; i < n; i++)
        if (hit[i]) { if (cnt < cap) out_idx[cnt] = (uint32_t)i; cnt++; }
    free(hit);
    if (hash) *hash = h;
    cl_free(&G); cl_free(&C);
    return (int64_t)cnt;
}

typedef struct { double d; uint32_t i; } kent;
/* (distance, idx) order by the distance's bit pattern: the value order for the non-negative
   distances of this path, NaN after +Infinity (the device's total order) */
static inline uint64_t dbits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static int kless(kent a, kent b) {
    uint64_t x = dbits(a.d), y = dbits(b.d);
    return x < y || (x == y && a.i < b.i);
}
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
static void heap_offer(kent* h, int* hn, uint32_t k, kent e) {
    if (*hn < (int)k) { h[*hn] = e; heap_up(h, *hn); (*hn)++; }
    else if (kless(e, h[0])) { h[0] = e; heap_down(h, *hn, 0); }
}

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
    const int T = nthreads();
    kent* hs = (kent*)malloc(sizeof(kent) * (size_t)k * T);
    int* hns = (int*)calloc((size_t)T, sizeof(int));
#pragma omp parallel num_threads(T)
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num();
#else
        const int t = 0;
#endif
        kent* h = hs + (size_t)k * t;
        int hn = 0;
#pragma omp for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; i++) {
            int32_t cx, cy;
            geohip_oracle_cell(g, x[i], y[i], &cx, &cy);
            if (!cl_has(&G, cx, cy) && !cl_has(&C, cx, cy)) continue;
            kent e = {geohip_oracle_pp_distance(qx, qy, x[i], y[i]), (uint32_t)i};
            heap_offer(h, &hn, k, e);
        }
        hns[t] = hn;
    }
    kent* h = (kent*)malloc(sizeof(kent) * k);
    int hn = 0;
    for (int t = 0; t < T; t++)
        for (int j = 0; j < hns[t]; j++) heap_offer(h, &hn, k, hs[(size_t)k * t + j]);
    qsort(h, (size_t)hn, sizeof(kent), kcmp);
    for (int i = 0; i < hn; i++) { out_idx[i] = h[i].i; out_dist[i] = h[i].d; }
    *out_count = (uint32_t)hn;
    free(h); free(hs); free(hns); cl_free(&G); cl_free(&C);
    return OR_OK;
}

/* PointPointJoinQuery window join (PointPointJoinQuery.java:113-172) with
   JoinQuery.getReplicatedPointQueryStream (JoinQuery.java:73-90) and
   UniformGrid.getNeighboringCells (UniformGrid.java:261-293).  Pairs (p_idx, q_idx). */
int64_t geohip_oracle_join_pp(const or_grid* gd, const or_grid* gq, const double* dx, const double* dy,
                              uint64_t nd, const double* qx, const double* qy, uint64_t nq, double r,
                              int approximate, uint32_t* out_pairs, uint64_t cap, uint64_t* hash) {
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
            /* probe: data points in parallel chunks (ascending p within a chunk), counted and
               hashed first, written at the chunk's prefix offset when an output is asked for */
            const int T = nthreads();
            const int64_t NC = (int64_t)T * 16;
            uint64_t* coff = (uint64_t*)calloc((size_t)NC + 1, 8);
            uint64_t h = 0;
            for (int write = 0; write < 2; write++) {
                if (write && (!out_pairs || cap == 0)) break;
#pragma omp parallel for schedule(dynamic) num_threads(T) reduction(+ : h)
                for (int64_t ch = 0; ch < NC; ch++) {
                    const uint64_t lo = nd * (uint64_t)ch / (uint64_t)NC, hi = nd * (uint64_t)(ch + 1) / (uint64_t)NC;
                    uint64_t m = 0, o = write ? coff[ch] : 0;
                    for (uint64_t p = lo; p < hi; p++) {
                        int32_t cx, cy;
                        geohip_oracle_cell(gd, dx[p], dy[p], &cx, &cy);
                        /* data key (uGrid) must equal a replicated key (valid in qGrid) */
                        if (cx < 0 || cy < 0 || cx >= gq->n || cy >= gq->n) continue;
                        int64_t c = (int64_t)cx * gq->n + cy;
                        for (uint32_t t = cnt[c]; t < cnt[c + 1]; t++) {
                            uint32_t q = list[t];
                            if (approximate || geohip_oracle_pp_distance(dx[p], dy[p], qx[q], qy[q]) <= r) {
                                if (write) {
                                    if (o < cap) { out_pairs[2 * o] = (uint32_t)p; out_pairs[2 * o + 1] = q; }
                                    o++;
                                } else {
                                    m++;
                                    h += mix64(((uint64_t)p << 32) | q);
                                }
                            }
                        }
                    }
                    if (!write) coff[ch + 1] = m;
                }
                if (!write)
                    for (int64_t ch = 0; ch < NC; ch++) coff[ch + 1] += coff[ch];
            }
            const uint64_t out = coff[NC];
            free(coff);
            if (hash) *hash = h;
            free(list); free(fill); free(cnt);
            return (int64_t)out;
        }
    }
    free(cnt);
    return OR_ERR_ARG;
}

/* One query polygon as the reference builds it: Polygon(List<List<Coordinate>>, UniformGrid)
   (Polygon.java:52-66) -> createPolygon (Polygon.java:147-165): one ring -> closed (:149-153);
   several -> createPolygonArray (:115-145): each ring padded (1..3 coords: first appended 4
   times) and closed, ordered by JTS area (largest first, the list's insertion rule; a NaN area is
   never inserted), shell = first, holes = the rest.  Envelope = the shell's (Polygon envelope),
   gridIDsSet = bbox cells on grid g unclipped (HelperClass.java:123-143), then
   G = union of guaranteed squares, C = union of candidate squares minus G
   (UniformGrid.java:193-206, 398-410).
   Polygon p = rings [poly_rings[p], poly_rings[p+1]) (poly_rings NULL: ring p), ring j =
   vertices [ring_off[j], ring_off[j+1]) of vx/vy. */
typedef struct { double* rx; double* ry; int* roff; or_env* renv; int nring; or_env env; cellset G, C; } or_poly;
static void poly_free(or_poly* P) {
    cl_free(&P->G); cl_free(&P->C);
    free(P->rx); free(P->ry); free(P->roff); free(P->renv);
}

/* JTS 1.16.1 Area.ofRingSigned (shoelace, first x subtracted); Polygon.getArea = |.| */
static double ring_area(const double* x, const double* y, int n) {
    if (n < 3) return 0.0;
    double sum = 0.0, x0 = x[0];
    for (int i = 1; i < n - 1; i++) sum += (x[i] - x0) * (y[i - 1] - y[i + 1]);
    return fabs(sum / 2.0);
}

static int poly_build(const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx, const double* vy,
                      uint32_t pi, or_poly* P) {
    memset(P, 0, sizeof *P);
    uint32_t r0 = poly_rings ? poly_rings[pi] : pi, r1 = poly_rings ? poly_rings[pi + 1] : pi + 1;
    if (r1 <= r0) return OR_ERR_ARG;
    int nr = (int)(r1 - r0);
    if (ring_off[r0 + 1] - ring_off[r0] <= 3) return OR_ERR_ARG; /* Polygon.java:53: polygon stays null */
    size_t cap = 0;
    for (int j = 0; j < nr; j++) cap += ring_off[r0 + j + 1] - ring_off[r0 + j] + 5;
    double* tx = (double*)malloc(sizeof(double) * cap);
    double* ty = (double*)malloc(sizeof(double) * cap);
    int* toff = (int*)malloc(sizeof(int) * (nr + 1));
    double* area = (double*)malloc(sizeof(double) * nr);
    int* order = (int*)malloc(sizeof(int) * nr);
    int rc = OR_OK, nord = 0;
    toff[0] = 0;
    for (int j = 0; j < nr && !rc; j++) {
        const uint32_t a = ring_off[r0 + j], b = ring_off[r0 + j + 1];
        int m = (int)(b - a), o = toff[j];
        if (m == 0) { rc = OR_ERR_ARG; break; } /* listCoordinate.get(0): IndexOutOfBounds */
        memcpy(tx + o, vx + a, sizeof(double) * m);
        memcpy(ty + o, vy + a, sizeof(double) * m);
        if (nr > 1 && m < 4) {
            for (int t = 0; t < 4; t++) { tx[o + m] = tx[o]; ty[o + m] = ty[o]; m++; }
        }
        if (!(tx[o] == tx[o + m - 1] && ty[o] == ty[o + m - 1])) { tx[o + m] = tx[o]; ty[o + m] = ty[o]; m++; }
        /* LinearRing: first == last (equals2D) or JTS throws (a NaN first coordinate) */
        if (!(tx[o] == tx[o + m - 1] && ty[o] == ty[o + m - 1])) { rc = OR_ERR_ARG; break; }
        toff[j + 1] = o + m;
        if (nr == 1) { order[nord++] = 0; break; }
        area[j] = ring_area(tx + o, ty + o, m);
        if (nord == 0 || area[order[nord - 1]] >= area[j]) {
            order[nord++] = j;
        } else {
            for (int i = 0; i < nord; i++)
                if (area[order[i]] <= area[j]) {
                    memmove(order + i + 1, order + i, sizeof(int) * (nord - i));
                    order[i] = j;
                    nord++;
                    break;
                }
        }
    }
    if (!rc && nord == 0) rc = OR_ERR_ARG; /* every ring's area NaN: no shell (listPolygon.get(0) throws) */
    if (!rc) {
        int tot = 0;
        for (int i = 0; i < nord; i++) tot += toff[order[i] + 1] - toff[order[i]];
        P->rx = (double*)malloc(sizeof(double) * tot);
        P->ry = (double*)malloc(sizeof(double) * tot);
        P->roff = (int*)malloc(sizeof(int) * (nord + 1));
        P->renv = (or_env*)malloc(sizeof(or_env) * nord);
        P->nring = nord;
        P->roff[0] = 0;
        for (int i = 0; i < nord; i++) {
            int j = order[i], m = toff[j + 1] - toff[j];
            memcpy(P->rx + P->roff[i], tx + toff[j], sizeof(double) * m);
            memcpy(P->ry + P->roff[i], ty + toff[j], sizeof(double) * m);
            P->roff[i + 1] = P->roff[i] + m;
            P->renv[i] = ring_env(P->rx + P->roff[i], P->ry + P->roff[i], m);
        }
        P->env = P->renv[0];
    }
    free(tx); free(ty); free(toff); free(area); free(order);
    return rc;
}

static int poly_prep(const or_grid* g, const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
                     const double* vy, uint32_t pi, double r, or_poly* P) {
    int rc = poly_build(poly_rings, ring_off, vx, vy, pi, P);
    if (rc) { free(P->rx); free(P->ry); free(P->roff); free(P->renv); return rc; }
    cl_init(&P->G); cl_init(&P->C);
    int32_t x1 = j_d2i(floor((P->env.minx - g->min_x) / g->cell_len));
    int32_t y1 = j_d2i(floor((P->env.miny - g->min_y) / g->cell_len));
    int32_t x2 = j_d2i(floor((P->env.maxx - g->min_x) / g->cell_len));
    int32_t y2 = j_d2i(floor((P->env.maxy - g->min_y) / g->cell_len));
    if (x2 == INT32_MAX || y2 == INT32_MAX) { poly_free(P); return OR_ERR_HANG; }
    for (int64_t a = x1; a <= x2 && !rc; a++)
        for (int64_t c = y1; c <= y2 && !rc; c++) rc = add_guaranteed(g, &P->G, r, (int32_t)a, (int32_t)c);
    for (int64_t a = x1; a <= x2 && !rc; a++)
        for (int64_t c = y1; c <= y2 && !rc; c++) rc = add_candidate(g, &P->C, &P->G, r, (int32_t)a, (int32_t)c);
    if (rc) poly_free(P);
    return rc;
}

static double poly_distance(const or_poly* P, double px, double py) {
    return poly_rings_distance(px, py, P->rx, P->ry, P->roff, P->renv, P->nring);
}

/* point.distance(polygon) of the polygon built from rings ring_off[0..nring] of vx/vy */
double geohip_oracle_point_polygon_rings(double px, double py, const uint32_t* ring_off, uint32_t nring,
                                         const double* vx, const double* vy, int* status) {
    or_poly P;
    uint32_t pr[2] = {0, nring};
    int rc = poly_build(pr, ring_off, vx, vy, 0, &P);
    if (status) *status = rc;
    if (rc) { free(P.rx); free(P.ry); free(P.roff); free(P.renv); return 0.0; }
    double d = poly_distance(&P, px, py);
    free(P.rx); free(P.ry); free(P.roff); free(P.renv);
    return d;
}

/* Points binned by their cell on one grid (test-infrastructure acceleration of the per-polygon
   window scan: a polygon visits the points of its G and C cells instead of filtering the whole
   window -- the same points, the same per-point predicate).  Valid cells (0 <= cx, cy < n) by a
   counting sort; points of other cells in one list that is scanned when a polygon's cell sets
   hold an invalid cell (Lg == 0 key matches outside the grid).  dense == 0 (n^2 too large): every
   polygon scans the whole window. */
typedef struct {
    int32_t n;
    int dense;
    uint32_t* start; /* n*n + 1 */
    uint32_t* idx;
    uint32_t* out;   /* out-of-grid points */
    uint64_t nout;
    int32_t* cxy;    /* cell per point (2 per point) */
} or_bins;

static void bins_free(or_bins* B) { free(B->start); free(B->idx); free(B->out); free(B->cxy); }

static int bins_build(const or_grid* g, const double* x, const double* y, uint64_t n, or_bins* B) {
    memset(B, 0, sizeof *B);
    B->n = g->n;
    B->cxy = (int32_t*)malloc(sizeof(int32_t) * 2 * (n ? n : 1));
    if (!B->cxy) return OR_ERR_OOM;
#pragma omp parallel for schedule(static) num_threads(nthreads())
    for (int64_t i = 0; i < (int64_t)n; i++) geohip_oracle_cell(g, x[i], y[i], &B->cxy[2 * i], &B->cxy[2 * i + 1]);
    const int64_t nc = (int64_t)g->n * g->n;
    if (nc > (1ll << 26)) return OR_OK;
    B->dense = 1;
    B->start = (uint32_t*)calloc((size_t)nc + 1, 4);
    B->idx = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    B->out = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    if (!B->start || !B->idx || !B->out) return OR_ERR_OOM;
    for (uint64_t i = 0; i < n; i++) {
        int32_t cx = B->cxy[2 * i], cy = B->cxy[2 * i + 1];
        if (cx >= 0 && cy >= 0 && cx < g->n && cy < g->n) B->start[(int64_t)cx * g->n + cy + 1]++;
        else B->out[B->nout++] = (uint32_t)i;
    }
    for (int64_t c = 0; c < nc; c++) B->start[c + 1] += B->start[c];
    uint32_t* fill = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)nc);
    if (!fill) return OR_ERR_OOM;
    memcpy(fill, B->start, sizeof(uint32_t) * (size_t)nc);
    for (uint64_t i = 0; i < n; i++) {
        int32_t cx = B->cxy[2 * i], cy = B->cxy[2 * i + 1];
        if (cx >= 0 && cy >= 0 && cx < g->n && cy < g->n) B->idx[fill[(int64_t)cx * g->n + cy]++] = (uint32_t)i;
    }
    free(fill);
    return OR_OK;
}

/* growable u32 list */
typedef struct { uint32_t* v; uint64_t n, cap; } u32vec;
static void uv_push(u32vec* a, uint32_t x) {
    if (a->n == a->cap) { a->cap = a->cap ? 2 * a->cap : 256; a->v = (uint32_t*)realloc(a->v, 4 * a->cap); }
    a->v[a->n++] = x;
}
static int u32cmp(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

/* The points of P's G u C cells (cell sets tested on the points' own cells) in ascending index
   order, with inG flags: calls visit(i, inG) */
static int cellset_has_invalid(const cellset* c, int32_t n) {
    if (c->has_m1m1) return 1;
    for (uint64_t s = 0; s < c->s.cap; s++) {
        uint64_t k = c->s.slot[s];
        if (k == EMPTY_SLOT) continue;
        int32_t cx = (int32_t)(uint32_t)(k >> 32), cy = (int32_t)(uint32_t)k;
        if (cx < 0 || cy < 0 || cx >= n || cy >= n) return 1;
    }
    return 0;
}
/* candidate point list of a polygon: points of G u C, ascending */
static void poly_candidates(const or_poly* P, const or_bins* B, uint64_t n, u32vec* out) {
    out->n = 0;
    if (!B->dense) {
        for (uint64_t i = 0; i < n; i++)
            if (cl_has(&P->G, B->cxy[2 * i], B->cxy[2 * i + 1]) || cl_has(&P->C, B->cxy[2 * i], B->cxy[2 * i + 1]))
                uv_push(out, (uint32_t)i);
        return;
    }
    const cellset* sets[2] = {&P->G, &P->C};
    for (int w = 0; w < 2; w++) {
        const cellset* c = sets[w];
        for (uint64_t s = 0; s < c->s.cap; s++) {
            uint64_t k = c->s.slot[s];
            if (k == EMPTY_SLOT) continue;
            int32_t cx = (int32_t)(uint32_t)(k >> 32), cy = (int32_t)(uint32_t)k;
            if (cx < 0 || cy < 0 || cx >= B->n || cy >= B->n) continue;
            int64_t cell = (int64_t)cx * B->n + cy;
            for (uint32_t t = B->start[cell]; t < B->start[cell + 1]; t++) uv_push(out, B->idx[t]);
        }
    }
    if (cellset_has_invalid(&P->G, B->n) || cellset_has_invalid(&P->C, B->n))
        for (uint64_t t = 0; t < B->nout; t++) {
            uint32_t i = B->out[t];
            if (cl_has(&P->G, B->cxy[2 * i], B->cxy[2 * i + 1]) || cl_has(&P->C, B->cxy[2 * i], B->cxy[2 * i + 1]))
                uv_push(out, i);
        }
    qsort(out->v, out->n, 4, u32cmp);
}

/* Shared driver of the point-polygon range / join oracles: polygons in parallel, each one's
   hits in ascending point order, concatenated in polygon order (written when out_pairs), counted
   and hashed (sum of mix64(first << 32 | second) over the output pairs). */
static int64_t ppoly_run(const or_grid* gp, const or_grid* gq, int join, const double* x, const double* y,
                         uint64_t n, const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
                         const double* vy, uint32_t npoly, double r, int approximate, uint32_t* out_pairs,
                         uint64_t cap, uint64_t* hash) {
    or_bins B;
    int rc = bins_build(gp, x, y, n, &B);
    if (rc) { bins_free(&B); return rc; }
    u32vec* hits = (u32vec*)calloc(npoly ? npoly : 1, sizeof(u32vec));
    int err = 0;
    uint64_t h = 0;
#pragma omp parallel num_threads(nthreads()) reduction(+ : h)
    {
        u32vec cand = {0};
#pragma omp for schedule(dynamic)
        for (int64_t pi = 0; pi < (int64_t)npoly; pi++) {
            or_poly P;
            int prc = poly_prep(gq, poly_rings, ring_off, vx, vy, (uint32_t)pi, r, &P);
            if (prc) {
#pragma omp critical
                if (!err) err = prc;
                continue;
            }
            poly_candidates(&P, &B, n, &cand);
            for (uint64_t t = 0; t < cand.n; t++) {
                uint32_t i = cand.v[t];
                int emit;
                if (join) { /* PointPolygonJoinQuery.java:183-195: every replicated pair is checked */
                    emit = approximate || poly_distance(&P, x[i], y[i]) <= r;
                } else {   /* PointPolygonRangeQuery.java:104-124 */
                    emit = cl_has(&P.G, B.cxy[2 * i], B.cxy[2 * i + 1]);
                    if (!emit) {
                        double d = approximate
                            ? geohip_oracle_bbox_distance(x[i], y[i], P.env.minx, P.env.miny, P.env.maxx, P.env.maxy)
                            : poly_distance(&P, x[i], y[i]);
                        emit = d <= r;
                    }
                }
                if (emit) {
                    uv_push(&hits[pi], i);
                    h += join ? mix64(((uint64_t)i << 32) | (uint64_t)pi) : mix64(((uint64_t)pi << 32) | i);
                }
            }
            poly_free(&P);
        }
        free(cand.v);
    }
    uint64_t out = 0;
    for (uint32_t pi = 0; pi < npoly; pi++) {
        for (uint64_t t = 0; t < hits[pi].n && out_pairs; t++, out++)
            if (out < cap) {
                out_pairs[2 * out] = join ? hits[pi].v[t] : pi;
                out_pairs[2 * out + 1] = join ? pi : hits[pi].v[t];
            }
        if (!out_pairs) out += hits[pi].n;
        free(hits[pi].v);
    }
    free(hits);
    bins_free(&B);
    if (err) return err;
    if (hash) *hash = h;
    return (int64_t)out;
}

/* PointPolygonRangeQuery window body (PointPolygonRangeQuery.java:76-124) for npoly independent
   query polygons (rings as in poly_prep).  Pairs (poly, pt): emit iff key(p) in G, or key(p) in
   C and distance <= r (JTS DistanceOp, or the bbox distance when approximate). */
int64_t geohip_oracle_range_ppoly(const or_grid* g, const double* x, const double* y, uint64_t n,
                                  const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
                                  const double* vy, uint32_t npoly, double r, int approximate,
                                  uint32_t* out_pairs, uint64_t cap, uint64_t* hash) {
    if (g->n <= 0 || g->n > 99999 || !(g->cell_len > 0)) return OR_ERR_ARG;
    return ppoly_run(g, g, 0, x, y, n, poly_rings, ring_off, vx, vy, npoly, r, approximate, out_pairs, cap, hash);
}

/* PointPolygonJoinQuery window join (PointPolygonJoinQuery.java:162-201) with the polygon
   stream replicated to its G and C cells on the query grid (JoinQuery.getReplicatedPolygonQueryStream,
   JoinQuery.java:93-115): a point joins a polygon iff its gridID (point grid) equals one of
   them, and approximate or JTS distance <= r.  No guaranteed-cell shortcut.  Pairs (pt, poly). */
int64_t geohip_oracle_join_ppoly(const or_grid* gp, const or_grid* gq, const double* x, const double* y, uint64_t n,
                                 const uint32_t* poly_rings, const uint32_t* ring_off, const double* vx,
                                 const double* vy, uint32_t npoly, double r, int approximate,
                                 uint32_t* out_pairs, uint64_t cap, uint64_t* hash) {
    if (gp->n <= 0 || gp->n > 99999 || !(gp->cell_len > 0)) return OR_ERR_ARG;
    if (gq->n <= 0 || gq->n > 99999 || !(gq->cell_len > 0)) return OR_ERR_ARG;
    return ppoly_run(gp, gq, 1, x, y, n, poly_rings, ring_off, vx, vy, npoly, r, approximate, out_pairs, cap, hash);
}

/* PointPolygonKNNQuery window body (PointPolygonKNNQuery.java:162-236): candidates are the
   points of G u C of the query polygon (rings ring_off[0..nring] of vx/vy, built as poly_prep),
   distance = JTS point.distance(polygon) (or the bbox distance, DistanceFunctions.java:150-200,
   when approximate); no radius filter; same build contract as geohip_oracle_knn_pp: the k
   smallest (dist, idx), ascending by distance bits then idx (a NaN canonicalised to
   0x7ff8000000000000 so it ranks after +Infinity -- the total order the device selects by). */
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
static void kb_offer(kbent* h, int* hn, uint32_t k, kbent e) {
    if (*hn < (int)k) { h[*hn] = e; kb_up(h, *hn); (*hn)++; }
    else if (kbless(e, h[0])) { h[0] = e; kb_down(h, *hn, 0); }
}
static int kbcmp(const void* a, const void* b) {
    kbent x = *(const kbent*)a, y = *(const kbent*)b;
    return kbless(x, y) ? -1 : kbless(y, x) ? 1 : 0;
}

int geohip_oracle_knn_ppoly(const or_grid* g, const double* x, const double* y, uint64_t n,
                            const uint32_t* ring_off, uint32_t nring, const double* vx, const double* vy,
                            double r, uint32_t k, int approximate, uint32_t* out_idx, double* out_dist,
                            uint32_t* out_count) {
    *out_count = 0;
    if (g->n <= 0 || g->n > 99999 || !(g->cell_len > 0) || k == 0) return OR_ERR_ARG;
    or_poly P;
    uint32_t pr[2] = {0, nring};
    int rc = poly_prep(g, pr, ring_off, vx, vy, 0, r, &P);
    if (rc) return rc;
    const int T = nthreads();
    kbent* hs = (kbent*)malloc(sizeof(kbent) * (size_t)k * T);
    int* hns = (int*)calloc((size_t)T, sizeof(int));
#pragma omp parallel num_threads(T)
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num();
#else
        const int t = 0;
#endif
        kbent* h = hs + (size_t)k * t;
        int hn = 0;
#pragma omp for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; i++) {
            int32_t cx, cy;
            geohip_oracle_cell(g, x[i], y[i], &cx, &cy);
            if (!cl_has(&P.G, cx, cy) && !cl_has(&P.C, cx, cy)) continue;
            double d = approximate
                ? geohip_oracle_bbox_distance(x[i], y[i], P.env.minx, P.env.miny, P.env.maxx, P.env.maxy)
                : poly_distance(&P, x[i], y[i]);
            uint64_t bits;
            memcpy(&bits, &d, 8);
            if (d != d) bits = 0x7ff8000000000000ull;
            kbent e = {bits, (uint32_t)i};
            kb_offer(h, &hn, k, e);
        }
        hns[t] = hn;
    }
    kbent* h = (kbent*)malloc(sizeof(kbent) * k);
    int hn = 0;
    for (int t = 0; t < T; t++)
        for (int j = 0; j < hns[t]; j++) kb_offer(h, &hn, k, hs[(size_t)k * t + j]);
    qsort(h, (size_t)hn, sizeof(kbent), kbcmp);
    for (int i = 0; i < hn; i++) { out_idx[i] = h[i].i; memcpy(&out_dist[i], &h[i].d, 8); }
    *out_count = (uint32_t)hn;
    free(h); free(hs); free(hns);
    poly_free(&P);
    return OR_OK;
}
