// plan.cpp -- host-side query planning of libgeohip (no device code).
//
// Turns a query (point + radius, or polygon + radius) into the reference's guaranteed /
// candidate cell sets expressed as cell rectangles, and each rectangle into an exact
// coordinate box (geohip_internal.h, Box).  Semantics follow
//   UniformGrid.java:165-206 (guaranteed cells), :224-229 (validKey), :261-293 (neighbours),
//   :367-410 (candidate cells), :427-444 (layer counts) and
//   HelperClass.java:54-63, 104-143, 263-276 (cell keys, "%05d%05d" strings, parse back),
// including Java int wrap-around in the layer loops and the string round trip of a cell key
// (a query cell outside [-9999, 99999] parses back to different indices, or throws).
#include <math.h>
#include <string.h>

#include <algorithm>

#include "geohip_internal.h"

namespace geohip {

int32_t java_d2i(double v) {  // JLS 5.1.3 narrowing of double to int
    if (v != v) return 0;
    if (v >= 2147483647.0) return INT32_MAX;
    if (v <= -2147483648.0) return INT32_MIN;
    return (int32_t)v;
}

static inline int32_t axis_cell(double min_v, double l, double v) {
    return java_d2i(floor((v - min_v) / l));
}

int cell_of(const geohip_grid& g, double x, double y, int32_t* cx, int32_t* cy) {
    *cx = axis_cell(g.min_x, g.cell_len, x);
    *cy = axis_cell(g.min_y, g.cell_len, y);
    return GEOHIP_OK;
}

int32_t layers_guaranteed(const geohip_grid& g, double r) {  // UniformGrid.java:427-438
    double cell_diagonal = g.cell_len * sqrt(2.0);
    return java_d2i(floor((r / cell_diagonal) - 1));
}

int32_t layers_candidate(const geohip_grid& g, double r) {  // UniformGrid.java:440-444
    return java_d2i(ceil(r / g.cell_len));
}

// ---------------------------------------------------------------- "%05d" keys -------------
static int format05(int32_t v, char* out) {
    char digits[16];
    int nd = 0;
    int64_t a = v;
    bool neg = a < 0;
    if (neg) a = -a;
    do {
        digits[nd++] = (char)('0' + (int)(a % 10));
        a /= 10;
    } while (a != 0);
    int width = nd + (neg ? 1 : 0);
    int p = 0;
    if (neg) out[p++] = '-';
    for (int i = width; i < 5; i++) out[p++] = '0';
    while (nd > 0) out[p++] = digits[--nd];
    return p;
}

// Integer.parseInt(s.replaceFirst("^0+(?!$)", ""))
static bool java_parse(const char* s, int len, int32_t* out) {
    int skip = 0;
    while (skip < len - 1 && s[skip] == '0') skip++;
    s += skip;
    len -= skip;
    if (len <= 0) return false;
    bool neg = false;
    int p = 0;
    if (s[0] == '+' || s[0] == '-') {
        if (len == 1) return false;
        neg = s[0] == '-';
        p = 1;
    }
    int64_t v = 0;
    for (; p < len; p++) {
        if (s[p] < '0' || s[p] > '9') return false;
        v = v * 10 + (s[p] - '0');
        if (v > 2147483648LL) return false;
    }
    if (neg) v = -v;
    if (v > INT32_MAX || v < INT32_MIN) return false;
    *out = (int32_t)v;
    return true;
}

bool key_roundtrip(int32_t cx, int32_t cy, int32_t* ox, int32_t* oy) {
    char key[32];
    int n = format05(cx, key);
    n += format05(cy, key + n);
    return java_parse(key, 5, ox) && java_parse(key + 5, n - 5, oy);
}

// does s[0..len) render some int exactly as "%05d" does?
static bool render_of(const char* s, int len, int32_t* v) {
    if (len < 5 || len > 11) return false;
    bool neg = s[0] == '-';
    int p = neg ? 1 : 0;
    if (p >= len) return false;
    int64_t a = 0;
    for (int i = p; i < len; i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        a = a * 10 + (s[i] - '0');
        if (a > 2147483648LL) return false;
    }
    int64_t val = neg ? -a : a;
    if (val > INT32_MAX || val < INT32_MIN) return false;
    char buf[16];
    int m = format05((int32_t)val, buf);
    if (m != len || memcmp(buf, s, (size_t)len) != 0) return false;
    *v = (int32_t)val;
    return true;
}

int key_matches(int32_t cx, int32_t cy, int32_t* pairs, int max_pairs) {
    char key[32];
    int n = format05(cx, key);
    n += format05(cy, key + n);
    int cnt = 0;
    for (int split = 5; split <= n - 5; split++) {
        int32_t a, b;
        if (render_of(key, split, &a) && render_of(key + split, n - split, &b)) {
            if (cnt < max_pairs) {
                pairs[2 * cnt] = a;
                pairs[2 * cnt + 1] = b;
            }
            cnt++;
        }
    }
    return cnt;
}

// ---------------------------------------------------------------- exact boxes -------------
static inline uint64_t ord_of(double v) {
    uint64_t b;
    memcpy(&b, &v, 8);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
static inline double dbl_of(uint64_t o) {
    uint64_t b = (o >> 63) ? (o & ~(1ull << 63)) : ~o;
    double v;
    memcpy(&v, &b, 8);
    return v;
}

bool axis_lower(double min_v, double l, int32_t c, double* out) {
    uint64_t lo = ord_of(-INFINITY), hi = ord_of(INFINITY);
    if (axis_cell(min_v, l, dbl_of(lo)) >= c) { *out = -INFINITY; return true; }
    if (axis_cell(min_v, l, dbl_of(hi)) < c) return false;
    while (hi - lo > 1) {  // cell(lo) < c <= cell(hi)
        uint64_t mid = lo + (hi - lo) / 2;
        if (axis_cell(min_v, l, dbl_of(mid)) >= c) hi = mid; else lo = mid;
    }
    *out = dbl_of(hi);
    return true;
}

bool axis_upper(double min_v, double l, int32_t c, double* out) {
    uint64_t lo = ord_of(-INFINITY), hi = ord_of(INFINITY);
    if (axis_cell(min_v, l, dbl_of(hi)) <= c) { *out = INFINITY; return true; }
    if (axis_cell(min_v, l, dbl_of(lo)) > c) return false;
    while (hi - lo > 1) {  // cell(lo) <= c < cell(hi)
        uint64_t mid = lo + (hi - lo) / 2;
        if (axis_cell(min_v, l, dbl_of(mid)) <= c) lo = mid; else hi = mid;
    }
    *out = dbl_of(lo);
    return true;
}

Box rect_to_box(const geohip_grid& g, const geohip_rect& r) {
    Box b;
    memset(&b, 0, sizeof b);
    bool ok = r.x0 <= r.x1 && r.y0 <= r.y1;
    ok = ok && axis_lower(g.min_x, g.cell_len, r.x0, &b.xlo) && axis_upper(g.min_x, g.cell_len, r.x1, &b.xhi);
    ok = ok && axis_lower(g.min_y, g.cell_len, r.y0, &b.ylo) && axis_upper(g.min_y, g.cell_len, r.y1, &b.yhi);
    ok = ok && b.xlo <= b.xhi && b.ylo <= b.yhi;
    b.nan_x = r.x0 <= 0 && 0 <= r.x1;
    b.nan_y = r.y0 <= 0 && 0 <= r.y1;
    if (!ok) {  // never contains anything (NaN coordinates included)
        b.xlo = INFINITY; b.xhi = -INFINITY; b.ylo = INFINITY; b.yhi = -INFINITY;
        b.nan_x = b.nan_y = 0;
        b.empty = 1;
    }
    return b;
}

// ---------------------------------------------------------------- cell squares ------------
static inline int32_t wrap32(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }

// The square loop "for (i = ci - L; i <= ci + L; i++) for (j = ...) if (validKey(i,j))" with
// Java int arithmetic, as a clipped rectangle.  Returns false when the reference loop would
// never terminate (upper bound == Integer.MAX_VALUE).
static bool clipped_square(const geohip_grid& g, int32_t ci, int32_t cj, int32_t layers,
                           geohip_rect* out, bool* nonempty) {
    int32_t lo_i = wrap32((int64_t)ci - layers), hi_i = wrap32((int64_t)ci + layers);
    int32_t lo_j = wrap32((int64_t)cj - layers), hi_j = wrap32((int64_t)cj + layers);
    *nonempty = false;
    if (lo_i > hi_i) return true;  // outer loop never runs
    if (hi_i == INT32_MAX) return false;
    if (lo_j > hi_j) return true;
    if (hi_j == INT32_MAX) return false;
    geohip_rect r;
    r.x0 = std::max(lo_i, 0);
    r.x1 = std::min(hi_i, g.n - 1);
    r.y0 = std::max(lo_j, 0);
    r.y1 = std::min(hi_j, g.n - 1);
    if (r.x0 <= r.x1 && r.y0 <= r.y1) {
        *out = r;
        *nonempty = true;
    }
    return true;
}

static bool rect_inside(const geohip_rect& a, const geohip_rect& b) {
    return a.x0 >= b.x0 && a.x1 <= b.x1 && a.y0 >= b.y0 && a.y1 <= b.y1;
}

static int check_grid(const geohip_grid& g, std::string* err) {
    if (!(g.n > 0)) { *err = "grid: numGridPartitions must be > 0"; return GEOHIP_ERR_ARG; }
    if (g.n > 99999) {
        *err = "grid: more than 99999 cells per side breaks the reference's 5-digit cell keys";
        return GEOHIP_ERR_UNSUPPORTED;
    }
    if (!(g.cell_len > 0) || !isfinite(g.cell_len) || !isfinite(g.min_x) || !isfinite(g.min_y)) {
        *err = "grid: cell length must be positive and finite, bounds finite";
        return GEOHIP_ERR_ARG;
    }
    return GEOHIP_OK;
}

int plan_point(const geohip_grid& g, double qx, double qy, double r, PointPlan* out,
               std::vector<geohip_rect>* g_rects, std::vector<geohip_rect>* c_rects, std::string* err) {
    int rc = check_grid(g, err);
    if (rc) return rc;
    memset(out, 0, sizeof *out);
    int32_t qcx, qcy;
    cell_of(g, qx, qy, &qcx, &qcy);  // Point(x, y, uGrid) -> gridID (Point.java:60-67)
    int32_t lg = layers_guaranteed(g, r), lc = layers_candidate(g, r);
    out->layers_g = lg;
    out->layers_c = lc;
    std::vector<geohip_rect> gr, cr;
    if (lg == 0) {  // G = { queryGridCellID } unvalidated (UniformGrid.java:171-174)
        int32_t pairs[2 * 16];
        int m = key_matches(qcx, qcy, pairs, 16);
        for (int i = 0; i < m && i < 16; i++) gr.push_back({pairs[2 * i], pairs[2 * i], pairs[2 * i + 1], pairs[2 * i + 1]});
    } else if (lg > 0) {
        int32_t ci, cj;
        if (!key_roundtrip(qcx, qcy, &ci, &cj)) {
            *err = "NumberFormatException in HelperClass.getIntCellIndices (query cell key)";
            return GEOHIP_ERR_ARG;
        }
        geohip_rect s;
        bool ne;
        if (!clipped_square(g, ci, cj, lg, &s, &ne)) { *err = "reference layer loop does not terminate"; return GEOHIP_ERR_ARG; }
        if (ne) gr.push_back(s);
    }
    if (lc > 0) {  // UniformGrid.java:374-392
        int32_t ci, cj;
        if (!key_roundtrip(qcx, qcy, &ci, &cj)) {
            *err = "NumberFormatException in HelperClass.getIntCellIndices (query cell key)";
            return GEOHIP_ERR_ARG;
        }
        geohip_rect s;
        bool ne;
        if (!clipped_square(g, ci, cj, lc, &s, &ne)) { *err = "reference layer loop does not terminate"; return GEOHIP_ERR_ARG; }
        if (ne) cr.push_back(s);
    }
    if ((int)gr.size() > kMaxPointBoxes) { *err = "internal: too many guaranteed rects"; return GEOHIP_ERR_UNSUPPORTED; }
    for (size_t i = 0; i < gr.size(); i++) out->g[out->ng++] = rect_to_box(g, gr[i]);
    if (!cr.empty()) { out->c = rect_to_box(g, cr[0]); out->nc = 1; }
    for (size_t i = 0; i < gr.size(); i++)
        if (cr.empty() || !rect_inside(gr[i], cr[0])) out->u[out->nu++] = out->g[i];
    if (!cr.empty()) out->u[out->nu++] = out->c;
    // drop empty boxes from the kernel-facing lists (they contain nothing)
    auto compact = [](Box* b, int32_t* n) {
        int w = 0;
        for (int i = 0; i < *n; i++) if (!b[i].empty) b[w++] = b[i];
        *n = w;
    };
    compact(out->g, &out->ng);
    compact(out->u, &out->nu);
    if (out->nc && out->c.empty) out->nc = 0;
    if (g_rects) *g_rects = gr;
    if (c_rects) *c_rects = cr;
    return GEOHIP_OK;
}

// JTS 1.16.1 Polygon.getArea of a shell-only polygon: |Area.ofRingSigned| (shoelace with the
// first x subtracted), evaluated in source order.
static double jts_ring_area(const double* x, const double* y, size_t n) {
    if (n < 3) return 0.0;
    double sum = 0.0;
    const double x0 = x[0];
    for (size_t i = 1; i + 1 < n; i++) sum += (x[i] - x0) * (y[i - 1] - y[i + 1]);
    return std::fabs(sum / 2.0);
}

// Polygon(List<List<Coordinate>>, UniformGrid).createPolygon (Polygon.java:52-66, 115-165):
// rings [ring_off[j], ring_off[j+1]) of vx/vy.  One ring: closed if open (:149-153).  Several:
// createPolygonArray (:115-145) -- each ring padded (1..3 coords: its first coordinate appended
// 4 times) and closed, then ordered by JTS area, largest first, with that method's insertion
// rule (a tie with the tail goes after it, a larger area goes before the first ring whose area is
// <= it; a NaN area is never inserted), shell = first, holes = the rest.  Where the reference
// leaves polygon null (first ring <= 3 coords) or JTS throws (an empty ring; a ring whose first
// coordinate is NaN: LinearRing not closed; no ring left) -> GEOHIP_ERR_ARG.
int build_polygon_rings(const uint32_t* ring_off, uint32_t nring, const double* vx, const double* vy,
                        PolyPlan* out, std::string* err) {
    out->rx.clear();
    out->ry.clear();
    out->ring_start.assign(1, 0u);
    if (nring == 0) { *err = "polygon without rings"; return GEOHIP_ERR_ARG; }
    if (ring_off[1] < ring_off[0] || ring_off[1] - ring_off[0] <= 3) {
        *err = "Polygon needs more than 3 coordinates in its first ring (Polygon.java:53)";
        return GEOHIP_ERR_ARG;
    }
    std::vector<std::vector<double>> rxs(nring), rys(nring);
    std::vector<double> area(nring, 0.0);
    std::vector<uint32_t> order;
    for (uint32_t j = 0; j < nring; j++) {
        if (ring_off[j + 1] < ring_off[j]) { *err = "ring_off not ascending"; return GEOHIP_ERR_ARG; }
        const uint32_t a = ring_off[j], m = ring_off[j + 1] - ring_off[j];
        if (m == 0) { *err = "empty ring (IndexOutOfBoundsException in Polygon.createPolygonArray)"; return GEOHIP_ERR_ARG; }
        std::vector<double>& X = rxs[j];
        std::vector<double>& Y = rys[j];
        X.assign(vx + a, vx + a + m);
        Y.assign(vy + a, vy + a + m);
        if (nring > 1 && m < 4)
            for (int t = 0; t < 4; t++) { X.push_back(X[0]); Y.push_back(Y[0]); }
        if (!(X.front() == X.back() && Y.front() == Y.back())) { X.push_back(X[0]); Y.push_back(Y[0]); }
        if (!(X.front() == X.back() && Y.front() == Y.back())) {
            *err = "LinearRing not closed (NaN first coordinate): JTS IllegalArgumentException";
            return GEOHIP_ERR_ARG;
        }
        if (nring == 1) { order.push_back(0); break; }
        area[j] = jts_ring_area(X.data(), Y.data(), X.size());
        if (order.empty() || area[order.back()] >= area[j]) {
            order.push_back(j);
        } else {
            for (size_t i = 0; i < order.size(); i++)
                if (area[order[i]] <= area[j]) { order.insert(order.begin() + i, j); break; }
        }
    }
    if (order.empty()) { *err = "no ring with a comparable area (createPolygonArray)"; return GEOHIP_ERR_ARG; }
    for (uint32_t j : order) {
        out->rx.insert(out->rx.end(), rxs[j].begin(), rxs[j].end());
        out->ry.insert(out->ry.end(), rys[j].begin(), rys[j].end());
        out->ring_start.push_back((uint32_t)out->rx.size());
    }
    return GEOHIP_OK;
}

int plan_polygon(const geohip_grid& g, const double* vx, const double* vy, uint32_t nv, double r,
                 PolyPlan* out, std::string* err) {
    const uint32_t ro[2] = {0, nv};
    return plan_polygon_rings(g, ro, 1, vx, vy, r, out, err);
}

int plan_polygon_rings(const geohip_grid& g, const uint32_t* ring_off, uint32_t nring, const double* vx,
                       const double* vy, double r, PolyPlan* out, std::string* err) {
    int rc = check_grid(g, err);
    if (rc) return rc;
    rc = build_polygon_rings(ring_off, nring, vx, vy, out, err);
    if (rc) return rc;
    const size_t nshell = out->ring_start[1];
    // JTS envelope (Polygon envelope = the shell's: Envelope.expandToInclude over the shell)
    double minx = out->rx[0], maxx = out->rx[0], miny = out->ry[0], maxy = out->ry[0];
    for (size_t i = 1; i < nshell; i++) {
        double x = out->rx[i], y = out->ry[i];
        if (x < minx) minx = x;
        if (x > maxx) maxx = x;
        if (y < miny) miny = y;
        if (y > maxy) maxy = y;
    }
    out->bbox[0] = minx; out->bbox[1] = miny; out->bbox[2] = maxx; out->bbox[3] = maxy;
    out->g.clear();
    out->c.clear();
    // HelperClass.assignGridCellID(bbox) (HelperClass.java:123-143)
    int32_t x1, y1, x2, y2;
    cell_of(g, minx, miny, &x1, &y1);
    cell_of(g, maxx, maxy, &x2, &y2);
    if (x1 > x2 || y1 > y2) return GEOHIP_OK;  // gridIDsSet empty
    if (x2 == INT32_MAX || y2 == INT32_MAX) { *err = "reference bbox loop does not terminate"; return GEOHIP_ERR_ARG; }
    int32_t lg = layers_guaranteed(g, r), lc = layers_candidate(g, r);
    if (lg >= (1 << 30) || lc >= (1 << 30)) {
        *err = "radius too large: layer count >= 2^30 (reference int loops wrap)";
        return GEOHIP_ERR_UNSUPPORTED;
    }
    bool identity = x1 >= -9999 && x2 <= 99999 && y1 >= -9999 && y2 <= 99999;
    auto clip = [&](geohip_rect q, std::vector<geohip_rect>* dst) {
        q.x0 = std::max(q.x0, 0); q.x1 = std::min(q.x1, g.n - 1);
        q.y0 = std::max(q.y0, 0); q.y1 = std::min(q.y1, g.n - 1);
        if (q.x0 <= q.x1 && q.y0 <= q.y1) dst->push_back(q);
    };
    if (identity) {
        // every bbox cell key is 10 chars: the key round trip is the identity and the union of
        // the per-cell squares is the dilated bbox-cell rectangle (UniformGrid.java:193-206, 398-410)
        if (lg == 0) out->g.push_back({x1, x2, y1, y2});  // keys added unvalidated
        else if (lg > 0) clip({x1 - lg, x2 + lg, y1 - lg, y2 + lg}, &out->g);
        if (lc > 0) clip({x1 - lc, x2 + lc, y1 - lc, y2 + lc}, &out->c);
        return GEOHIP_OK;
    }
    uint64_t ncell = (uint64_t)((int64_t)x2 - x1 + 1) * (uint64_t)((int64_t)y2 - y1 + 1);
    if (ncell > (1u << 20)) { *err = "polygon bbox spans more than 2^20 cells far outside the grid"; return GEOHIP_ERR_UNSUPPORTED; }
    for (int64_t a = x1; a <= x2; a++)
        for (int64_t b = y1; b <= y2; b++) {
            int32_t ci, cj;
            if (lg == 0) {
                int32_t pairs[2 * 16];
                int m = key_matches((int32_t)a, (int32_t)b, pairs, 16);
                for (int i = 0; i < m && i < 16; i++)
                    out->g.push_back({pairs[2 * i], pairs[2 * i], pairs[2 * i + 1], pairs[2 * i + 1]});
            }
            if (lg > 0 || lc > 0) {
                if (!key_roundtrip((int32_t)a, (int32_t)b, &ci, &cj)) {
                    *err = "NumberFormatException in HelperClass.getIntCellIndices (polygon cell key)";
                    return GEOHIP_ERR_ARG;
                }
                geohip_rect s;
                bool ne;
                if (lg > 0) {
                    if (!clipped_square(g, ci, cj, lg, &s, &ne)) { *err = "reference layer loop does not terminate"; return GEOHIP_ERR_ARG; }
                    if (ne) out->g.push_back(s);
                }
                if (lc > 0) {
                    if (!clipped_square(g, ci, cj, lc, &s, &ne)) { *err = "reference layer loop does not terminate"; return GEOHIP_ERR_ARG; }
                    if (ne) out->c.push_back(s);
                }
            }
        }
    auto dedupe = [](std::vector<geohip_rect>* v) {
        std::sort(v->begin(), v->end(), [](const geohip_rect& p, const geohip_rect& q) {
            return memcmp(&p, &q, sizeof p) < 0;
        });
        v->erase(std::unique(v->begin(), v->end(), [](const geohip_rect& p, const geohip_rect& q) {
            return memcmp(&p, &q, sizeof p) == 0;
        }), v->end());
    };
    dedupe(&out->g);
    dedupe(&out->c);
    return GEOHIP_OK;
}

}  // namespace geohip
