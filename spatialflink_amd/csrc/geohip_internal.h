// geohip_internal.h -- shared host/device declarations of libgeohip.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/geohip.h"

namespace geohip {

// A cell rectangle turned into an exact coordinate-space box.  Because a point's cell
// index (int)floor((x - minX)/l) is a monotone function of x over the non-NaN doubles
// (HelperClass.java:109-110), the set of x with x0 <= cell(x) <= x1 is an interval
// [xlo, xhi] of doubles; the planner finds its ends by bisection over the ordered doubles
// so the device classifies a point with four compares instead of two fp64 divisions.
// NaN coordinates land in cell 0 (Java (int)NaN == 0): nan_x/nan_y say whether 0 lies in
// the rectangle's range on that axis.
struct Box {
    double xlo, xhi, ylo, yhi;
    int32_t nan_x, nan_y;
    int32_t empty, pad;
};

constexpr int kMaxPointBoxes = 16;

// Point query plan: G = union of g[0..ng); C = c[0..nc) minus G; U = G u C as boxes.
struct PointPlan {
    Box g[kMaxPointBoxes];
    Box c;
    Box u[kMaxPointBoxes + 1];
    int32_t ng, nc, nu;
    int32_t layers_g, layers_c;
};

// Host planner (plan.cpp).  Returns GEOHIP_OK or an error code with a message.
int plan_point(const geohip_grid& g, double qx, double qy, double r, PointPlan* out,
               std::vector<geohip_rect>* g_rects, std::vector<geohip_rect>* c_rects,
               std::string* err);
int cell_of(const geohip_grid& g, double x, double y, int32_t* cx, int32_t* cy);
int32_t java_d2i(double v);
int32_t layers_guaranteed(const geohip_grid& g, double r);
int32_t layers_candidate(const geohip_grid& g, double r);
Box rect_to_box(const geohip_grid& g, const geohip_rect& r);
// Per-axis cell boundary: smallest double v with cell(v) >= c (returns false if none).
bool axis_lower(double min_v, double l, int32_t c, double* out);
bool axis_upper(double min_v, double l, int32_t c, double* out);

// Java getIntCellIndices(key(cx,cy)) round trip; false where the reference throws
// NumberFormatException.
bool key_roundtrip(int32_t cx, int32_t cy, int32_t* ox, int32_t* oy);
// All (a,b) whose "%05d%05d" key equals the key of (cx,cy).
int key_matches(int32_t cx, int32_t cy, int32_t* pairs, int max_pairs);

// Polygon plan (one query polygon of the point-polygon queries).
struct PolyPlan {
    std::vector<geohip_rect> g, c;   // G = union g; C = union c minus G
    double bbox[4];                  // minx, miny, maxx, maxy (JTS envelope: the shell's)
    std::vector<double> rx, ry;      // closed rings, shell first, then the holes
    std::vector<uint32_t> ring_start;  // ring j = [ring_start[j], ring_start[j+1]) of rx/ry
};
int plan_polygon(const geohip_grid& g, const double* vx, const double* vy, uint32_t nv, double r,
                 PolyPlan* out, std::string* err);
int plan_polygon_rings(const geohip_grid& g, const uint32_t* ring_off, uint32_t nring, const double* vx,
                       const double* vy, double r, PolyPlan* out, std::string* err);
int build_polygon_rings(const uint32_t* ring_off, uint32_t nring, const double* vx, const double* vy,
                        PolyPlan* out, std::string* err);

}  // namespace geohip
