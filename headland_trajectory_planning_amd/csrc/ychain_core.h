// The heuristic lowering between the two searches of the notebook planner, on the device: after the Y-type
// parking search (ypark_core.h) has fixed the intermediate pose, headland_planner_y_type_park builds a
// ReferenceLineHeuristic from the orchard's topology waypoints and hands it to the hybrid A* search
// (R/path_planner/headland_path_planning.py:124-255).  This core turns (rows, start pose, intermediate pose)
// into the search's heuristic inputs, one problem per thread:
//
//   waypoints .. orchard_geometry_environment.get_topology_waypoints (R/path_planner/
//                orchard_geometry_environment.py:199-248): the row ends strictly between the start and the goal
//                on the start's headland side (get_row_ids_between_start_and_end :93-127), nearest to the start
//                first (stable sort), moved by drive_row_offset away from the field (check_side_of_a_point
//                :49-64, its np.random.uniform(-0.5, 0.5) draws as inputs), between the start and goal points;
//   guide ...... reference_line_heuristic.py get_guide_line :50-82: per waypoint segment np.linspace at
//                int(dist / 0.1) points with the segment's yaw, arc length by the sequential cumsum;
//   lanes ...... the segment lanes LineString(segment).buffer(LANE_HALF_WIDTH = 6) (GEOS round caps, 16
//                segments per quadrant; path_planner/geom.py buffer_segment_round restates the ring);
//   lengths .... create_segment_lengths :84-96 without obstacle polygons (the combined planner passes none):
//                default_search_length, LARGE_SEARCH_LENGTH on lanes [2, n - 1) when there are more than 4.
#pragma once
#include <cmath>
#include <cstdint>

#ifndef HTP_HD
#error "define HTP_HD before including ychain_core.h"
#endif

#include "htp_libm.h"
#include "oge_core.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace htp {
namespace yc {

constexpr int MAXROWS = 32;     // rows per scene
constexpr int MAXWP = 10;       // waypoints: start, <= 8 row ends, goal
constexpr int MAXSEG = MAXWP - 1;
constexpr int CAPV = 80;        // ring vertices per lane (GEOS round-cap segment buffer: 2 x 34 at most)
constexpr double LANE_HALF_WIDTH = 6.0, LARGE_SEARCH_LENGTH = 1.0, GUIDE_STEP = 0.1;
constexpr double PI = 3.141592653589793;
enum { ST_OK = 0, ST_TOO_MANY_WAYPOINTS = 1, ST_GUIDE_OVERFLOW = 2, ST_BAD_INPUT = 3, ST_RING_OVERFLOW = 4 };

inline HTP_HD double npsign(double v) { return v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0); }

// rows[r] = {near x, near y, far x, far y} (map_tree_rows[r][0], [r][1]); eps[r] the side check's draws.
// Returns the waypoint count (or -1 when more than MAXWP).
HTP_HD inline int waypoints(const double* rows, int nrows, const double* eps, const double* start, const double* goal,
                            double drive_row_offset, double (*wp)[2]) {
  // get_row_ids_between_start_and_end: nearest near-end row to the start (first minimum, np.argmin)
  int row_id = 0;
  double best = fabs(start[1] - rows[1]);
  for (int r = 1; r < nrows; ++r) {
    const double d = fabs(start[1] - rows[4 * r + 1]);
    if (d < best) { best = d; row_id = r; }
  }
  const bool near = fabs(start[0] - rows[4 * row_id]) < fabs(start[0] - rows[4 * row_id + 2]);
  const int ox = near ? 0 : 2;
  const double sy = start[1], ey = goal[1];
  double ix[MAXROWS], iy[MAXROWS], key[MAXROWS];
  int n = 0;
  for (int r = 0; r < nrows; ++r) {
    const double y = rows[4 * r + ox + 1];
    const bool in = sy > ey ? (y > ey && y < sy) : (y > sy && y < ey);
    if (in) { ix[n] = rows[4 * r + ox]; iy[n] = y; key[n] = fabs(y - sy); ++n; }
  }
  if (n + 2 > MAXWP) return -1;
  // np.argsort of |iy - start_y|: numpy sorts arrays this short by insertion sort, i.e. stably
  for (int a = 1; a < n; ++a)
    for (int b = a; b > 0 && key[b] < key[b - 1]; --b) {
      double t = key[b]; key[b] = key[b - 1]; key[b - 1] = t;
      t = ix[b]; ix[b] = ix[b - 1]; ix[b - 1] = t;
      t = iy[b]; iy[b] = iy[b - 1]; iy[b - 1] = t;
    }
  // check_side_of_a_point(start): the centre-line fit through the row centres (+ the uniform draws)
  double cx[MAXROWS], cy[MAXROWS];
  for (int r = 0; r < nrows; ++r) {
    cx[r] = (rows[4 * r] + rows[4 * r + 2]) / 2.0 + eps[r];
    cy[r] = (rows[4 * r + 1] + rows[4 * r + 3]) / 2.0;
  }
  double k, b;
  oge::polyfit1(cx, cy, nrows, k, b);
  const bool near_side = npsign(0 * k + b - 0) == npsign(start[0] * k + b - start[1]);
  const double off = near_side ? -drive_row_offset : drive_row_offset;
  wp[0][0] = start[0]; wp[0][1] = start[1];
  for (int j = 0; j < n; ++j) { wp[1 + j][0] = ix[j] + off; wp[1 + j][1] = iy[j]; }
  wp[n + 1][0] = goal[0]; wp[n + 1][1] = goal[1];
  return n + 2;
}

// get_guide_line: rows [x, y, yaw, s]; returns the row count or -1 past cap
HTP_HD inline int guide(const double (*wp)[2], int nwp, double* g, int cap) {
  int m = 0;
  for (int i = 1; i < nwp; ++i) {
    const double xe = wp[i][0], xs = wp[i - 1][0], ye = wp[i][1], ys = wp[i - 1][1];
    const double dist = hm::hypot(xe - xs, ye - ys);
    const int num = (int)(dist / GUIDE_STEP);
    if (m + num > cap) return -1;
    const double yaw = hm::atan2(ye - ys, xe - xs);
    // np.linspace(start, stop, num): step = (stop - start) / (num - 1), the last point = stop
    const double stx = num > 1 ? (xe - xs) / (num - 1) : 0.0, sty = num > 1 ? (ye - ys) / (num - 1) : 0.0;
    for (int q = 0; q < num; ++q) {
      double* r = g + 4 * (int64_t)(m + q);
      r[0] = (num > 1 && q == num - 1) ? xe : xs + q * stx;
      r[1] = (num > 1 && q == num - 1) ? ye : ys + q * sty;
      r[2] = yaw;
    }
    m += num;
  }
  double s = 0.0;   // way_ss[1:] = np.cumsum(np.hypot(np.diff(xs), np.diff(ys)))
  for (int q = 0; q < m; ++q) {
    if (q > 0) s += hm::hypot(g[4 * q] - g[4 * (q - 1)], g[4 * q + 1] - g[4 * (q - 1) + 1]);
    g[4 * q + 3] = s;
  }
  return m;
}

// GEOS computeOffsetSegment (geom._offset): the offset of p0 -> p1 on `side` (+1 left, -1 right); its end point
HTP_HD inline void offset_end(const double* p0, const double* p1, double side, double d, double* o) {
  const double dx = p1[0] - p0[0], dy = p1[1] - p0[1];
  const double ln = sqrt(dx * dx + dy * dy);
  const double ux = side * d * dx / ln, uy = side * d * dy / ln;
  o[0] = p1[0] - uy;
  o[1] = p1[1] + ux;
}

// geom._add: append unless within `snap` of the previous vertex
HTP_HD inline void add_pt(double (*ring)[2], int& n, double x, double y, double snap) {
  if (n > 0 && hm::hypot(x - ring[n - 1][0], y - ring[n - 1][1]) < snap) return;
  if (n < CAPV) { ring[n][0] = x; ring[n][1] = y; }
  ++n;
}

// LineString([p0, p1]).buffer(d) with round caps (geom.buffer_segment_round, quad_segs = 16); returns the vertex
// count (no closing vertex) or -1 past CAPV
HTP_HD inline int capsule(const double* p0, const double* p1, double d, double (*ring)[2]) {
  const double snap = d * 1e-6;
  int n = 0;
  for (int pass = 0; pass < 2; ++pass) {
    const double* a = pass == 0 ? p0 : p1;
    const double* b = pass == 0 ? p1 : p0;
    double o[2];
    offset_end(a, b, 1.0, d, o);
    add_pt(ring, n, o[0], o[1], snap);                 // addLastSegment
    const double ang = hm::atan2(b[1] - a[1], b[0] - a[0]);
    add_pt(ring, n, o[0], o[1], snap);                 // cap: offsetL.p1
    const double st = ang + PI / 2.0, en = ang - PI / 2.0;
    const double quantum = PI / 2.0 / 16.0, total = fabs(st - en);
    const int nf = (int)(total / quantum + 0.5);
    if (nf >= 1) {
      const double inc = total / nf;
      for (int i = 0; i < nf; ++i)
        add_pt(ring, n, b[0] + d * hm::cos(st + (-i) * inc), b[1] + d * hm::sin(st + (-i) * inc), snap);
    }
    offset_end(a, b, -1.0, d, o);
    add_pt(ring, n, o[0], o[1], snap);                 // cap: offsetR.p1
  }
  if (n > CAPV) return -1;
  if (n > 1 && hm::hypot(ring[0][0] - ring[n - 1][0], ring[0][1] - ring[n - 1][1]) < snap) --n;
  // as the search's packer stores a lane (_native._clean_ring, _ccw): consecutive exact duplicates and a
  // repeated closing vertex dropped, then counter-clockwise (the GEOS ring runs clockwise: reversed)
  int m = n > 0 ? 1 : 0;
  for (int i = 1; i < n; ++i)
    if (!(ring[i][0] == ring[m - 1][0] && ring[i][1] == ring[m - 1][1])) { ring[m][0] = ring[i][0]; ring[m][1] = ring[i][1]; ++m; }
  if (m > 1 && ring[0][0] == ring[m - 1][0] && ring[0][1] == ring[m - 1][1]) --m;
  double area = 0.0;
  for (int i = 0; i < m; ++i) {
    const int j = i + 1 < m ? i + 1 : 0;
    area += ring[i][0] * ring[j][1] - ring[j][0] * ring[i][1];
  }
  if (!(area > 0))
    for (int i = 0, j = m - 1; i < j; ++i, --j) {
      double t = ring[i][0]; ring[i][0] = ring[j][0]; ring[j][0] = t;
      t = ring[i][1]; ring[i][1] = ring[j][1]; ring[j][1] = t;
    }
  return m;
}

// create_segment_lengths without obstacle polygons
HTP_HD inline double search_length(int seg, int nseg, double default_len) {
  return (nseg > 4 && seg >= 2 && seg < nseg - 1) ? LARGE_SEARCH_LENGTH : default_len;
}

}  // namespace yc
}  // namespace htp
