// Orchard scene -> OBCA obstacle polygons: the synthetic orchard producer and the
// OGE_OBCA obstacle producer of the reference, as one __host__ __device__ routine
// per scene.
//
//   tree rows ............ create_tree_rows           R/path_planner/utils/map_utils.py:45-61
//   field polygon ........ get_map_exterior_pts       R/path_planner/orchard_geometry_environment.py:288-334
//                          get_headland_angle         :463-472
//   contour split ........ create_headland_countour_lines :66-91
//   simplification ....... rdp (third-party `rdp`: Ramer-Douglas-Peucker, recursive, first maximum kept)
//   boundary quads ....... cover_side_points          R/path_planner/OGE_OBCA.py:171-262
//                          create_boundary_polygons   :306-373
//   tree-row rectangles .. get_obstacle_tree_rows     :477-591
//   OBCA obstacle list ... get_obstacles_for_OBCA     :593-677
//   halfspaces ........... compute_polytope_halfspaces (pypoman/cdd as R/obca_py/optimizer.py:184-186 calls it;
//                          the repo's geometry.polytope_halfspaces restatement)
//
// The reference's global np.random draws (one uniform(-l_std, l_std) per tree row in create_tree_rows,
// one uniform(-0.5, 0.5) per row for the centre-line fit) are inputs: the host draws them from the same
// MT19937 stream, so a scene is the reference's scene.  One thread runs one scene (the work per scene
// is a few thousand flops of sequential geometry); polygons are written in the reference's order.
#pragma once
#include <cmath>
#include <cstdint>

#ifndef HTP_HD
#error "define HTP_HD before including oge_core.h"
#endif

#include "htp_libm.h"

namespace htp {
namespace oge {

constexpr int MAXR = 32;             // tree rows per scene
constexpr int MAXC = 2 * MAXR;       // field contour points
constexpr int MAXPOLY = 32;          // obstacle polygons per scene
constexpr int MAXV = 12;             // vertices per polygon
constexpr int NEAR = 1, FAR = -1;    // OrchardGeometryEnvironment.NEAR_SIDE / FAR_SIDE
constexpr double SAFETY_BOUND = 0.2; // orchard_environment_OBCA.SAFETY_BOUND
constexpr double RDP_EPS = 0.15;     // create_boundary_polygons epsilon
constexpr double COVER_WIDTH = 2.0;  // cover_side_points / get_obstacles_for_OBCA width
constexpr double BUFFER_DIST = 1.0;  // get_obstacles_for_OBCA buffer_distance

enum Status { OK = 0, ST_BAD_INPUT = 1, ST_NO_ROW_BETWEEN = 2, ST_OVERFLOW = 3, ST_EMPTY_SIDE = 4 };

// One scene (all lengths in metres, angles in radians).
struct SceneIn {
  int nrows;
  double row_width, row_length, slope, tree_width, headland_width;
  const double* row_draws;   // [nrows]  create_tree_rows' uniform(-l_std, l_std) draws
  const double* eps_draws;   // [nrows]  create_headland_countour_lines' uniform(-0.5, 0.5) draws
  double start[3], end[3];
  int side;                  // NEAR (1) or FAR (-1)
};

struct PolyOut {
  int n;                     // polygons
  int nv[MAXPOLY];
  double xy[MAXPOLY][MAXV][2];
};

HTP_HD inline double sgn(double v) { return v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0); }

// np.polyfit(x, y, 1) -> (k, b), least squares in centred form
HTP_HD inline void polyfit1(const double* x, const double* y, int n, double& k, double& b) {
  double mx = 0, my = 0;
  for (int i = 0; i < n; ++i) { mx += x[i]; my += y[i]; }
  mx /= n;
  my /= n;
  double sxx = 0, sxy = 0;
  for (int i = 0; i < n; ++i) { sxx += (x[i] - mx) * (x[i] - mx); sxy += (x[i] - mx) * (y[i] - my); }
  k = sxy / sxx;
  b = my - k * mx;
}

HTP_HD inline double pstd(const double* x, int n) {   // np.std (ddof = 0)
  double m = 0;
  for (int i = 0; i < n; ++i) m += x[i];
  m /= n;
  double s = 0;
  for (int i = 0; i < n; ++i) s += (x[i] - m) * (x[i] - m);
  return sqrt(s / n);
}

HTP_HD inline double round7(double v) { return rint(v * 1e7) / 1e7; }   // np.round(v, 7)

struct Scene {
  int n;
  double rx[MAXR][2], ry[MAXR][2];   // row r: near end (0), far end (1)
  double row_width;                  // abs(mean(diff(near ys)))  (orchard_environment_OBCA.__init__)
};

// create_tree_rows(row_num, row_width, row_lengths, slope_angle, l_std) with the given draws
HTP_HD inline void make_rows(const SceneIn& in, Scene& S) {
  S.n = in.nrows;
  const double dx = in.row_width * hm::tan(in.slope);
  for (int i = 0; i < S.n; ++i) {
    const double y = in.row_width * i;
    double x = dx * i;
    x += in.row_draws[i];
    S.rx[i][0] = x;
    S.ry[i][0] = y;
    S.rx[i][1] = x + in.row_length;
    S.ry[i][1] = y;
  }
  double acc = 0;
  for (int i = 1; i < S.n; ++i) acc += S.ry[i][0] - S.ry[i - 1][0];
  S.row_width = fabs(acc / (S.n - 1));
}

// get_headland_angle(side) :463-472
HTP_HD inline double headland_angle(const Scene& S, int side) {
  const int e = side == NEAR ? 0 : 1;
  double xs[MAXR], ys[MAXR];
  for (int i = 0; i < S.n; ++i) { xs[i] = S.rx[i][e]; ys[i] = S.ry[i][e]; }
  if (pstd(xs, S.n) < 0.01) return 3.141592653589793 / 2;
  double k, b;
  polyfit1(xs, ys, S.n, k, b);
  return hm::atan(k);
}

// get_map_exterior_pts(headland_width) :288-334 -> 2 n points (near rows, then far rows reversed)
HTP_HD inline int exterior_pts(const Scene& S, double hw, double (*P)[2]) {
  const int n = S.n;
  double acc = 0;
  for (int i = 1; i < n; ++i) acc += S.ry[i][0] - S.ry[i - 1][0];
  const double rw = acc / (n - 1);
  const double na = headland_angle(S, NEAR), fa = headland_angle(S, FAR);
  const double dxn = fabs(hw / hm::sin(na)), dxf = fabs(hw / hm::sin(fa));
  int up = 0, lo = 0;
  for (int i = 0; i < n; ++i) {
    P[i][0] = S.rx[i][0] - dxn;
    P[i][1] = S.ry[i][0];
  }
  for (int i = 1; i < n; ++i) if (P[i][1] > P[up][1]) up = i;
  P[up][1] += rw;
  double d = fabs(hm::sin(na)) < 1e-5 ? 0.0 : rw / hm::tan(na);
  P[up][0] += d;
  for (int i = 1; i < n; ++i) if (P[i][1] < P[lo][1]) lo = i;
  P[lo][1] -= rw;
  P[lo][0] -= d;
  double (*F)[2] = P + n;
  for (int i = 0; i < n; ++i) {
    F[i][0] = S.rx[n - 1 - i][1] + dxf;
    F[i][1] = S.ry[n - 1 - i][1];
  }
  up = 0;
  lo = 0;
  d = fabs(hm::sin(fa)) < 1e-5 ? 0.0 : rw / hm::tan(fa);
  for (int i = 1; i < n; ++i) if (F[i][1] > F[up][1]) up = i;
  F[up][1] += rw;
  F[up][0] += d;
  for (int i = 1; i < n; ++i) if (F[i][1] < F[lo][1]) lo = i;
  F[lo][1] -= rw;
  F[lo][0] -= d;
  return 2 * n;
}

// rdp.pldist
HTP_HD inline double pldist(const double* p, const double* s, const double* e) {
  if (s[0] == e[0] && s[1] == e[1]) return sqrt((p[0] - s[0]) * (p[0] - s[0]) + (p[1] - s[1]) * (p[1] - s[1]));
  const double ex = e[0] - s[0], ey = e[1] - s[1], sx = s[0] - p[0], sy = s[1] - p[1];
  return fabs(ex * sy - ey * sx) / sqrt(ex * ex + ey * ey);
}

// rdp(M, epsilon): recursive Ramer-Douglas-Peucker (first farthest point on ties), written as an explicit
// stack of [a, b] spans marking the kept points; the kept points in order are rdp's output.
HTP_HD inline int rdp(const double (*M)[2], int n, double eps, double (*out)[2]) {
  if (n <= 0) return 0;
  bool keep[MAXC];
  for (int i = 0; i < n; ++i) keep[i] = false;
  keep[0] = keep[n - 1] = true;
  int sa[MAXC], sb[MAXC], top = 0;
  sa[top] = 0;
  sb[top] = n - 1;
  ++top;
  while (top > 0) {
    --top;
    const int a = sa[top], b = sb[top];
    double dmax = 0.0;
    int idx = -1;
    for (int i = a + 1; i < b + 1; ++i) {   // rdp_rec scans M[1:] of the span (the end point included)
      const double dd = pldist(M[i], M[a], M[b]);
      if (dd > dmax) { idx = i; dmax = dd; }
    }
    if (dmax > eps) {
      keep[idx] = true;
      sa[top] = idx; sb[top] = b; ++top;
      sa[top] = a; sb[top] = idx; ++top;
    }
  }
  int m = 0;
  for (int i = 0; i < n; ++i)
    if (keep[i]) { out[m][0] = M[i][0]; out[m][1] = M[i][1]; ++m; }
  return m;
}

HTP_HD inline void along_rect(const double* A, const double* B, double d, double* p1, double* p2) {
  const double mx = (A[0] + B[0]) / 2.0, my = (A[1] + B[1]) / 2.0;
  const double L = sqrt((B[0] - A[0]) * (B[0] - A[0]) + (B[1] - A[1]) * (B[1] - A[1]));
  const double nx = (B[1] - A[1]) / L, ny = -(B[0] - A[0]) / L;
  const double ex = mx + nx * d, ey = my + ny * d;
  const double hx = (A[0] - B[0]) / 2, hy = (A[1] - B[1]) / 2;
  p1[0] = ex + hx; p1[1] = ey + hy;
  p2[0] = ex - hx; p2[1] = ey - hy;
}

struct Quads {
  int n;
  double q[MAXC][4][2];
};

// cover_side_points(contour_points, side, width=2) OGE_OBCA.py:171-262
HTP_HD inline int cover_side_points(const double (*cp)[2], int n, int side, Quads& Q) {
  Q.n = 0;
  if (n < 2) return ST_EMPTY_SIDE;
  double xs[MAXC], ys[MAXC];
  for (int i = 0; i < n; ++i) { xs[i] = cp[i][0]; ys[i] = cp[i][1]; }
  const double shift = side == NEAR ? -COVER_WIDTH : COVER_WIDTH;
  if (pstd(xs, n) < 1e-3 || n == 2) {
    int up = 0, dn = 0;
    for (int i = 1; i < n; ++i) { if (ys[i] > ys[up]) up = i; if (ys[i] < ys[dn]) dn = i; }
    double (*q)[2] = Q.q[0];
    q[0][0] = xs[up] + shift; q[0][1] = ys[up];
    q[1][0] = xs[up]; q[1][1] = ys[up];
    q[2][0] = xs[dn]; q[2][1] = ys[dn];
    q[3][0] = xs[dn] + shift; q[3][1] = ys[dn];
    Q.n = 1;
    return OK;
  }
  double k, b;
  polyfit1(ys, xs, n, k, b);
  double dsum = 0, dbest = -1;
  int cnt = 0, far = -1;
  const double den = sqrt(1.0 + k * k);
  for (int i = 0; i < n; ++i) {
    const double v = xs[i] - k * ys[i] - b;
    if (side == NEAR ? v >= 0 : v <= 0) {
      const double dd = fabs(xs[i] + (-k) * ys[i] + (-b)) / den;
      dsum += dd;
      ++cnt;
      if (dd > dbest) { dbest = dd; far = i; }
    }
  }
  if (cnt > 0 && dsum / cnt < 0.1) {
    const double bmax = xs[far] - k * ys[far];
    double maxy = ys[0], miny = ys[0];
    for (int i = 1; i < n; ++i) { maxy = ys[i] > maxy ? ys[i] : maxy; miny = ys[i] < miny ? ys[i] : miny; }
    const double ux = maxy * k + bmax, dx = miny * k + bmax;
    double (*q)[2] = Q.q[0];
    q[0][0] = ux + shift; q[0][1] = maxy;
    q[1][0] = ux; q[1][1] = maxy;
    q[2][0] = dx; q[2][1] = miny;
    q[3][0] = dx + shift; q[3][1] = miny;
    Q.n = 1;
    return OK;
  }
  const double ds = (side == NEAR ? -COVER_WIDTH : COVER_WIDTH) * sgn(cp[1][1] - cp[0][1]);
  for (int i = 0; i + 1 < n; ++i) {
    double (*q)[2] = Q.q[Q.n++];
    q[0][0] = cp[i][0]; q[0][1] = cp[i][1];
    q[1][0] = cp[i + 1][0]; q[1][1] = cp[i + 1][1];
    along_rect(cp[i], cp[i + 1], ds, q[2], q[3]);
  }
  return OK;
}

HTP_HD inline void put(PolyOut& out, const double (*v)[2], int nv) {
  out.nv[out.n] = nv;
  for (int j = 0; j < nv; ++j) { out.xy[out.n][j][0] = v[j][0]; out.xy[out.n][j][1] = v[j][1]; }
  ++out.n;
}

// _row_rect of get_obstacle_tree_rows (SAFETY_BOUND past the row ends, tree_width / 2 across)
HTP_HD inline void row_rect(const Scene& S, int r, double tw, bool rnd, double (*v)[2]) {
  v[0][0] = S.rx[r][0] - SAFETY_BOUND; v[0][1] = S.ry[r][0] - tw / 2.0;
  v[1][0] = S.rx[r][0] - SAFETY_BOUND; v[1][1] = S.ry[r][0] + tw / 2.0;
  v[2][0] = S.rx[r][1] + SAFETY_BOUND; v[2][1] = S.ry[r][1] + tw / 2.0;
  v[3][0] = S.rx[r][1] + SAFETY_BOUND; v[3][1] = S.ry[r][1] - tw / 2.0;
  if (rnd)
    for (int j = 0; j < 4; ++j) { v[j][0] = round7(v[j][0]); v[j][1] = round7(v[j][1]); }
}

HTP_HD inline double point_side(const double* A, const double* B, const double* C) {
  return sgn((B[0] - A[0]) * (C[1] - A[1]) - (B[1] - A[1]) * (C[0] - A[0]));
}

// The whole producer: orchard rows -> create_boundary_polygons -> get_obstacle_tree_rows ->
// get_obstacles_for_OBCA.  Returns a Status; `out` holds the polygons in the reference's order.
HTP_HD inline int produce(const SceneIn& in, PolyOut& out) {
  out.n = 0;
  if (in.nrows < 3 || in.nrows > MAXR || !(in.side == NEAR || in.side == FAR)) return ST_BAD_INPUT;
  Scene S;
  make_rows(in, S);
  const int n = S.n;
  // create_headland_countour_lines :66-91 on the field polygon's exterior points
  double P[MAXC][2];
  const int np_ = exterior_pts(S, in.headland_width, P);
  double cx[MAXR], cy[MAXR];
  for (int i = 0; i < n; ++i) {
    cx[i] = (S.rx[i][0] + S.rx[i][1]) / 2.0 + in.eps_draws[i];
    cy[i] = (S.ry[i][0] + S.ry[i][1]) / 2.0;
  }
  double k, b;
  polyfit1(cx, cy, n, k, b);
  const double origin = sgn(0 * k + b - 0);
  double side_pts[MAXC][2];
  int ns = 0;
  for (int i = 0; i < np_; ++i) {
    const bool near = sgn(P[i][0] * k + b - P[i][1]) == origin;
    if (near == (in.side == NEAR)) { side_pts[ns][0] = P[i][0]; side_pts[ns][1] = P[i][1]; ++ns; }
  }
  double red[MAXC][2];
  const int nr = rdp(side_pts, ns, RDP_EPS, red);
  Quads Q;
  int st = cover_side_points(red, nr, in.side, Q);
  if (st != OK) return st;
  // up / low bound quads (create_boundary_polygons :336-371)
  int ui = 0, li = 0;
  for (int i = 1; i < n; ++i) { if (S.ry[i][0] > S.ry[ui][0]) ui = i; if (S.ry[i][0] < S.ry[li][0]) li = i; }
  double upq[4][2], loq[4][2];
  {
    const double rw = S.row_width;
    upq[0][0] = S.rx[ui][0] - 8; upq[0][1] = S.ry[ui][0] + rw;
    upq[1][0] = S.rx[ui][0] - 8; upq[1][1] = S.ry[ui][0] + rw + 1;
    upq[2][0] = S.rx[ui][1] + 8; upq[2][1] = S.ry[ui][1] + rw + 1;
    upq[3][0] = S.rx[ui][1] + 8; upq[3][1] = S.ry[ui][1] + rw;
    loq[0][0] = S.rx[li][0] - 8; loq[0][1] = S.ry[li][0] - rw;
    loq[1][0] = S.rx[li][0] - 8; loq[1][1] = S.ry[li][0] - rw - 1;
    loq[2][0] = S.rx[li][1] + 8; loq[2][1] = S.ry[li][1] - rw - 1;
    loq[3][0] = S.rx[li][1] + 8; loq[3][1] = S.ry[li][1] - rw;
  }
  // get_obstacles_for_OBCA :593-677, part 1: the side's boundary quads, combined into convex chains
  if (Q.n <= 1) {
    put(out, Q.q[0], 4);
  } else {
    const double ymax = in.start[1] > in.end[1] ? in.start[1] : in.end[1];
    const double ymin = in.start[1] < in.end[1] ? in.start[1] : in.end[1];
    int sel[MAXC], nsel = 0;
    for (int i = 0; i < Q.n; ++i) {
      const double a = Q.q[i][0][1], c = Q.q[i][1][1];
      const double pmin = a < c ? a : c, pmax = a > c ? a : c;
      if (pmax > ymin - BUFFER_DIST && pmin < ymax + BUFFER_DIST) sel[nsel++] = i;
    }
    if (nsel == 0) return ST_EMPTY_SIDE;   // the reference indexes rectangle_obstacles[-1] (IndexError)
    double cp[MAXC + 1][2];
    int nc = 0;
    for (int t = 0; t < nsel; ++t) { cp[nc][0] = Q.q[sel[t]][0][0]; cp[nc][1] = Q.q[sel[t]][0][1]; ++nc; }
    cp[nc][0] = Q.q[sel[nsel - 1]][1][0];
    cp[nc][1] = Q.q[sel[nsel - 1]][1][1];
    ++nc;
    double dsg = in.side == NEAR ? -COVER_WIDTH : COVER_WIDTH;
    double dir = in.side == NEAR ? 1.0 : -1.0;
    const double ydir = sgn(cp[1][1] - cp[0][1]);
    dsg *= ydir;
    dir *= ydir;
    double cur[MAXV][2];
    int ncur = 0, e = 1;
    auto restart = [&](int s_, int e_) {
      cur[0][0] = cp[s_][0]; cur[0][1] = cp[s_][1];
      cur[1][0] = cp[e_][0]; cur[1][1] = cp[e_][1];
      ncur = 2;
    };
    auto close = [&]() -> bool {
      if (ncur + 2 > MAXV || out.n >= MAXPOLY) return false;
      along_rect(cur[0], cur[ncur - 1], dsg, cur[ncur], cur[ncur + 1]);
      put(out, cur, ncur + 2);
      return true;
    };
    restart(0, 1);
    while (e < nc - 1) {
      if (point_side(cp[e - 1], cp[e], cp[e + 1]) == dir) {
        if (ncur + 1 > MAXV - 2) return ST_OVERFLOW;
        cur[ncur][0] = cp[e + 1][0];
        cur[ncur][1] = cp[e + 1][1];
        ++ncur;
        ++e;
      } else {
        if (!close()) return ST_OVERFLOW;
        restart(e, e + 1);
        e = e + 1;
      }
    }
    if (!close()) return ST_OVERFLOW;
  }
  // part 2: the up or low bound quad
  if (out.n >= MAXPOLY) return ST_OVERFLOW;
  put(out, in.start[1] > in.end[1] ? loq : upq, 4);
  // part 3: get_obstacle_tree_rows :477-591
  const double hi = in.start[1] > in.end[1] ? in.start[1] : in.end[1];
  const double lo = in.start[1] < in.end[1] ? in.start[1] : in.end[1];
  int low_idx = -1, up_idx = -1;
  for (int i = 0; i < n; ++i)
    if (S.ry[i][0] > lo && S.ry[i][0] < hi) { if (low_idx < 0) low_idx = i; up_idx = i; }
  if (low_idx < 0) return ST_NO_ROW_BETWEEN;
  int a, c;
  bool rnd;
  if (low_idx == up_idx) {
    a = up_idx - 2 > 0 ? up_idx - 2 : 0;
    c = up_idx + 2 < n - 1 ? up_idx + 2 : n - 1;
    rnd = true;
  } else {
    a = low_idx - 2 > 0 ? low_idx - 2 : 0;
    c = up_idx + 3 < n - 1 ? up_idx + 3 : n - 1;
    rnd = false;
  }
  for (int r = a; r < c; ++r) {
    if (out.n >= MAXPOLY) return ST_OVERFLOW;
    double v[4][2];
    row_rect(S, r, in.tree_width, rnd, v);
    put(out, v, 4);
  }
  return OK;
}

// compute_polytope_halfspaces of one convex polygon (geometry.polytope_halfspaces): vertices rounded to 7
// decimals, monotone-chain hull counter-clockwise from the lexicographically smallest vertex (collinear
// points dropped), rows [b | -A] scaled by their smallest |entry| > 1e-7, rounded to 7 decimals.
// Returns the facet count (or -1 for fewer than 3 distinct vertices).
HTP_HD inline int halfspaces(const double (*v)[2], int nv, double* A, double* b) {
  double P[MAXV][2];
  int m = 0;
  for (int i = 0; i < nv; ++i) { P[m][0] = round7(v[i][0]); P[m][1] = round7(v[i][1]); ++m; }
  for (int i = 1; i < m; ++i) {   // insertion sort, lexicographic
    double x = P[i][0], y = P[i][1];
    int j = i - 1;
    while (j >= 0 && (P[j][0] > x || (P[j][0] == x && P[j][1] > y))) { P[j + 1][0] = P[j][0]; P[j + 1][1] = P[j][1]; --j; }
    P[j + 1][0] = x;
    P[j + 1][1] = y;
  }
  int u = 0;   // np.unique
  for (int i = 0; i < m; ++i)
    if (u == 0 || P[i][0] != P[u - 1][0] || P[i][1] != P[u - 1][1]) { P[u][0] = P[i][0]; P[u][1] = P[i][1]; ++u; }
  if (u < 3) return -1;
  double H[2 * MAXV][2];
  int nh = 0;
  for (int pass = 0; pass < 2; ++pass) {
    double C[2 * MAXV][2];
    int nc = 0;
    for (int t = 0; t < u; ++t) {
      const double* p = pass == 0 ? P[t] : P[u - 1 - t];
      while (nc >= 2) {
        const double* o = C[nc - 2];
        const double* a = C[nc - 1];
        if ((a[0] - o[0]) * (p[1] - o[1]) - (a[1] - o[1]) * (p[0] - o[0]) > 0) break;
        --nc;
      }
      C[nc][0] = p[0];
      C[nc][1] = p[1];
      ++nc;
    }
    for (int t = 0; t + 1 < nc; ++t) { H[nh][0] = C[t][0]; H[nh][1] = C[t][1]; ++nh; }
  }
  for (int f = 0; f < nh; ++f) {
    const double* h = H[f];
    const double* q = H[(f + 1) % nh];
    const double nx = q[1] - h[1], ny = h[0] - q[0];
    double row[3] = {nx * h[0] + ny * h[1], -nx, -ny};
    double sc = INFINITY;
    for (int j = 0; j < 3; ++j) {
      const double mg = fabs(row[j]);
      if (mg > 1e-7 && mg < sc) sc = mg;
    }
    if (!(sc < INFINITY)) sc = 1.0;
    for (int j = 0; j < 3; ++j) row[j] /= sc;
    A[2 * f] = round7(-row[1]);
    A[2 * f + 1] = round7(-row[2]);
    b[f] = round7(row[0]);
  }
  return nh;
}

}  // namespace oge
}  // namespace htp
