// Dubins shortest path + arc-length cubic spline, as the reference's Pawn goal
// shot builds them (R/path_planner/hybrid_a_star_search.py get_dubins_path
// :289-304):
//   * pydubins (dubins.c): intermediate results, the six words LSL LSR RSL RSR
//     RLR LRL in that order (a strictly cheaper word wins), dubins_segment /
//     dubins_path_sample, sample_many (x = 0, x += step while x < length);
//   * R/path_planner/utils/cubic_spline.py calc_spline_course :92-112 over
//     scipy.interpolate.CubicSpline (not-a-knot): consecutive duplicate points
//     dropped, s = [0] + cumsum(hypot), the tridiagonal slope system of
//     scipy's CubicSpline (n == 2: the chord slope; n == 3: the parabola), the
//     Hermite coefficients of CubicHermiteSpline, PPoly evaluation (scipy's
//     evaluate_poly1 term order, find_interval_ascending with extrapolation),
//     yaw = atan2(y', x'), curvature (y''x' - x''y') / (x'^2 + y'^2)^1.5.
// The tridiagonal solve is Gaussian elimination with partial pivoting (LAPACK
// gtsv style); scipy calls gbsv, so the last bits may differ.
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#ifndef HTP_HD
#error "define HTP_HD before including dubins_core.h"
#endif

#include "htp_libm.h"

namespace htp {
namespace dub {

constexpr double TWO_PI = 6.283185307179586;
enum { LSL, LSR, RSL, RSR, RLR, LRL };
enum { SL, SS, SR };

HTP_HD inline double mod2pi(double t) { return t - TWO_PI * floor(t / TWO_PI); }

HTP_HD inline int seg_type(int word, int k) {
  const int8_t T[6][3] = {{SL, SS, SL}, {SL, SS, SR}, {SR, SS, SL}, {SR, SS, SR}, {SR, SL, SR}, {SL, SR, SL}};
  return T[word][k];
}

struct Path {
  double q0[3];
  double prm[3];
  double rho;
  int word;
};

// dubins_shortest_path; false when no word exists
HTP_HD inline bool shortest(const double* q0, const double* q1, double rho, Path& P) {
  const double dx = q1[0] - q0[0], dy = q1[1] - q0[1];
  const double D = sqrt(dx * dx + dy * dy);
  const double d = D / rho;
  const double th = d > 0 ? mod2pi(hm::atan2(dy, dx)) : 0.0;
  const double a = mod2pi(q0[2] - th), b = mod2pi(q1[2] - th);
  const double sa = hm::sin(a), sb = hm::sin(b), ca = hm::cos(a), cb = hm::cos(b);
  const double cab = hm::cos(a - b), dd = d * d;
  double best = __builtin_huge_val();
  int bw = -1;
  double bp[3] = {0, 0, 0};
  auto take = [&](int w, double t, double p, double q) {
    const double c = t + p + q;
    if (c < best) { best = c; bw = w; bp[0] = t; bp[1] = p; bp[2] = q; }
  };
  double p2 = 2 + dd - (2 * cab) + (2 * d * (sa - sb));
  if (p2 >= 0) {
    const double t1 = hm::atan2(cb - ca, d + sa - sb);
    take(LSL, mod2pi(t1 - a), sqrt(p2), mod2pi(b - t1));
  }
  p2 = -2 + dd + (2 * cab) + (2 * d * (sa + sb));
  if (p2 >= 0) {
    const double p = sqrt(p2);
    const double t0 = hm::atan2(-ca - cb, d + sa + sb) - hm::atan2(-2.0, p);
    take(LSR, mod2pi(t0 - a), p, mod2pi(t0 - mod2pi(b)));
  }
  p2 = -2 + dd + (2 * cab) - (2 * d * (sa + sb));
  if (p2 >= 0) {
    const double p = sqrt(p2);
    const double t0 = hm::atan2(ca + cb, d - sa - sb) - hm::atan2(2.0, p);
    take(RSL, mod2pi(a - t0), p, mod2pi(b - t0));
  }
  p2 = 2 + dd - (2 * cab) + (2 * d * (sb - sa));
  if (p2 >= 0) {
    const double t1 = hm::atan2(ca - cb, d - sa + sb);
    take(RSR, mod2pi(a - t1), sqrt(p2), mod2pi(t1 - b));
  }
  double t0 = (6. - dd + 2 * cab + 2 * d * (sa - sb)) / 8.;
  double phi = hm::atan2(ca - cb, d - sa + sb);
  if (fabs(t0) <= 1) {
    const double p = mod2pi(TWO_PI - hm::acos(t0));
    const double t = mod2pi(a - phi + mod2pi(p / 2.));
    take(RLR, t, p, mod2pi(a - b - t + mod2pi(p)));
  }
  t0 = (6. - dd + 2 * cab + 2 * d * (sb - sa)) / 8.;
  phi = hm::atan2(ca - cb, d + sa - sb);
  if (fabs(t0) <= 1) {
    const double p = mod2pi(TWO_PI - hm::acos(t0));
    const double t = mod2pi(-a - phi + p / 2.);
    take(LRL, t, p, mod2pi(mod2pi(b) - a - t + mod2pi(p)));
  }
  if (bw < 0) return false;
  P.q0[0] = q0[0]; P.q0[1] = q0[1]; P.q0[2] = q0[2];
  P.prm[0] = bp[0]; P.prm[1] = bp[1]; P.prm[2] = bp[2];
  P.rho = rho;
  P.word = bw;
  return true;
}

HTP_HD inline double length(const Path& P) {
  double l = 0.;
  l += P.prm[0];
  l += P.prm[1];
  l += P.prm[2];
  return l * P.rho;
}

HTP_HD inline void segment(double t, const double* qi, double* qt, int typ) {
  const double st = hm::sin(qi[2]), ct = hm::cos(qi[2]);
  if (typ == SL) { qt[0] = hm::sin(qi[2] + t) - st; qt[1] = -hm::cos(qi[2] + t) + ct; qt[2] = t; }
  else if (typ == SR) { qt[0] = -hm::sin(qi[2] - t) + st; qt[1] = hm::cos(qi[2] - t) - ct; qt[2] = -t; }
  else { qt[0] = ct * t; qt[1] = st * t; qt[2] = 0.0; }
  qt[0] += qi[0];
  qt[1] += qi[1];
  qt[2] += qi[2];
}

// dubins_path_sample at arc length t
HTP_HD inline void sample(const Path& P, double t, double* q) {
  const double tp = t / P.rho;
  const double qi[3] = {0.0, 0.0, P.q0[2]};
  double q1[3], q2[3];
  segment(P.prm[0], qi, q1, seg_type(P.word, 0));
  segment(P.prm[1], q1, q2, seg_type(P.word, 1));
  if (tp < P.prm[0]) segment(tp, qi, q, seg_type(P.word, 0));
  else if (tp < (P.prm[0] + P.prm[1])) segment(tp - P.prm[0], q1, q, seg_type(P.word, 1));
  else segment(tp - P.prm[0] - P.prm[1], q2, q, seg_type(P.word, 2));
  q[0] = q[0] * P.rho + P.q0[0];
  q[1] = q[1] * P.rho + P.q0[1];
  q[2] = mod2pi(q[2]);
}

// ------------------------------------------------------------ cubic spline
// slopes d[0..n) of scipy's not-a-knot CubicSpline through (x[i], y[i]).
// work: 4n doubles.  Returns false for n < 2.
HTP_HD inline bool spline_slopes(const double* x, const double* y, int n, double* d, double* work) {
  if (n < 2) return false;
  if (n == 2) {
    const double sl = (y[1] - y[0]) / (x[1] - x[0]);
    d[0] = sl;
    d[1] = sl;
    return true;
  }
  const double dx0 = x[1] - x[0], dx1 = x[2] - x[1];
  if (n == 3) {  // parabola: [[1,1,0],[dx1, 2(dx0+dx1), dx0],[0,1,1]] s = b, Gaussian elimination w/ partial pivoting
    const double sl0 = (y[1] - y[0]) / dx0, sl1 = (y[2] - y[1]) / dx1;
    double A[3][4] = {{1.0, 1.0, 0.0, 2 * sl0},
                      {dx1, 2 * (dx0 + dx1), dx0, 3 * (dx0 * sl1 + dx1 * sl0)},
                      {0.0, 1.0, 1.0, 2 * sl1}};
    for (int k = 0; k < 3; ++k) {
      int piv = k;
      for (int r = k + 1; r < 3; ++r)
        if (fabs(A[r][k]) > fabs(A[piv][k])) piv = r;
      if (piv != k)
        for (int c = 0; c < 4; ++c) { const double t = A[k][c]; A[k][c] = A[piv][c]; A[piv][c] = t; }
      for (int r = k + 1; r < 3; ++r) {
        const double f = A[r][k] / A[k][k];
        for (int c = k; c < 4; ++c) A[r][c] -= f * A[k][c];
      }
    }
    for (int k = 2; k >= 0; --k) {
      double v = A[k][3];
      for (int c = k + 1; c < 3; ++c) v -= A[k][c] * d[c];
      d[k] = v / A[k][k];
    }
    return true;
  }
  // tridiagonal system: lower dl[i] = A(i+1, i), diagonal dg[i], upper du[i] = A(i, i+1), rhs b
  double* dl = work;
  double* dg = work + n;
  double* du = work + 2 * n;
  double* du2 = work + 3 * n;
  for (int i = 1; i < n - 1; ++i) {
    const double dxm = x[i] - x[i - 1], dxi = x[i + 1] - x[i];
    const double slm = (y[i] - y[i - 1]) / dxm, sli = (y[i + 1] - y[i]) / dxi;
    dg[i] = 2 * (dxm + dxi);
    du[i] = dxm;
    dl[i - 1] = dxi;
    d[i] = 3 * (dxi * slm + dxm * sli);
  }
  {
    const double sl0 = (y[1] - y[0]) / dx0, sl1 = (y[2] - y[1]) / dx1;
    const double dd = x[2] - x[0];
    dg[0] = dx1;
    du[0] = dd;
    d[0] = ((dx0 + 2 * dd) * dx1 * sl0 + dx0 * dx0 * sl1) / dd;
  }
  {
    const double dxa = x[n - 2] - x[n - 3], dxb = x[n - 1] - x[n - 2];
    const double sla = (y[n - 2] - y[n - 3]) / dxa, slb = (y[n - 1] - y[n - 2]) / dxb;
    const double dd = x[n - 1] - x[n - 3];
    dg[n - 1] = dxa;
    dl[n - 2] = dd;
    d[n - 1] = (dxb * dxb * sla + (2 * dd + dxb) * dxa * slb) / dd;
  }
  // elimination with partial pivoting (gtsv): du2 holds the fill-in
  for (int i = 0; i < n - 1; ++i) {
    if (fabs(dg[i]) >= fabs(dl[i])) {
      const double f = dl[i] / dg[i];
      dg[i + 1] -= f * du[i];
      d[i + 1] -= f * d[i];
      du2[i] = 0.0;
    } else {
      const double f = dg[i] / dl[i];
      dg[i] = dl[i];
      const double t = dg[i + 1];
      dg[i + 1] = du[i] - f * t;
      if (i < n - 2) {
        du2[i] = du[i + 1];
        du[i + 1] = -f * du2[i];
      } else {
        du2[i] = 0.0;
      }
      du[i] = t;
      const double tb = d[i];
      d[i] = d[i + 1];
      d[i + 1] = tb - f * d[i + 1];
    }
  }
  d[n - 1] = d[n - 1] / dg[n - 1];
  d[n - 2] = (d[n - 2] - du[n - 2] * d[n - 1]) / dg[n - 2];
  for (int i = n - 3; i >= 0; --i) d[i] = (d[i] - du[i] * d[i + 1] - du2[i] * d[i + 2]) / dg[i];
  return true;
}

// PPoly interval of v (scipy find_interval_ascending, extrapolating)
HTP_HD inline int interval(const double* x, int n, double v) {
  if (!(x[0] <= v && v <= x[n - 1])) return v < x[0] ? 0 : n - 2;
  if (v == x[n - 1]) return n - 2;
  int lo = 0, hi = n - 2;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (v < x[mid]) hi = mid - 1;
    else lo = mid;
  }
  return lo;
}

// value, first and second derivative of the Hermite cubic on interval i at v
HTP_HD inline void eval3(const double* x, const double* y, const double* d, int i, double v, double& f0, double& f1,
                         double& f2) {
  const double dx = x[i + 1] - x[i];
  const double sl = (y[i + 1] - y[i]) / dx;
  const double t = (d[i] + d[i + 1] - 2 * sl) / dx;
  const double c0 = t / dx, c1 = (sl - d[i]) / dx - t, c2 = d[i], c3 = y[i];
  const double s = v - x[i];
  // scipy evaluate_poly1: terms from the constant up, z = s^k accumulated
  f0 = 0.0;
  f0 = f0 + c3 * 1.0 * 1.0;
  double z = s;
  f0 = f0 + c2 * z * 1.0;
  z = z * s;
  f0 = f0 + c1 * z * 1.0;
  z = z * s;
  f0 = f0 + c0 * z * 1.0;
  f1 = 0.0;
  f1 = f1 + c2 * 1.0 * 1.0;
  z = s;
  f1 = f1 + c1 * z * 2.0;
  z = z * s;
  f1 = f1 + c0 * z * 3.0;
  f2 = 0.0;
  f2 = f2 + c1 * 1.0 * 2.0;
  f2 = f2 + c0 * s * 6.0;
}

}  // namespace dub
}  // namespace htp
