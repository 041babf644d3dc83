// Reeds-Shepp path enumeration + sampling (one query per thread).
//
// Behaviour of R/path_planner/utils/reeds_shepp.py calc_all_paths (:39-65):
// the 46 candidate words of the six families (:131-468) in the reference's
// order, its de-duplication rule (same ctypes and signed sum of length
// differences <= 0.01, :73-77), the MAX_LENGTH filter (:81), the sampler
// generate_local_course / interpolate (:471-562, including the trailing
// exact-0.0 pop) and the global transform (:46-62).  Arithmetic follows the
// reference expression order so the host build reproduces its doubles
// (tests build it with -fno-builtin so that libm is called exactly where
// CPython calls it: pow(x, 2.0) for `**2`, sin(-a) not folded to -sin(a)).
// On the device, ocml's sin/cos/tan/atan2/asin/acos may differ from glibc in
// the last ulp; parity there is structural-exact + coordinates within 1e-9.
#pragma once
#include <cmath>
#include <cstdint>

// Keep the reference's rounding: no a*b+c contraction into FMA on the device.
#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#ifndef HTP_HD
#error "define HTP_HD before including rs_core.h"
#endif

#include "htp_libm.h"
#include "htp_fastm.h"

namespace htp {
namespace rs {

constexpr int MAXP = 48;        // >= 46 candidates
constexpr double PI = 3.141592653589793;
constexpr double MAX_LENGTH = 1000.0;
enum Seg : int8_t { SEG_L = 0, SEG_S = 1, SEG_R = 2, SEG_NONE = 3 };

struct Path {
  double len[5];
  int8_t typ[5];
  int nseg;
  double L;  // normalised total length
};

struct PathSet {
  Path* p;   // MAXP slots (caller storage)
  int n;
  int err;   // 1: the reference would raise (assert L >= 0.01)
};

HTP_HD inline double pymod(double x, double y) {  // Python float %
  double r = fmod(x, y);
  if (r != 0.0) {
    if ((y < 0.0) != (r < 0.0)) r += y;
  } else {
    r = copysign(0.0, y);
  }
  return r;
}

HTP_HD inline double Mreg(double theta) {  // M(): regulate to [-pi, pi]
  double phi = pymod(theta, 2.0 * PI);
  if (phi < -PI) phi += 2.0 * PI;
  if (phi > PI) phi -= 2.0 * PI;
  return phi;
}

// math.hypot of CPython 3.10 (Modules/mathmodule.c vector_norm): not libm's
// hypot but an extended-precision sum of squares with a differential
// correction; the reference's R() (:607-614) uses it, so the words do too.
HTP_HD inline double py_hypot(double a, double b) {
  double v0 = fabs(a), v1 = fabs(b);
  const double mx = v0 > v1 ? v0 : v1;
  if (mx == __builtin_huge_val()) return mx;
  if (a != a || b != b) return a + b;
  if (mx == 0.0) return mx;
  int e;
  frexp(mx, &e);
  double post = 1.0;
  if (e < -1023) {  // tiny subnormal max: rescale by DBL_MIN like the original
    const double dmin = 2.2250738585072014e-308;
    v0 /= dmin;
    v1 /= dmin;
    frexp(mx / dmin, &e);
    post = dmin;
  }
  const double T27 = 134217729.0;  // 2^27 + 1 (Veltkamp split)
  const double scale = ldexp(1.0, -e);
  double csum = 1.0, f1 = 0.0, f2 = 0.0, f3 = 0.0, x, t, hi, lo, old;
  for (int i = 0; i < 2; ++i) {
    x = (i == 0 ? v0 : v1) * scale;
    t = x * T27;
    hi = t - (t - x);
    lo = x - hi;
    x = hi * hi;
    old = csum; csum += x; f1 += (old - csum) + x;
    x = 2.0 * hi * lo;
    old = csum; csum += x; f2 += (old - csum) + x;
    f3 += lo * lo;
  }
  const double h = sqrt(csum - 1.0 + (f1 + f2 + f3));
  x = h;
  t = x * T27;
  hi = t - (t - x);
  lo = x - hi;
  x = -hi * hi;
  old = csum; csum += x; f1 += (old - csum) + x;
  x = -2.0 * hi * lo;
  old = csum; csum += x; f2 += (old - csum) + x;
  x = -lo * lo;
  old = csum; csum += x; f3 += (old - csum) + x;
  x = csum - 1.0 + (f1 + f2 + f3);
  return post * ((h + x / (2.0 * h)) / scale);
}

HTP_HD inline double pi2pi(double t) {
  while (t > PI) t -= 2.0 * PI;
  while (t < -PI) t += 2.0 * PI;
  return t;
}

HTP_HD inline void add_path(PathSet& S, int n, const double* l, const int8_t* ty) {
  for (int k = 0; k < S.n; ++k) {
    const Path& e = S.p[k];
    if (e.nseg != n) continue;
    bool same = true;
    for (int j = 0; j < n; ++j) same = same && (e.typ[j] == ty[j]);
    if (!same) continue;
    double sum = 0.0;  // Python sum() of signed differences
    for (int j = 0; j < n; ++j) sum = sum + (e.len[j] - l[j]);
    if (sum <= 0.01) return;
  }
  double L = 0.0;
  for (int j = 0; j < n; ++j) L = L + fabs(l[j]);
  if (L >= MAX_LENGTH) return;
  if (!(L >= 0.01)) { S.err = 1; return; }
  if (S.n >= MAXP) { S.err = 2; return; }
  Path& q = S.p[S.n++];
  q.nseg = n;
  q.L = L;
  for (int j = 0; j < 5; ++j) {
    q.len[j] = j < n ? l[j] : 0.0;
    q.typ[j] = j < n ? ty[j] : SEG_NONE;
  }
}

// ---------------------------------------------------------------- words
HTP_HD inline bool w_SLS(double x, double y, double phi, double& t, double& u, double& v) {
  phi = Mreg(phi);
  if (y > 0.0 && 0.0 < phi && phi < PI * 0.99) {
    const double xd = -y / hm::tan(phi) + x;
    t = xd - hm::tan(phi / 2.0);
    u = phi;
    v = sqrt(hm::pow(x - xd, 2.0) + hm::pow(y, 2.0)) - hm::tan(phi / 2.0);
    return true;
  }
  if (y < 0.0 && 0.0 < phi && phi < PI * 0.99) {
    const double xd = -y / hm::tan(phi) + x;
    t = xd - hm::tan(phi / 2.0);
    u = phi;
    v = -sqrt(hm::pow(x - xd, 2.0) + hm::pow(y, 2.0)) - hm::tan(phi / 2.0);
    return true;
  }
  return false;
}

HTP_HD inline bool w_LSL(double x, double y, double phi, double& t, double& u, double& v) {
  const double a = x - hm::sin(phi), b = y - 1.0 + hm::cos(phi);
  u = py_hypot(a, b);
  t = hm::atan2(b, a);
  if (t >= 0.0) {
    v = Mreg(phi - t);
    if (v >= 0.0) return true;
  }
  return false;
}

HTP_HD inline bool w_LSR(double x, double y, double phi, double& t, double& u, double& v) {
  const double a = x + hm::sin(phi), b = y - 1.0 - hm::cos(phi);
  double u1 = py_hypot(a, b);
  const double t1 = hm::atan2(b, a);
  u1 = hm::pow(u1, 2.0);  // Python u1**2 (libm pow on the host harness)
  if (u1 >= 4.0) {
    u = sqrt(u1 - 4.0);
    const double theta = hm::atan2(2.0, u);
    t = Mreg(t1 + theta);
    v = Mreg(t - phi);
    if (t >= 0.0 && v >= 0.0) return true;
  }
  return false;
}

HTP_HD inline bool w_LRL(double x, double y, double phi, double& t, double& u, double& v) {
  const double a = x - hm::sin(phi), b = y - 1.0 + hm::cos(phi);
  const double u1 = py_hypot(a, b);
  const double t1 = hm::atan2(b, a);
  if (u1 <= 4.0) {
    u = -2.0 * hm::asin(0.25 * u1);
    t = Mreg(t1 + 0.5 * u + PI);
    v = Mreg(phi - t + u);
    if (t >= 0.0 && u <= 0.0) return true;
  }
  return false;
}

HTP_HD inline void tau_omega(double u, double v, double xi, double eta, double phi, double& tau, double& omega) {
  const double delta = Mreg(u - v);
  const double A = hm::sin(u) - hm::sin(delta);
  const double B = hm::cos(u) - hm::cos(delta) - 1.0;
  const double t1 = hm::atan2(eta * A - xi * B, xi * A + eta * B);
  const double t2 = 2.0 * (hm::cos(delta) - hm::cos(v) - hm::cos(u)) + 3.0;
  tau = (t2 < 0) ? Mreg(t1 + PI) : Mreg(t1);
  omega = Mreg(tau - u + v - phi);
}

HTP_HD inline bool w_LRLRn(double x, double y, double phi, double& t, double& u, double& v) {
  const double xi = x + hm::sin(phi), eta = y - 1.0 - hm::cos(phi);
  const double rho = 0.25 * (2.0 + sqrt(xi * xi + eta * eta));
  if (rho <= 1.0) {
    u = hm::acos(rho);
    tau_omega(u, -u, xi, eta, phi, t, v);
    if (t >= 0.0 && v <= 0.0) return true;
  }
  return false;
}

HTP_HD inline bool w_LRLRp(double x, double y, double phi, double& t, double& u, double& v) {
  const double xi = x + hm::sin(phi), eta = y - 1.0 - hm::cos(phi);
  const double rho = (20.0 - xi * xi - eta * eta) / 16.0;
  if (0.0 <= rho && rho <= 1.0) {
    u = -hm::acos(rho);
    if (u >= -0.5 * PI) {
      tau_omega(u, u, xi, eta, phi, t, v);
      if (t >= 0.0 && v >= 0.0) return true;
    }
  }
  return false;
}

HTP_HD inline bool w_LRSR(double x, double y, double phi, double& t, double& u, double& v) {
  const double xi = x + hm::sin(phi), eta = y - 1.0 - hm::cos(phi);
  const double rho = py_hypot(-eta, xi), theta = hm::atan2(xi, -eta);
  if (rho >= 2.0) {
    t = theta;
    u = 2.0 - rho;
    v = Mreg(t + 0.5 * PI - phi);
    if (t >= 0.0 && u <= 0.0 && v <= 0.0) return true;
  }
  return false;
}

HTP_HD inline bool w_LRSL(double x, double y, double phi, double& t, double& u, double& v) {
  const double xi = x - hm::sin(phi), eta = y - 1.0 + hm::cos(phi);
  const double rho = py_hypot(xi, eta), theta = hm::atan2(eta, xi);
  if (rho >= 2.0) {
    const double r = sqrt(rho * rho - 4.0);
    u = 2.0 - r;
    t = Mreg(theta + hm::atan2(r, -2.0));
    v = Mreg(phi - 0.5 * PI - t);
    if (t >= 0.0 && u <= 0.0 && v <= 0.0) return true;
  }
  return false;
}

HTP_HD inline bool w_LRSLR(double x, double y, double phi, double& t, double& u, double& v) {
  const double xi = x + hm::sin(phi), eta = y - 1.0 - hm::cos(phi);
  const double rho = py_hypot(xi, eta);
  if (rho >= 2.0) {
    u = 4.0 - sqrt(rho * rho - 4.0);
    if (u <= 0.0) {
      t = Mreg(hm::atan2((4.0 - u) * xi - 2.0 * eta, -2.0 * xi + (u - 4.0) * eta));
      v = Mreg(t - phi);
      if (t >= 0.0 && v >= 0.0) return true;
    }
  }
  return false;
}

// One table row: word kind, argument reflection, how (t,u,v) map to lengths, segment types.
enum Word : int8_t { W_SLS, W_LSL, W_LSR, W_LRL, W_LRLRn, W_LRLRp, W_LRSL, W_LRSR, W_LRSLR };
// arg mode: 0 (x,y,phi) 1 (-x,y,-phi) 2 (x,-y,-phi) 3 (-x,-y,phi); +4: backwards (xb,yb) variant
// len mode: see lengths_of()
struct Cand { int8_t word, arg, lmode, n; int8_t ty[5]; };

#define L_ SEG_L
#define S_ SEG_S
#define R_ SEG_R
#define X_ SEG_NONE
// lmode: 0 [t,u,v] 1 [-t,-u,-v] 2 [v,u,t] 3 [-v,-u,-t]
//        4 [t,u,-u,v] 5 [-t,-u,u,-v] 6 [t,u,u,v] 7 [-t,-u,-u,-v]
//        8 [t,-pi/2,u,v] 9 [-t,pi/2,-u,-v] 10 [v,u,-pi/2,t] 11 [-v,-u,pi/2,-t]
//        12 [t,-pi/2,u,-pi/2,v] 13 [-t,pi/2,-u,pi/2,-v]
HTP_HD inline const Cand* cand_table() {
  static constexpr Cand T[46] = {
      {W_SLS, 0, 0, 3, {S_, L_, S_, X_, X_}},  {W_SLS, 2, 0, 3, {S_, R_, S_, X_, X_}},
      {W_LSL, 0, 0, 3, {L_, S_, L_, X_, X_}},  {W_LSL, 1, 1, 3, {L_, S_, L_, X_, X_}},
      {W_LSL, 2, 0, 3, {R_, S_, R_, X_, X_}},  {W_LSL, 3, 1, 3, {R_, S_, R_, X_, X_}},
      {W_LSR, 0, 0, 3, {L_, S_, R_, X_, X_}},  {W_LSR, 1, 1, 3, {L_, S_, R_, X_, X_}},
      {W_LSR, 2, 0, 3, {R_, S_, L_, X_, X_}},  {W_LSR, 3, 1, 3, {R_, S_, L_, X_, X_}},
      {W_LRL, 0, 0, 3, {L_, R_, L_, X_, X_}},  {W_LRL, 1, 1, 3, {L_, R_, L_, X_, X_}},
      {W_LRL, 2, 0, 3, {R_, L_, R_, X_, X_}},  {W_LRL, 3, 1, 3, {R_, L_, R_, X_, X_}},
      {W_LRL, 4, 2, 3, {L_, R_, L_, X_, X_}},  {W_LRL, 5, 3, 3, {L_, R_, L_, X_, X_}},
      {W_LRL, 6, 2, 3, {R_, L_, R_, X_, X_}},  {W_LRL, 7, 3, 3, {R_, L_, R_, X_, X_}},
      {W_LRLRn, 0, 4, 4, {L_, R_, L_, R_, X_}}, {W_LRLRn, 1, 5, 4, {L_, R_, L_, R_, X_}},
      {W_LRLRn, 2, 4, 4, {R_, L_, R_, L_, X_}}, {W_LRLRn, 3, 5, 4, {R_, L_, R_, L_, X_}},
      {W_LRLRp, 0, 6, 4, {L_, R_, L_, R_, X_}}, {W_LRLRp, 1, 7, 4, {L_, R_, L_, R_, X_}},
      {W_LRLRp, 2, 6, 4, {R_, L_, R_, L_, X_}}, {W_LRLRp, 3, 7, 4, {R_, L_, R_, L_, X_}},
      {W_LRSL, 0, 8, 4, {L_, R_, S_, L_, X_}}, {W_LRSL, 1, 9, 4, {L_, R_, S_, L_, X_}},
      {W_LRSL, 2, 8, 4, {R_, L_, S_, R_, X_}}, {W_LRSL, 3, 9, 4, {R_, L_, S_, R_, X_}},
      {W_LRSR, 0, 8, 4, {L_, R_, S_, R_, X_}}, {W_LRSR, 1, 9, 4, {L_, R_, S_, R_, X_}},
      {W_LRSR, 2, 8, 4, {R_, L_, S_, L_, X_}}, {W_LRSR, 3, 9, 4, {R_, L_, S_, L_, X_}},
      {W_LRSL, 4, 10, 4, {L_, S_, R_, L_, X_}}, {W_LRSL, 5, 11, 4, {L_, S_, R_, L_, X_}},
      {W_LRSL, 6, 10, 4, {R_, S_, L_, R_, X_}}, {W_LRSL, 7, 11, 4, {R_, S_, L_, R_, X_}},
      {W_LRSR, 4, 10, 4, {R_, S_, R_, L_, X_}}, {W_LRSR, 5, 11, 4, {R_, S_, R_, L_, X_}},
      {W_LRSR, 6, 10, 4, {L_, S_, L_, R_, X_}}, {W_LRSR, 7, 11, 4, {L_, S_, L_, R_, X_}},
      {W_LRSLR, 0, 12, 5, {L_, R_, S_, L_, R_}}, {W_LRSLR, 1, 13, 5, {L_, R_, S_, L_, R_}},
      {W_LRSLR, 2, 12, 5, {R_, L_, S_, R_, L_}}, {W_LRSLR, 3, 13, 5, {R_, L_, S_, R_, L_}},
  };
  return T;
}
#undef L_
#undef S_
#undef R_
#undef X_

HTP_HD inline bool eval_word(int w, double x, double y, double phi, double& t, double& u, double& v) {
  switch (w) {
    case W_SLS: return w_SLS(x, y, phi, t, u, v);
    case W_LSL: return w_LSL(x, y, phi, t, u, v);
    case W_LSR: return w_LSR(x, y, phi, t, u, v);
    case W_LRL: return w_LRL(x, y, phi, t, u, v);
    case W_LRLRn: return w_LRLRn(x, y, phi, t, u, v);
    case W_LRLRp: return w_LRLRp(x, y, phi, t, u, v);
    case W_LRSL: return w_LRSL(x, y, phi, t, u, v);
    case W_LRSR: return w_LRSR(x, y, phi, t, u, v);
    default: return w_LRSLR(x, y, phi, t, u, v);
  }
}

HTP_HD inline int lengths_of(int lmode, double t, double u, double v, double* l) {
  const double h = 0.5 * PI;
  switch (lmode) {
    case 0: l[0] = t; l[1] = u; l[2] = v; return 3;
    case 1: l[0] = -t; l[1] = -u; l[2] = -v; return 3;
    case 2: l[0] = v; l[1] = u; l[2] = t; return 3;
    case 3: l[0] = -v; l[1] = -u; l[2] = -t; return 3;
    case 4: l[0] = t; l[1] = u; l[2] = -u; l[3] = v; return 4;
    case 5: l[0] = -t; l[1] = -u; l[2] = u; l[3] = -v; return 4;
    case 6: l[0] = t; l[1] = u; l[2] = u; l[3] = v; return 4;
    case 7: l[0] = -t; l[1] = -u; l[2] = -u; l[3] = -v; return 4;
    case 8: l[0] = t; l[1] = -h; l[2] = u; l[3] = v; return 4;
    case 9: l[0] = -t; l[1] = h; l[2] = -u; l[3] = -v; return 4;
    case 10: l[0] = v; l[1] = u; l[2] = -h; l[3] = t; return 4;
    case 11: l[0] = -v; l[1] = -u; l[2] = h; l[3] = -t; return 4;
    case 12: l[0] = t; l[1] = -h; l[2] = u; l[3] = -h; l[4] = v; return 5;
    default: l[0] = -t; l[1] = h; l[2] = -u; l[3] = h; l[4] = -v; return 5;
  }
}

// generate_path (:565-582): all admissible de-duplicated words, normalised lengths
HTP_HD inline void generate_paths(double sx, double sy, double syaw, double gx, double gy, double gyaw,
                                  double maxc, PathSet& S) {
  S.n = 0;
  S.err = 0;
  const double dx = gx - sx, dy = gy - sy, dth = gyaw - syaw;
  const double c = hm::cos(syaw), s = hm::sin(syaw);
  const double x = (c * dx + s * dy) * maxc;
  const double y = (-s * dx + c * dy) * maxc;
  const double xb = x * hm::cos(dth) + y * hm::sin(dth);
  const double yb = x * hm::sin(dth) - y * hm::cos(dth);
  const Cand* T = cand_table();
  for (int k = 0; k < 46; ++k) {
    const Cand& cd = T[k];
    const bool back = cd.arg >= 4;
    const double bx = back ? xb : x, by = back ? yb : y;
    const int am = cd.arg & 3;
    const double ax = (am == 1 || am == 3) ? -bx : bx;
    const double ay = (am == 2 || am == 3) ? -by : by;
    const double ap = (am == 1 || am == 2) ? -dth : dth;
    double t = 0, u = 0, v = 0;
    if (!eval_word(cd.word, ax, ay, ap, t, u, v)) continue;
    double l[5];
    const int n = lengths_of(cd.lmode, t, u, v, l);
    add_path(S, n, l, cd.ty);
  }
}

// interpolate (:533-562) for one point
// FAST: the sin / cos of htp_fastm.h (explicit FMA, <= 2 ulp, the same doubles on the device and every host build)
// for callers whose samples only feed a collision boolean (the hybrid A* goal shot's per-sample footprint test,
// hastar_core.h rs_path_hits); every sample the library returns is produced with FAST = false.
template <bool FAST = false>
HTP_HD inline void interp(double l, int m, double maxc, double ox, double oy, double oyaw, double& px, double& py,
                          double& pyaw, double& cs, int& dir) {
  if (m == SEG_S) {
    double so, co;
    if constexpr (FAST) fm::sincos(oyaw, so, co);
    else { co = hm::cos(oyaw); so = hm::sin(oyaw); }
    px = ox + l / maxc * co;
    py = oy + l / maxc * so;
    pyaw = oyaw;
    cs = 0.0;
  } else {
    double sl, cl, sm, cm;   // sin / cos of l and of -oyaw
    if constexpr (FAST) { fm::sincos(l, sl, cl); fm::sincos(-oyaw, sm, cm); }
    else { sl = hm::sin(l); cl = hm::cos(l); sm = hm::sin(-oyaw); cm = hm::cos(-oyaw); }
    const double ldx = sl / maxc;
    double ldy;
    if (m == SEG_L) { ldy = (1.0 - cl) / maxc; cs = maxc; }
    else { ldy = (1.0 - cl) / (-maxc); cs = -maxc; }
    const double gdx = cm * ldx + sm * ldy;
    const double gdy = -sm * ldx + cm * ldy;
    px = ox + gdx;
    py = oy + gdy;
  }
  if (m == SEG_L) pyaw = oyaw + l;
  else if (m == SEG_R) pyaw = oyaw - l;
  dir = (l > 0.0) ? 1 : -1;
}

// generate_local_course (:471-530) as a stream of point writes.  The reference
// fills zero-initialised lists of point_num entries, rewinds one index at every
// segment start (the first sample of a segment overwrites the last sample of the
// previous one) and finally pops trailing entries whose local x is exactly 0.0.
// Writes only ever go to the current index or the next one, so the final list
// length is recoverable from (current index, its x, last earlier non-zero index)
// without storing the list.  Sink::put(k, local x, y, yaw, cs, dir) sees every
// write in order (later writes to k supersede earlier ones); the return value is
// the reference's list length, -1 where the reference would raise IndexError.
HTP_HD inline int point_num(const Path& p, double step) { return (int)(p.L / step) + p.nseg + 3; }

struct NullSink {
  HTP_HD void put(int, double, double, double, double, int) const {}
};

template <class Sink>
HTP_HD inline int local_course(const Path& p, double maxc, double step, Sink& sink) {
  const int np = point_num(p, step);
  const int dir0 = (p.len[0] > 0.0) ? 1 : -1;
  sink.put(0, 0.0, 0.0, 0.0, 0.0, dir0);
  int cur = 0, nz_prev = -1;
  double cx = 0.0, cy = 0.0, cyaw = 0.0;  // local values at index cur
  bool bad = false;
  auto write = [&](int k, double x, double y, double yaw, double cs, int dir) {
    if (k == cur + 1) {
      if (cx != 0.0) nz_prev = cur;
      cur = k;
    } else if (k != cur) {
      bad = true;
    }
    if (k >= np) bad = true;
    cx = x; cy = y; cyaw = yaw;
    sink.put(k, x, y, yaw, cs, dir);
  };
  int ind = 1;
  double d = (p.len[0] > 0.0) ? step : -step;
  double pd = d, ll = 0.0;
  for (int i = 0; i < p.nseg; ++i) {
    const double l = p.len[i];
    const int m = p.typ[i];
    d = (l > 0.0) ? step : -step;
    // origin = list entry at ind: the last written sample (zeros before the first write)
    const double ox = cx, oy = cy, oyaw = cyaw;
    ind -= 1;
    if (i >= 1 && (p.len[i - 1] * p.len[i]) > 0) pd = -d - ll;
    else pd = d - ll;
    double x, y, yaw, cs;
    int dir;
    while (fabs(pd) <= fabs(l)) {
      ind += 1;
      interp(pd, m, maxc, ox, oy, oyaw, x, y, yaw, cs, dir);
      write(ind, x, y, yaw, cs, dir);
      pd += d;
    }
    ll = l - pd - d;
    ind += 1;
    interp(l, m, maxc, ox, oy, oyaw, x, y, yaw, cs, dir);
    write(ind, x, y, yaw, cs, dir);
  }
  const int n = (cx != 0.0) ? cur + 1 : nz_prev + 1;
  if (bad || n == 0) return -1;
  return n;
}

// Writes the final (global-frame) samples of one path, indices < limit only.
struct GlobalSink {
  double *x, *y, *yaw, *cs;
  int8_t* dir;
  int limit;
  double sx, sy, syaw, cq, sq;  // cq = cos(-syaw), sq = sin(-syaw)
  HTP_HD void put(int k, double lx, double ly, double lyaw, double c, int d) const {
    if (k >= limit) return;
    x[k] = cq * lx + sq * ly + sx;
    y[k] = -sq * lx + cq * ly + sy;
    yaw[k] = pi2pi(lyaw + syaw);
    cs[k] = c;
    dir[k] = (int8_t)d;
  }
};

}  // namespace rs
}  // namespace htp
