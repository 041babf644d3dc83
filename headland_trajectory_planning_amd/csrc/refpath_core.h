// Warm start -> OBCA initial guess on the device:
// R/obca_py/util.py get_init_ref_path :62-113 with
// R/path_planner/utils/cubic_spline.py calc_spline_course :92-112, one path
// per 64-lane wavefront.
//
//   * split the path where the gear (dirs) changes (:74-83);
//   * per segment: drop consecutive duplicate points (:94-99), arc length by
//     the sequential cumsum of hypot, scipy's not-a-knot slopes for x(s) and
//     y(s) (dubins_core.h, one lane per axis), samples s = k ds for
//     k < len(np.arange(0, s_end + ds, ds)) evaluated lane-parallel (PPoly
//     term order, extrapolating past s_end like scipy); yaw = atan2(y', x')
//     (+pi wrapped in reverse), steer = atan(L kappa) * gear sign, v = gear *
//     desired_v, v[0] = steer[0] = 0 per segment (:85-104);
//   * process_angle over the stacked headings (sequential unwrap, :16-43) and
//     v = 0 at both ends (:108-111).
#pragma once
#include <cmath>
#include "htp_libm.h"
#include <cstdint>

#include "dubins_core.h"
#include "rs_core.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace htp {
namespace rp {

enum { ST_OK = 0, ST_OVERFLOW = 1, ST_BAD_SEGMENT = 2, ST_BAD_INPUT = 3 };
constexpr double PI = 3.141592653589793;

HTP_HD inline double wrap_angle(double a) { return rs::pymod(a + PI, 2.0 * PI) - PI; }  // util.py:7-13

struct Out {
  int32_t status, n_rows, n_seg, pad;
};

// Per-path scratch (HBM): X, Y, S, DX, DY (cap each) + 2 x 4 cap tridiagonal work.
constexpr int SCRATCH_PER_POINT = 13;

template <class C>
struct Course {
  C& c;
  const double *px, *py, *pdir;  // path points of this search
  int np;
  double wb, desired_v, ds;
  double* scr;
  int cap;  // points capacity of the scratch

  // one gear segment [a, b] -> rows [row0, row0 + ns); returns ns (or -1)
  HTP_HD int segment(int a, int b, double* out, int row0, int cap_out, int& status) {
    double* X = scr;
    double* Y = X + cap;
    double* S = Y + cap;
    double* DX = S + cap;
    double* DY = DX + cap;
    double* WK = DY + cap;
    int m = 0;
    for (int i = a; i <= b; ++i) {  // uniform: every lane writes the same compacted values
      const bool dup = i < b && px[i + 1] == px[i] && py[i + 1] == py[i];
      if (!dup) {
        const double xi = px[i], yi = py[i];
        X[m] = xi;
        Y[m] = yi;
        ++m;
      }
    }
    c.sync();
    if (m < 2) {  // scipy CubicSpline needs two distinct points
      status = ST_BAD_SEGMENT;
      return -1;
    }
    S[0] = 0.0;
    for (int i = 1; i < m; ++i) S[i] = S[i - 1] + hm::hypot(X[i] - X[i - 1], Y[i] - Y[i - 1]);
    c.sync();
    if (c.lane == 0 || C::width == 1) dub::spline_slopes(S, X, m, DX, WK);
    if (c.lane == (C::width > 1 ? 1 : 0)) dub::spline_slopes(S, Y, m, DY, WK + 4 * cap);
    c.sync();
    const double nsd = ceil((S[m - 1] + ds) / ds);
    if (!(nsd >= 1.0) || nsd > 1e9) {
      status = ST_BAD_SEGMENT;
      return -1;
    }
    const int ns = (int)nsd;
    if (row0 + ns > cap_out) {
      status = ST_OVERFLOW;
      return ns;
    }
    const double gear = pdir[a];       // path[0, -1]
    const bool rev = pdir[b] < 0;      // path[-1, -1] < 0
    for (int k = c.lane; k < ns; k += C::width) {
      const double v = (double)k * ds;
      const int iv = dub::interval(S, m, v);
      double x, x1, x2, y, y1, y2;
      dub::eval3(S, X, DX, iv, v, x, x1, x2);
      dub::eval3(S, Y, DY, iv, v, y, y1, y2);
      double yaw = hm::atan2(y1, x1);
      const double kap = (y2 * x1 - x2 * y1) / hm::pow(x1 * x1 + y1 * y1, 1.5);
      if (rev) yaw = wrap_angle(yaw + PI);
      double steer = hm::atan(wb * kap) * (rev ? -1.0 : 1.0);
      double vel = 1.0 * gear * desired_v;
      if (k == 0) {
        vel = 0.0;
        steer = 0.0;
      }
      double* r = out + 5 * (int64_t)(row0 + k);
      r[0] = x;
      r[1] = y;
      r[2] = vel;
      r[3] = yaw;
      r[4] = steer;
    }
    c.sync();
    return ns;
  }

  HTP_HD void run(Out& o, double* out, int cap_out) {
    o = Out{};
    if (np < 1) {
      o.status = ST_BAD_INPUT;
      return;
    }
    int row = 0, a = 0, status = ST_OK;
    for (int i = 0; i < np; ++i) {
      if (i + 1 < np && pdir[i + 1] == pdir[i]) continue;  // np.diff(dirs) != 0 ends a segment
      if (i + 1 - a > cap) {
        status = ST_BAD_INPUT;
        break;
      }
      const int ns = segment(a, i, out, row, cap_out, status);
      o.n_seg += 1;
      if (ns < 0) break;
      row += ns;  // on overflow: the rows needed up to this segment
      a = i + 1;
      if (status != ST_OK) break;
    }
    o.n_rows = row;
    o.status = status;
    if (status != ST_OK || row < 1) {
      if (status == ST_OK) o.status = ST_BAD_INPUT;
      return;
    }
    // process_angle (wrap each heading, then the sequential unwrap) and v = 0 at the ends
    if (c.lane == 0 || C::width == 1) {
      double prev_raw = wrap_angle(out[3]);
      double acc = prev_raw;
      out[3] = acc;
      for (int k = 1; k < row; ++k) {
        const double raw = wrap_angle(out[5 * (int64_t)k + 3]);
        acc = acc + wrap_angle(raw - prev_raw);
        prev_raw = raw;
        out[5 * (int64_t)k + 3] = acc;
      }
      out[2] = 0.0;
      out[5 * (int64_t)(row - 1) + 2] = 0.0;
    }
    c.sync();
  }
};

}  // namespace rp
}  // namespace htp
