// Classic headland turns on the device: the warm-start path of one turn per
// 64-lane wavefront, rows [x, y, yaw, k, dir] exactly as the reference's planners return them.
//
//   Dubins ....... get_dubins_path_full(start, end, R, step)      R/path_planner/safety_forward_path_plan.py:286-297
//                  (pydubins shortest_path(...).sample_many(step), then cubic_spline.calc_spline_course at
//                  ds = 0.1; the Dubins fallback of OBCA_warm_start.py:166-174)
//   circle-back .. get_circle_back_path_full(start, end, R, car, side, step)   :395-454 (radii grown by 5 % until
//                  the reverse arc ends short of the row, forward arc + reverse arc by car_model.py:236-269
//                  calculate_motion_path_new, Dubins lead to the row pose; rows 2R or more apart: Dubins)
//   fish-tail .... R/test/classic_planner.ipynb cells 10-11: get_start_end_pose_for_reeds_shepp (:300-364, the
//                  offset poses whose 45-degree turn-out arcs -- car_model.py:202-234 calculate_motion_path --
//                  clear the blockers, both moved to one outmost x), every Reeds-Shepp word
//                  (utils/reeds_shepp.py:39-65), the collision-free word with the least backward length, Dubins
//                  lead-in / lead-out when an offset exceeds 0.1
//
// Footprints: the body polygon at every pose against the blocker polygons (orchard_geometry_environment.py
// check_path_feasibility :423-458 with boundary_check=False), the separating-axis predicate of hastar_core.h.
// Lane-parallel: Dubins / arc sampling, spline evaluation, footprint checks of the offset arcs; one Reeds-Shepp
// word per lane for the word checks.  Sequential pieces (pydubins' accumulated sample times, the spline's
// tridiagonal solve, cumulative sums) run on one lane, as the reference runs them.
#pragma once
#include <cmath>
#include "htp_libm.h"
#include <cstdint>

#include "hastar_core.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace htp {
namespace ct {

enum { T_DUBINS = 0, T_CIRCLEBACK = 1, T_FISHTAIL = 2 };
enum { ST_OK = 0, ST_OVERFLOW = 1, ST_NO_WORD = 2, ST_BAD_INPUT = 3, ST_RS_ERROR = 4, ST_NO_DUBINS = 5 };
enum { NEAR_SIDE = 1, FAR_SIDE = 2, LEAVE_POSE = 1, ENTER_POSE = 2 };   // map_utils constants
constexpr double PI = 3.141592653589793;
constexpr int SCR_PER_POINT = 10;   // Dubins scratch: T X Y S DX DY + 4 tridiagonal work

HTP_HD inline double wrap(double a) { return rs::pymod(a + PI, 2.0 * PI) - PI; }   // angle_wrap
HTP_HD inline double sgnf(double v) { return v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0); }

struct Spec {
  int type, side;
  double start[3], end[3];
  double wb, max_steer, radius, step;   // car.WHEEL_BASE, car.MAX_STEER, turning radius argument, step_size
};

template <class C>
struct Turn {
  C& c;
  const Spec& sp;
  ha::Footprint fp;    // body + blockers (no field, no lanes)
  double* scr;         // SCR_PER_POINT * cap_scr doubles (HBM)
  int cap_scr;
  double* out;         // [cap_out][5]
  int cap_out;
  rs::Path* paths;     // MAXP slots (wave-shared)
  int* flags;          // MAXP ints (wave-shared)
  int n_out = 0, status = ST_OK;

  HTP_HD double curvature() const { return hm::tan(sp.max_steer) / sp.wb; }   // car_model.py:34

  HTP_HD void put_row(int r, double x, double y, double yaw, double k, double d) {
    double* o = out + 5 * (int64_t)r;
    o[0] = x; o[1] = y; o[2] = yaw; o[3] = k; o[4] = d;
  }

  // get_dubins_path_full(q0, q1, r, step) -> rows [row0, row0 + n); drop the first / last row if asked.
  HTP_HD int dubins_full(const double* q0, const double* q1, double r, double step, int row0, bool drop_first,
                         bool drop_last) {
    dub::Path P;
    if (!dub::shortest(q0, q1, r, P)) { status = ST_NO_DUBINS; return -1; }
    P.q0[0] = q0[0]; P.q0[1] = q0[1]; P.q0[2] = q0[2]; P.rho = r;
    double* T = scr;
    double* X = T + cap_scr;
    double* Y = X + cap_scr;
    double* S = Y + cap_scr;
    double* DX = S + cap_scr;
    double* DY = DX + cap_scr;
    double* WK = DY + cap_scr;
    const double L = dub::length(P);
    int n = 0;
    {   // sample_many: x accumulates step by step (pydubins / the restated dubins.py)
      double x = 0.0;
      while (x < L) {
        if (n >= cap_scr) { status = ST_OVERFLOW; return -1; }
        if (c.lane == 0) T[n] = x;
        ++n;
        x += step;
      }
    }
    c.sync();
    for (int k = c.lane; k < n; k += C::width) {
      double q[3];
      dub::sample(P, T[k], q);
      X[k] = q[0];
      Y[k] = q[1];
    }
    c.sync();
    // calc_spline_course(x, y, ds=0.1): consecutive duplicates removed, arc length by sequential cumsum
    int m = 0;
    if (c.lane == 0 || C::width == 1) {
      for (int i = 0; i < n; ++i) {
        const bool dup = i + 1 < n && X[i + 1] == X[i] && Y[i + 1] == Y[i];
        if (!dup) { T[m] = X[i]; WK[m] = Y[i]; ++m; }
      }
      for (int i = 0; i < m; ++i) { X[i] = T[i]; Y[i] = WK[i]; }
      S[0] = 0.0;
      for (int i = 1; i < m; ++i) S[i] = S[i - 1] + hm::hypot(X[i] - X[i - 1], Y[i] - Y[i - 1]);
    }
    m = c.uniform_i(m);
    c.sync();
    if (m < 2) { status = ST_NO_DUBINS; return -1; }
    if (c.lane == 0 || C::width == 1) dub::spline_slopes(S, X, m, DX, WK);
    c.sync();
    // WK (4 cap_scr doubles) is free again once the X solve has finished: the Y solve uses it too
    if (c.lane == (C::width > 1 ? 1 : 0)) dub::spline_slopes(S, Y, m, DY, WK);
    c.sync();
    const double ds = 0.1;
    const double nsd = ceil((S[m - 1] + ds) / ds);
    if (!(nsd >= 1.0) || nsd > 1e9) { status = ST_NO_DUBINS; return -1; }
    const int ns = (int)nsd;
    const int k0 = drop_first ? 1 : 0, k1 = drop_last ? ns - 1 : ns;
    if (row0 + (k1 - k0) > cap_out) { status = ST_OVERFLOW; return -1; }
    for (int k = k0 + c.lane; k < k1; k += C::width) {
      const double v = (double)k * ds;
      const int iv = dub::interval(S, m, v);
      double x, x1, x2, y, y1, y2;
      dub::eval3(S, X, DX, iv, v, x, x1, x2);
      dub::eval3(S, Y, DY, iv, v, y, y1, y2);
      const double kap = (y2 * x1 - x2 * y1) / hm::pow(x1 * x1 + y1 * y1, 1.5);
      put_row(row0 + k - k0, x, y, hm::atan2(y1, x1), kap, 1.0);
    }
    c.sync();
    return k1 - k0;
  }

  // calculate_motion_path_new(init_pose, motion_dir, steer_dir, turning_radius, delta_yaw, step) car_model.py:236-269
  HTP_HD int arc_new(const double* p0, double mdir, double sdir, double R, double dyaw, double step, int row0) {
    const double tr = fmax(1.0 / curvature(), R);
    const double steer = hm::atan(sp.wb / tr) * sdir;
    const double arc = fabs(dyaw * tr);
    const int num = (int)(arc / step);
    if (num < 1) { status = ST_BAD_INPUT; return -1; }
    const double act = arc / num;
    const double ystep = mdir * act / sp.wb * hm::tan(steer);
    const double iy = wrap(p0[2]);
    const double stop = iy + ystep * num;
    const double lstep = (stop - iy) / num;
    const double kap = fabs(steer) > 0.00001 ? hm::tan(steer) / sp.wb : 0.0;
    if (row0 + num + 2 > cap_out) { status = ST_OVERFLOW; return -1; }
    if (c.lane == 0) put_row(row0, p0[0], p0[1], p0[2], kap, mdir);
    for (int k = c.lane; k <= num; k += C::width) {
      const double yl = k == num ? stop : (double)k * lstep + iy;   // np.linspace
      const double yaw = wrap(yl);
      const double x = p0[0] + tr * (hm::sin(yaw) - hm::sin(iy)) * sdir;
      const double y = p0[1] - tr * (hm::cos(yaw) - hm::cos(iy)) * sdir;
      put_row(row0 + 1 + k, x, y, yaw, kap, mdir);
    }
    c.sync();
    return num + 2;
  }

  HTP_HD static double enter_steer_dir(const double* s, const double* e) {   // :37-45
    return e[1] - s[1] > 0 ? sgnf(1.0 * hm::cos(s[2])) : sgnf(-1.0 * hm::cos(s[2]));
  }

  // get_offset_pose (:248-283): first dist = 0, 0.1, ... 5 whose 45-degree arc clears the blockers
  HTP_HD void offset_pose(const double* init, int pose_type, double turn_dir, double* pose) {
    const double mdir = pose_type == ENTER_POSE ? -1.0 : 1.0, odir = pose_type == ENTER_POSE ? -1.0 : 1.0;
    const double st = 0.55 * turn_dir, step = 0.1, dyaw = 0.7853981633974483;   // math.radians(45)
    const double search_len = dyaw / curvature();
    const int num = (int)rint(search_len / step);
    const double ystep = mdir * step / sp.wb * hm::tan(st);
    double* PX = scr;
    double* PY = scr + cap_scr;
    double* PW = scr + 2 * cap_scr;
    if (num + 1 > cap_scr) { status = ST_OVERFLOW; return; }
    for (int kd = 0; kd < 51; ++kd) {   // np.arange(0, max_offset + accuracy, accuracy)
      const double dist = 0.0 + (double)kd * 0.1;
      const double x0 = init[0] + dist * hm::cos(init[2]) * odir, y0 = init[1] + dist * hm::sin(init[2]) * odir;
      pose[0] = x0; pose[1] = y0; pose[2] = init[2];
      if (c.lane == 0 || C::width == 1) {   // calculate_motion_path :202-234 (sequential cumsum)
        const double iy = wrap(init[2] + ystep);
        const double stop = iy + ystep * (num + 1);
        const double lstep = num > 0 ? (stop - iy) / num : 0.0;
        PX[0] = x0; PY[0] = y0; PW[0] = init[2];
        double cx = 0.0, cy = 0.0, prev = wrap(iy);   // np.cumsum of the steps, then added to the pose
        for (int k = 1; k <= num; ++k) {
          cx = cx + step * hm::cos(prev) * mdir;
          cy = cy + step * hm::sin(prev) * mdir;
          const double yk = wrap(k == num ? stop : (double)k * lstep + iy);
          PX[k] = x0 + cx; PY[k] = y0 + cy; PW[k] = yk;
          prev = yk;
        }
      }
      c.sync();
      int hit = 0;
      for (int k = c.lane; k <= num; k += C::width)
        if (fp.pose_hits(PX[k], PY[k], PW[k])) hit = 1;
      c.sync();
      if (c.isum(hit) == 0) return;
    }
  }

  // per-lane feasibility of one Reeds-Shepp word: the final samples (indices < n) through the footprint test
  struct CheckSink {
    const ha::Footprint* fp;
    double sx, sy, syaw, cq, sq;
    int n, cur = 0;
    double px = 0, py = 0, pyaw = 0;
    bool have = false, hit = false;
    HTP_HD void test(int k) {
      if (!have || k >= n || hit) return;
      const double gx = cq * px + sq * py + sx, gy = -sq * px + cq * py + sy;
      if (fp->pose_hits(gx, gy, rs::pi2pi(pyaw + syaw))) hit = true;
    }
    HTP_HD void put(int k, double lx, double ly, double lyaw, double, int) {
      if (k != cur) test(cur);   // index advanced: the previous entry is final
      cur = k; px = lx; py = ly; pyaw = lyaw; have = true;
    }
  };

  HTP_HD void fishtail() {
    const double* s0 = sp.start;
    const double* e0 = sp.end;
    const double td = enter_steer_dir(s0, e0);
    double so[3], eo[3];
    offset_pose(s0, LEAVE_POSE, td, so);
    if (status != ST_OK) return;
    offset_pose(e0, ENTER_POSE, td, eo);
    if (status != ST_OK) return;
    const double ox = sp.side == NEAR_SIDE ? fmin(s0[0], eo[0]) : fmax(s0[0], eo[0]);
    so[0] = ox;
    eo[0] = ox;
    const double leave = fabs(ox - s0[0]), enter = fabs(ox - e0[0]);
    const double maxc = curvature(), step = 0.1;
    rs::PathSet S{paths, 0, 0};
    if (c.lane == 0 || C::width == 1) rs::generate_paths(so[0], so[1], so[2], eo[0], eo[1], eo[2], maxc, S);
    c.sync();
    const int np_ = c.uniform_i(S.n), err = c.uniform_i(S.err);
    if (err) { status = ST_RS_ERROR; return; }
    // one word per lane: final list length (NullSink), then the footprint of every final sample
    for (int p = c.lane; p < np_; p += C::width) {
      rs::NullSink ns;
      const int n = rs::local_course(paths[p], maxc, step * maxc, ns);
      int f = 0;
      if (n < 0) {
        f = -1;
      } else {
        CheckSink ck{&fp, so[0], so[1], so[2], hm::cos(-so[2]), hm::sin(-so[2]), n};
        rs::local_course(paths[p], maxc, step * maxc, ck);
        ck.test(ck.cur);
        f = ck.hit ? 0 : 1;
      }
      flags[p] = f;
    }
    c.sync();
    int best = -1;
    double bcost = 99999.0;
    for (int p = 0; p < np_; ++p) {   // uniform: the reference's first minimum (cost < best)
      if (flags[p] < 0) { status = ST_RS_ERROR; return; }
      if (flags[p] == 0) continue;
      double acc = 0.0;
      for (int j = 0; j < paths[p].nseg; ++j) {
        const double l = paths[p].len[j] / maxc;
        if (l < 0) acc += l;
      }
      const double cost = fabs(acc);
      if (cost < bcost) { best = p; bcost = cost; }
    }
    if (best < 0) { status = ST_NO_WORD; return; }
    const double r = 1.0 / maxc;
    int row = 0;
    if (leave > 0.1) {
      const int n = dubins_full(s0, so, r, 0.1, row, false, true);
      if (n < 0) return;
      row += n;
    }
    {
      rs::NullSink ns;
      const int n = rs::local_course(paths[best], maxc, step * maxc, ns);
      if (row + n > cap_out) { status = ST_OVERFLOW; return; }
      if (c.lane == 0 || C::width == 1) {
        double* o = out + 5 * (int64_t)row;
        // GlobalSink writes strided columns; rows are [x, y, yaw, cs, dir] with stride 5
        struct RowSink {
          double* o;
          int limit;
          double sx, sy, syaw, cq, sq;
          HTP_HD void put(int k, double lx, double ly, double lyaw, double cv, int d) const {
            if (k >= limit) return;
            double* r = o + 5 * (int64_t)k;
            r[0] = cq * lx + sq * ly + sx;
            r[1] = -sq * lx + cq * ly + sy;
            r[2] = rs::pi2pi(lyaw + syaw);
            r[3] = cv;
            r[4] = (double)d;
          }
        } rsk{o, n, so[0], so[1], so[2], hm::cos(-so[2]), hm::sin(-so[2])};
        rs::local_course(paths[best], maxc, step * maxc, rsk);
      }
      c.sync();
      row += n;
    }
    if (enter > 0.1) {
      const int n = dubins_full(eo, e0, r, 0.1, row, true, false);
      if (n < 0) return;
      row += n;
    }
    n_out = row;
  }

  HTP_HD void circleback() {
    const double* s0 = sp.start;
    const double* e0 = sp.end;
    const double w = fabs(s0[1] - e0[1]);
    const double tr = fmax(sp.radius, 1.0 / curvature());
    if (w >= tr * 2) {
      const int n = dubins_full(s0, e0, tr, sp.step, 0, false, false);
      if (n >= 0) n_out = n;
      return;
    }
    double Rf = tr, Rb = tr, theta = 0.0;
    for (int it = 0; it < 100000; ++it) {
      theta = PI / 2 + hm::asin((Rb + w - Rf) / (Rf + Rb));
      if (sp.side == NEAR_SIDE && s0[0] - (Rf + Rb) * hm::cos(theta - PI / 2) < e0[0] - sp.step) break;
      if (sp.side == FAR_SIDE && s0[0] + (Rf + Rb) * hm::cos(theta - PI / 2) > e0[0] + sp.step) break;
      Rf *= 1.05;
      Rb *= 1.05;
    }
    const double td = enter_steer_dir(s0, e0);
    int row = 0;
    const int n1 = arc_new(s0, 1.0, td, Rf, theta, sp.step, row);
    if (n1 < 0) return;
    row += n1;
    double f_end[3] = {out[5 * (int64_t)(row - 1)], out[5 * (int64_t)(row - 1) + 1], out[5 * (int64_t)(row - 1) + 2]};
    const int n2 = arc_new(f_end, -1.0, -td, Rb, PI - theta, sp.step, row);
    if (n2 < 0) return;
    row += n2;
    double b_end[3] = {out[5 * (int64_t)(row - 1)], out[5 * (int64_t)(row - 1) + 1], out[5 * (int64_t)(row - 1) + 2]};
    const int n3 = dubins_full(b_end, e0, tr, sp.step, row, false, false);
    if (n3 < 0) return;
    n_out = row + n3;
  }

  HTP_HD void run() {
    status = ST_OK;
    n_out = 0;
    if (!(sp.wb > 0.0) || !(sp.step > 0.0) || !(sp.radius > 0.0)) { status = ST_BAD_INPUT; return; }
    if (sp.type == T_DUBINS) {
      const int n = dubins_full(sp.start, sp.end, sp.radius, sp.step, 0, false, false);
      if (n >= 0) n_out = n;
    } else if (sp.type == T_CIRCLEBACK) {
      circleback();
    } else if (sp.type == T_FISHTAIL) {
      fishtail();
    } else {
      status = ST_BAD_INPUT;
    }
  }
};

}  // namespace ct
}  // namespace htp
