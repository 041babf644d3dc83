// Y-type parking grid search (R/path_planner/headland_path_planning.py
// search_y_type_parking_path :382-451), one search per 64-lane wavefront.
//
// The reference walks the 4-D parameter grid (backward length desc, forward
// length desc, backward steer asc, forward steer asc) and returns the first
// candidate whose manoeuvre is collision free.  Here each lane builds one
// candidate of a 64-candidate chunk (get_y_type_parking_path :487-516: two
// calculate_motion_path arcs :455-484 with numpy linspace / angle_wrap /
// cumsum rounding, reversed and stacked, then get_path_in_odom :519-527), all
// lanes test the (candidate, pose) footprints (hastar_core.h Footprint:
// blockers + field polygon, env.check_path_feasibility :423-458 with
// boundary_check=True), and the smallest feasible index of the chunk is the
// reference's answer; later chunks are never built.
#pragma once
#include <cmath>
#include "htp_libm.h"
#include <cstdint>

#include "hastar_core.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace htp {
namespace yp {

constexpr int MAXARC = 64;            // poses per arc (round(L/step) + 1)
constexpr int MAXPOSE = 2 * MAXARC;   // poses per candidate path
constexpr int CH = 64;                // candidates per chunk (one per lane)

// per-search double parameters (htp.h HTP_YP_P_*)
enum { P_EX, P_EY, P_EYAW, P_BDIR, P_FDIR, P_WB, P_STEP, P_R00, P_R01, P_R10, P_R11, P_TX, P_TY, P_YAW_ODOM,
       P_NP = 16 };
// per-search int descriptor (htp.h HTP_YP_D_*): polygons + grid axes in the value pool
enum { D_BODY, D_BLK0, D_BLK1, D_FIELD, D_BL0, D_NBL, D_FL0, D_NFL, D_SB0, D_NSB, D_SF0, D_NSF, D_NDESC = 12 };
enum { ST_FOUND = 0, ST_NONE = 1, ST_END_BLOCKED = 2, ST_BAD_INPUT = 3 };

// calculate_motion_path :455-484 into P[(n+1)][5] (x, y, yaw, k, dir); returns n+1
HTP_HD inline int motion_path(double x0, double y0, double yaw0, double steer, double dir, double length,
                              double wb, double step, double* P) {
  const int n = (int)rint(length / step);
  const double yaw_step = dir * step / wb * hm::tan(steer);
  const double init_yaw = ha::angle_wrap(yaw0 + yaw_step);
  const double stop = init_yaw + yaw_step * (double)n;
  const double div = (double)n;
  const double delta = stop - init_yaw;
  const double stp = delta / div;
  const double curv = fabs(steer) > 0.00001 ? hm::tan(steer) / wb : 0.0;
  P[0] = x0; P[1] = y0; P[2] = yaw0; P[3] = curv; P[4] = dir;
  double ax = 0.0, ay = 0.0;
  for (int i = 0; i < n; ++i) {  // xs from yaws[:-1], path yaw = yaws[1:]
    const double yi = (stp == 0) ? ((double)i / div) * delta + init_yaw : (double)i * stp + init_yaw;
    const double wy = ha::angle_wrap(yi);
    const double dx = step * hm::cos(wy) * dir;
    const double dy = step * hm::sin(wy) * dir;
    ax = (i == 0) ? dx : ax + dx;
    ay = (i == 0) ? dy : ay + dy;
    const double ni = (i + 1 == n) ? stop
                                   : ((stp == 0) ? ((double)(i + 1) / div) * delta + init_yaw
                                                 : (double)(i + 1) * stp + init_yaw);
    double* q = P + 5 * (i + 1);
    q[0] = x0 + ax; q[1] = y0 + ay; q[2] = ha::angle_wrap(ni); q[3] = curv; q[4] = dir;
  }
  return n + 1;
}

// One candidate's path in the odom frame into Q[MAXPOSE][5]; returns its pose count.
HTP_HD inline int candidate_path(const double* prm, double bl, double fl, double sb, double sf, double* Q,
                                 double* back) {
  const double wb = prm[P_WB], step = prm[P_STEP];
  // back arc from the origin, then the forward arc from its last pose (:495-509)
  const int nb = motion_path(0.0, 0.0, 0.0, sb * prm[P_BDIR], -1.0, bl, wb, step, back);
  const double* e = back + 5 * (nb - 1);
  const int nf = motion_path(e[0], e[1], e[2], sf * prm[P_FDIR], 1.0, fl, wb, step, Q + 5 * MAXPOSE);
  // [forward reversed (dir -1), backward reversed (dir +1)] (:510-514)
  int k = 0;
  const double* F = Q + 5 * MAXPOSE;
  for (int i = nf - 1; i >= 0; --i, ++k)
    for (int c = 0; c < 5; ++c) Q[5 * k + c] = (c == 4) ? -1.0 : F[5 * i + c];
  for (int i = nb - 1; i >= 0; --i, ++k)
    for (int c = 0; c < 5; ++c) Q[5 * k + c] = (c == 4) ? 1.0 : back[5 * i + c];
  // get_path_in_odom: yaw += SE32states(T) yaw, (x, y) <- T (x, y, 0, 1)
  for (int i = 0; i < k; ++i) {
    double* q = Q + 5 * i;
    const double x = q[0], y = q[1];
    q[2] = q[2] + prm[P_YAW_ODOM];
    q[0] = prm[P_R00] * x + prm[P_R01] * y + prm[P_TX];
    q[1] = prm[P_R10] * x + prm[P_R11] * y + prm[P_TY];
  }
  return k;
}

struct Out {
  int32_t status, cand, n_path;
  double bl, fl, sb, sf;
  int64_t n_pose;
};

constexpr int SCR = (MAXPOSE + 2 * MAXARC) * 5;  // scratch doubles per candidate slot

template <class C>
struct Search {
  C& c;
  const double* prm;
  const int32_t* dsc;
  ha::Geo g;
  const double* axis;   // value pool of the grid axes
  double* scratch;      // [CH][SCR] per search (HBM)
  double* body;         // LDS [MAXB][2]
  int32_t* cnt;         // LDS [CH] pose count per candidate
  int32_t* hit;         // LDS [CH] collision flag per candidate
  ha::Footprint fp;

  HTP_HD Search(C& c_, const double* p, const int32_t* d, const ha::Geo& g_, const double* ax, double* scr,
                double* body_lds, int32_t* cnt_lds, int32_t* hit_lds)
      : c(c_), prm(p), dsc(d), g(g_), axis(ax), scratch(scr), body(body_lds), cnt(cnt_lds), hit(hit_lds) {
    const int b0 = g.poly_off[dsc[D_BODY]];
    const int nb = g.poly_off[dsc[D_BODY] + 1] - b0;
    for (int q = c.lane; q < 2 * nb; q += C::width) body[q] = g.vert[2 * b0 + q];
    c.sync();
    fp = ha::Footprint{g, body, nb, dsc[D_BLK0], dsc[D_BLK1], dsc[D_FIELD], 0, 0};
  }

  // candidate k in the reference's loop order (:411-414): bl outermost, sf innermost
  HTP_HD void params_of(int k, double& bl, double& fl, double& sb, double& sf) const {
    const int nsf = dsc[D_NSF], nsb = dsc[D_NSB], nfl = dsc[D_NFL];
    const int isf = k % nsf;
    k /= nsf;
    const int isb = k % nsb;
    k /= nsb;
    const int ifl = k % nfl;
    const int ibl = k / nfl;
    bl = axis[dsc[D_BL0] + ibl];
    fl = axis[dsc[D_FL0] + ifl];
    sb = axis[dsc[D_SB0] + isb];
    sf = axis[dsc[D_SF0] + isf];
  }

  // -> o (status, chosen candidate, parameters); the chosen path into out[cap][5]
  HTP_HD void run(Out& o, double* out, int cap) {
    o = Out{};
    o.cand = -1;
    o.status = ST_NONE;
    int h = 0;  // the end pose itself must be feasible (:400-402)
    if (c.lane == 0 || C::width == 1) h = fp.pose_hits(prm[P_EX], prm[P_EY], prm[P_EYAW]) ? 1 : 0;
    o.n_pose += 1;
    if (c.isum(h) > 0) { o.status = ST_END_BLOCKED; return; }
    const int total = dsc[D_NBL] * dsc[D_NFL] * dsc[D_NSB] * dsc[D_NSF];
    for (int base = 0; base < total; base += CH) {
      const int nc = (total - base) < CH ? (total - base) : CH;
      for (int l = c.lane; l < nc; l += C::width) {  // lane l builds candidate base + l
        double bl, fl, sb, sf;
        params_of(base + l, bl, fl, sb, sf);
        double* Q = scratch + (int64_t)l * SCR;
        cnt[l] = candidate_path(prm, bl, fl, sb, sf, Q, Q + 5 * (MAXPOSE + MAXARC));
        hit[l] = 0;
      }
      c.sync();
      int maxp = 0, sum = 0;
      for (int l = 0; l < nc; ++l) {
        maxp = cnt[l] > maxp ? cnt[l] : maxp;
        sum += cnt[l];
      }
      for (int q = c.lane; q < nc * maxp; q += C::width) {  // (candidate, pose) pairs
        const int l = q / maxp, i = q - l * maxp;
        if (i >= cnt[l]) continue;
        const double* P = scratch + (int64_t)l * SCR + 5 * i;
        if (fp.pose_hits(P[0], P[1], P[2])) hit[l] = 1;
      }
      c.sync();
      o.n_pose += sum;
      int first = -1;
      for (int l = 0; l < nc && first < 0; ++l)
        if (!hit[l]) first = l;
      c.sync();
      if (first >= 0) {
        o.status = ST_FOUND;
        o.cand = base + first;
        params_of(o.cand, o.bl, o.fl, o.sb, o.sf);
        o.n_path = cnt[first];
        const double* Q = scratch + (int64_t)first * SCR;
        for (int e = c.lane; e < 5 * o.n_path; e += C::width)
          if (e / 5 < cap) out[e] = Q[e];
        c.sync();
        return;
      }
    }
  }
};

}  // namespace yp
}  // namespace htp
