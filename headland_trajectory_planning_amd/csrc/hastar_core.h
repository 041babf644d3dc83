// Hybrid A* warm-start search, one search per 64-lane wavefront.
//
// Behaviour of R/path_planner/hybrid_a_star_search.py (HybridAStarSearch with
// motion_type="King": Reeds-Shepp goal shots) over lowered geometry:
//   * open/closed dicts keyed by the grid index (calculate_node_index :82-89,
//     Python round = half-to-even = rint) -> one open-addressing table whose
//     slots carry the state (open / closed), the node and the heap position;
//   * heapdict 1.0.1 priority queue (:504-596, value max(g, 50 h)) restated
//     exactly (delete = unconditional bubble to the root + popitem; sift-up
//     while parent >= child; sift-down with strict <), so ties pop in the
//     reference's order;
//   * goal extension (:232-287): all Reeds-Shepp words current -> goal
//     (rs_core.h; the 46 candidate words are evaluated one per lane, then
//     de-duplicated in reference order), costed by
//     calculate_reeds_shepp_path_cost (:129-160, quirks kept), ordered by a
//     second heapdict, each sampled path streamed through the collision test
//     64 samples at a time with early exit;
//   * motion expansion (:357-410): one lane per motion primitive integrates
//     the numpy linspace / angle_wrap / cumsum trajectory sequentially (same
//     rounding as numpy), then all lanes test the (motion, pose) pairs;
//   * collision (:412-427): body polygon at every pose vs blocker polygons
//     (separating axes), inside the field polygon, inside the union of the
//     heuristic's lane polygons (edge coverage by clip intervals);
//   * heuristic (reference_line_heuristic.py:120-158): search length from the
//     last lane polygon that strictly contains the pose, wave argmin over the
//     guide samples (first index on ties, like np.argmin).
// Arithmetic follows the reference's expression order; no FMA contraction.
#pragma once
#include <cmath>
#include "htp_libm.h"
#include "htp_fastm.h"
#include <cstdint>
#ifdef HTP_HA_DEBUG
#include <cstdio>
#endif

#include "dubins_core.h"
#include "rs_core.h"
#include "../../include/htp.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace htp {
namespace ha {

// in_lanes: keep each lane polygon's clip interval in a per-lane array and sweep it (1: round 5; the array is
// run-time indexed, so it lives in scratch memory) or re-clip the polygons on every sweep pass (0: no private array)
#ifndef HTP_HA_LANE_ARRAYS
#define HTP_HA_LANE_ARRAYS 0
#endif

constexpr int MAXB = 8;       // body polygon vertices
constexpr int MAXMOT = 16;    // motion primitives (King: 14, Pawn: 8)
constexpr int MAXTRAJ = 64;   // poses per motion primitive (round(L/res) + 1)
// Poses of one expansion's rollouts held in LDS (every primitive of a search length shares n + 1 poses, stored
// primitive-major at stride n + 1): nmot (n + 1) <= TRAJCAP.  The reference's settings need 14 x 16 = 224 (King,
// search length 1.5 m at 0.1 m); 512 keeps a search's LDS at ~21 KB, 7 resident searches per CU instead of 4.
constexpr int TRAJCAP = 512;
constexpr int MAXJ = 32;      // lane polygons
static_assert(MAXB == HTP_HA_MAX_BODY && MAXMOT == HTP_HA_MAX_MOTIONS && MAXTRAJ == HTP_HA_MAX_POSES &&
              TRAJCAP == HTP_HA_TRAJ_CAP && MAXJ == HTP_HA_MAX_LANES, "include/htp.h documents these limits");
constexpr int MAXCHAIN = 1 << 20;
constexpr double PI = 3.141592653589793;

// per-search double parameters (htp.h HTP_HA_P_*)
enum {
  P_SX, P_SY, P_SYAW, P_GX, P_GY, P_GYAW, P_RES, P_YAWRES, P_WB, P_MAXSTEER, P_CURV, P_DEFLEN, P_MAXNODES,
  P_NP = 16
};
// per-search int descriptor (htp.h HTP_HA_D_*)
enum {
  D_BODY, D_BLK0, D_BLK1, D_LANE0, D_LANE1, D_FIELD, D_GUIDE0, D_GUIDE1, D_MOT0, D_MOT1, D_KING,
  D_NDESC = 12
};
// search status (htp.h HTP_HA_*)
enum { ST_FOUND = 0, ST_NO_PATH = 1, ST_MAX_NODES = 2, ST_START_GOAL_BLOCKED = 3, ST_RS_ERROR = 4,
       ST_CAPACITY = 5, ST_BAD_INPUT = 6, ST_BACKTRACK = 7 };  // ST_CAPACITY also: Dubins shot beyond cap_dub

struct Geo {
  const int32_t* poly_off;  // [npoly+1] vertex ranges
  const double* vert;       // [nvert][2]
  const double* lane_len;   // [npoly] search length of lane polygons
  const double* guide;      // [nguide][4] x, y, yaw, s
  const double* motion;     // [nmotion][2] steer, direction
};

// A batch's pools (htp.h htp_hastar_batch) as the search reads them.
struct Pools {
  const double* params;
  const int32_t* desc;
  Geo g;
  int32_t npoly, nvert, nguide, nmotion;
};

// The polygon table's ranges (the searches trust poly_off): checked once per batch on the host.
inline bool poly_table_ok(const int32_t* poly_off, int npoly, int nvert) {
  for (int p = 0; p < npoly; ++p)
    if (poly_off[p] < 0 || poly_off[p + 1] < poly_off[p] || poly_off[p + 1] > nvert) return false;
  return true;
}

// Per-search shape checks the search relies on (descriptor ranges, body vertex count <= MAXB, lane count <= MAXJ,
// motion count <= MAXMOT, positive resolutions, max_nodes <= the workspace's cap).  Every search length L (the
// default and each lane's) must give n = rint(L / res) with 1 <= n, n + 1 <= MAXTRAJ and nmot (n + 1) <= TRAJCAP:
// one expansion's rollouts live in LDS (King's 14 motions: n + 1 <= 36, i.e. L <= 35 res).  A search failing any
// check ends HTP_HA_BAD_INPUT on the device and on the host build alike.
HTP_HD inline bool valid_search(const Pools& P, const double* prm, const int32_t* d, int max_nodes_cap) {
  auto poly_ok = [&](int p) { return p >= 0 && p < P.npoly; };
  if (!poly_ok(d[D_BODY])) return false;
  const int nb = P.g.poly_off[d[D_BODY] + 1] - P.g.poly_off[d[D_BODY]];
  if (nb < 3 || nb > MAXB) return false;
  if (d[D_BLK0] < 0 || d[D_BLK1] < d[D_BLK0] || d[D_BLK1] > P.npoly) return false;
  if (d[D_LANE0] < 0 || d[D_LANE1] <= d[D_LANE0] || d[D_LANE1] > P.npoly || d[D_LANE1] - d[D_LANE0] > MAXJ) return false;
  if (d[D_FIELD] != -1 && !poly_ok(d[D_FIELD])) return false;
  if (d[D_GUIDE0] < 0 || d[D_GUIDE1] <= d[D_GUIDE0] || d[D_GUIDE1] > P.nguide) return false;
  if (d[D_MOT0] < 0 || d[D_MOT1] <= d[D_MOT0] || d[D_MOT1] > P.nmotion || d[D_MOT1] - d[D_MOT0] > MAXMOT) return false;
  if (d[D_KING] != 0 && d[D_KING] != 1) return false;
  const double res = prm[P_RES];
  if (!(res > 0) || !(prm[P_YAWRES] > 0) || !(prm[P_WB] > 0) || !(prm[P_CURV] > 0)) return false;
  const double mn = prm[P_MAXNODES];
  if (!(mn >= 0) || mn > (double)max_nodes_cap) return false;
  const int nmot = d[D_MOT1] - d[D_MOT0];
  auto len_ok = [&](double L) {
    const double n = rint(L / res);
    return n >= 1 && n + 1 <= MAXTRAJ && (double)nmot * (n + 1) <= (double)TRAJCAP;
  };
  if (!len_ok(prm[P_DEFLEN])) return false;
  for (int p = d[D_LANE0]; p < d[D_LANE1]; ++p)
    if (!len_ok(P.g.lane_len[p])) return false;
  for (int p = d[D_BLK0]; p < d[D_BLK1]; ++p)
    if (P.g.poly_off[p + 1] - P.g.poly_off[p] < 1) return false;
  for (int p = d[D_LANE0]; p < d[D_LANE1]; ++p)
    if (P.g.poly_off[p + 1] - P.g.poly_off[p] < 3) return false;
  return true;
}

struct Node {  // 64 B
  double x, y, yaw, cost, curv;
  int32_t kx, ky, kt;       // grid index
  int32_t pkx, pky, pkt;    // parent grid index
  int32_t parent;           // node id of the expanding node (-1: start)
  int16_t kind;             // 0 start, 1 motion, 2 Reeds-Shepp goal shot, 3 Dubins goal shot
  int16_t aux;              // motion index / RS path index
  int32_t dir;
};

struct Slot {  // 24 B
  int32_t kx, ky, kt;
  int32_t state;  // 0 empty, 1 open, 2 closed
  int32_t node;
  int32_t hpos;
};

struct Work {  // per-search HBM workspace
  Node* node;
  Slot* slot;
  double* hval;
  int32_t* hslot;
  int32_t cap_node, cap_slot;  // cap_slot: power of two
  double* dub;                 // Pawn goal shot scratch: DUBW * (cap_dub + 16) doubles
  int32_t cap_dub;             // Dubins samples per shot
};
constexpr int DUBW = 16;       // X Y S DX DY | work 4 + 4 | XS YS YAW
constexpr int CAP_DUB = 4096;  // Dubins samples per Pawn goal shot (409.6 m at res 0.1)

struct Out {
  int32_t status, counter, n_path, n_expanded;
  int64_t n_pose, n_checks;
};

// Wave-shared scratch (LDS on the device).
struct Shared {
  double body[MAXB * 2];
  double traj[TRAJCAP * 3];
  int32_t hit[MAXMOT];
  double ccost[MAXMOT];
  double ccurv[MAXMOT];
  int32_t ckey[MAXMOT * 3];
  // Reeds-Shepp
  rs::Path paths[rs::MAXP];
  double cand_len[rs::MAXP * 5];
  int32_t cand_n[rs::MAXP];
  double rval[rs::MAXP];
  int32_t rkey[rs::MAXP];
  int32_t rpos[rs::MAXP];
  double pd[64];
  int32_t pseg[64];
  double org[6 * 3];
  int32_t flag[2];
  double red_d[64];
  int32_t red_i[64];
};

HTP_HD inline double pymod(double x, double y) { return rs::pymod(x, y); }
HTP_HD inline double angle_wrap(double a) { return pymod(a + PI, 2.0 * PI) - PI; }  // path_utils.angle_wrap

// Footprint predicates at one pose (car_model.get_path_poly :39-73 body at the
// pose): blocker polygons (separating axes, closed sets: touching collides),
// field polygon containment (all corners inside by crossing number, no proper
// crossing of edges), containment in the union of the lane polygons (every
// body edge covered by the union of its clip intervals; skipped when the lane
// range is empty, as for orchard_geometry_environment.check_path_feasibility).
struct Footprint {
  Geo g;
  const double* body;  // [nb][2] car-frame vertices (LDS on the device)
  int nb, blk0, blk1, field, lane0, lane1;

  // Exact shortcut of the separating-axis test: a blocker whose bounding box is apart from the body's by more
  // than SAT_EPS (metres) in x or y is disjoint from it by at least that much, and for the convex rectangles and
  // quads the planners lower (tree rows, obstacle squares) some edge normal separates them by a comparable
  // amount, far above rounding -- the full test returns false for it too.
  static constexpr double SAT_EPS = 1e-6;
  template <int NBC>
  HTP_HD bool sat_hit(const double* bx, const double* by, int p) const {
    const int nb = NBC ? NBC : this->nb;
    const int o = g.poly_off[p], m = g.poly_off[p + 1] - o;
    const double* V = g.vert + 2 * o;
    {
      double ax0 = bx[0], ax1 = bx[0], ay0 = by[0], ay1 = by[0];
      for (int j = 1; j < nb; ++j) {
        ax0 = fmin(ax0, bx[j]); ax1 = fmax(ax1, bx[j]); ay0 = fmin(ay0, by[j]); ay1 = fmax(ay1, by[j]);
      }
      double qx0 = V[0], qx1 = V[0], qy0 = V[1], qy1 = V[1];
      for (int j = 1; j < m; ++j) {
        qx0 = fmin(qx0, V[2 * j]); qx1 = fmax(qx1, V[2 * j]); qy0 = fmin(qy0, V[2 * j + 1]); qy1 = fmax(qy1, V[2 * j + 1]);
      }
      if (qx0 > ax1 + SAT_EPS || ax0 > qx1 + SAT_EPS || qy0 > ay1 + SAT_EPS || ay0 > qy1 + SAT_EPS) return false;
    }
    for (int k = 0; k < nb; ++k) {  // body edges
      const int k1 = (k + 1) == nb ? 0 : k + 1;
      const double ex = bx[k1] - bx[k], ey = by[k1] - by[k];
      const double nx = ey, ny = -ex;
      double amin = 0, amax = 0, qmin = 0, qmax = 0;
      for (int j = 0; j < nb; ++j) {
        const double d = bx[j] * nx + by[j] * ny;
        if (j == 0 || d < amin) amin = d;
        if (j == 0 || d > amax) amax = d;
      }
      for (int j = 0; j < m; ++j) {
        const double d = V[2 * j] * nx + V[2 * j + 1] * ny;
        if (j == 0 || d < qmin) qmin = d;
        if (j == 0 || d > qmax) qmax = d;
      }
      if (amax < qmin || qmax < amin) return false;
    }
    for (int k = 0; k < m; ++k) {  // blocker edges
      const int k1 = (k + 1) == m ? 0 : k + 1;
      const double ex = V[2 * k1] - V[2 * k], ey = V[2 * k1 + 1] - V[2 * k + 1];
      const double nx = ey, ny = -ex;
      double amin = 0, amax = 0, qmin = 0, qmax = 0;
      for (int j = 0; j < nb; ++j) {
        const double d = bx[j] * nx + by[j] * ny;
        if (j == 0 || d < amin) amin = d;
        if (j == 0 || d > amax) amax = d;
      }
      for (int j = 0; j < m; ++j) {
        const double d = V[2 * j] * nx + V[2 * j + 1] * ny;
        if (j == 0 || d < qmin) qmin = d;
        if (j == 0 || d > qmax) qmax = d;
      }
      if (amax < qmin || qmax < amin) return false;
    }
    return true;
  }

  template <int NBC>
  HTP_HD bool in_field(const double* bx, const double* by, int p) const {
    const int nb = NBC ? NBC : this->nb;
    const int o = g.poly_off[p], m = g.poly_off[p + 1] - o;
    const double* V = g.vert + 2 * o;
    for (int k = 0; k < nb; ++k) {  // crossing number of each corner
      const double X = bx[k], Y = by[k];
      bool inside = false;
      for (int i = 0; i < m; ++i) {
        const int j = (i + 1) == m ? 0 : i + 1;
        const double xi = V[2 * i], yi = V[2 * i + 1], xj = V[2 * j], yj = V[2 * j + 1];
        if ((yi > Y) != (yj > Y)) {
          const double xc = (xj - xi) * (Y - yi) / (yj - yi) + xi;
          if (X < xc) inside = !inside;
        }
      }
      if (!inside) return false;
    }
    for (int k = 0; k < nb; ++k) {  // no proper crossing of body and field edges
      const int k1 = (k + 1) == nb ? 0 : k + 1;
      const double ax = bx[k], ay = by[k], bbx = bx[k1], bby = by[k1];
      for (int i = 0; i < m; ++i) {
        const int j = (i + 1) == m ? 0 : i + 1;
        const double cx = V[2 * i], cy = V[2 * i + 1], dx = V[2 * j], dy = V[2 * j + 1];
        const double o1 = (bbx - ax) * (cy - ay) - (bby - ay) * (cx - ax);
        const double o2 = (bbx - ax) * (dy - ay) - (bby - ay) * (dx - ax);
        const double o3 = (dx - cx) * (ay - cy) - (dy - cy) * (ax - cx);
        const double o4 = (dx - cx) * (bby - cy) - (dy - cy) * (bbx - cx);
        if (o1 * o2 < 0 && o3 * o4 < 0) return false;
      }
    }
    return true;
  }

  // Exact shortcut of in_lanes: the body lies inside ONE lane polygon (convex, CCW) with every corner at least
  // LANE_EPS (distance, metres) inside every edge line of it.  For such a polygon and each body edge A -> B the
  // clip of in_lanes computes c0 = cross(A) > 0 with the same expression, and c1 = cross(B) - cross(A) to within
  // a few ulp of |e| |B - A|, far below the margin: every t = -c0 / c1 is < 0 (c1 > 0) or > 1 (c1 < 0), so the
  // interval stays [0, 1] and the sweep reaches 1 -- in_lanes returns true with the same doubles.  Poses that
  // straddle two lane polygons, or come within LANE_EPS of an edge, take the full test.
  static constexpr double LANE_EPS = 1e-9;
  mutable int lane_hint = 0;   // the lane polygon that held the last body (any holding polygon gives the result)
  template <int NBC>
  HTP_HD bool in_one_lane(const double* bx, const double* by) const {
    const int nb = NBC ? NBC : this->nb;
    const int nl = lane1 - lane0;
    for (int r = 0; r < nl; ++r) {
      int p = lane0 + lane_hint + r;
      if (p >= lane1) p -= nl;
      const int o = g.poly_off[p], m = g.poly_off[p + 1] - o;
      const double* V = g.vert + 2 * o;
      bool in = true;
      for (int i = 0; i < m && in; ++i) {
        const int j = (i + 1) == m ? 0 : i + 1;
        const double vx = V[2 * i], vy = V[2 * i + 1];
        const double ex = V[2 * j] - vx, ey = V[2 * j + 1] - vy;
        const double tol = LANE_EPS * (fabs(ex) + fabs(ey));
        for (int k = 0; k < nb && in; ++k) in = ex * (by[k] - vy) - ey * (bx[k] - vx) > tol;
      }
      if (in) { lane_hint = p - lane0; return true; }
    }
    return false;
  }

  // every body edge covered by the union of the lane polygons (CCW, convex).  Per edge A -> B each lane polygon
  // clips the segment to a parameter interval [l, h] (the same expressions as before); the edge is covered iff the
  // chain of intervals reachable from 0 reaches 1.  The reach is the least fixpoint of reach = max(reach, h over
  // intervals with l <= reach), found by re-clipping the polygons each pass instead of keeping the intervals in a
  // per-lane array (a run-time-indexed array lives in scratch memory on the device): the same fixpoint, so the same
  // boolean as the sorted sweep of the reference's shapely union, and no private memory.
  template <int NBC>
  HTP_HD bool in_lanes(const double* bx, const double* by) const {
    const int nb = NBC ? NBC : this->nb;
    if (in_one_lane<NBC>(bx, by)) return true;
    const int j0 = lane0, j1 = lane1;
    for (int k = 0; k < nb; ++k) {
      const int k1 = (k + 1) == nb ? 0 : k + 1;
      const double Ax = bx[k], Ay = by[k], Bx = bx[k1], By = by[k1];
#if HTP_HA_LANE_ARRAYS
      double lo[MAXJ], hi[MAXJ];
      int n = 0;
      for (int p = j0; p < j1; ++p) {
        const int o = g.poly_off[p], m = g.poly_off[p + 1] - o;
        const double* V = g.vert + 2 * o;
        double l = 0.0, h = 1.0;
        bool dead = false;
        for (int i = 0; i < m; ++i) {
          const int j = (i + 1) == m ? 0 : i + 1;
          const double vx = V[2 * i], vy = V[2 * i + 1];
          const double ex = V[2 * j] - vx, ey = V[2 * j + 1] - vy;
          const double c0 = ex * (Ay - vy) - ey * (Ax - vx);
          const double c1 = ex * (By - Ay) - ey * (Bx - Ax);
          if (c1 > 0) { const double t = -c0 / c1; if (t > l) l = t; }
          else if (c1 < 0) { const double t = -c0 / c1; if (t < h) h = t; }
          else if (c0 < 0) dead = true;
        }
        if (!dead && l <= h) { lo[n] = l; hi[n] = h; ++n; }
      }
      // == sorted sweep "no gap, reach >= 1" (intervals lie in [0, 1])
      double reach = 0.0;
      bool grew = true;
      while (grew) {
        grew = false;
        for (int i = 0; i < n; ++i) {
          if (lo[i] <= reach) {
            if (hi[i] > reach) reach = hi[i];
            lo[i] = 2.0;  // consumed
            grew = true;
          }
        }
      }
#else
      double reach = 0.0;
      for (int pass = 0; pass <= j1 - j0 && reach < 1.0; ++pass) {
        // another pass can only help if this one grew the reach AND left an interval starting beyond it
        bool grew = false, skipped = false;
        for (int p = j0; p < j1 && reach < 1.0; ++p) {
          const int o = g.poly_off[p], m = g.poly_off[p + 1] - o;
          const double* V = g.vert + 2 * o;
          double l = 0.0, h = 1.0;
          bool dead = false;
          for (int i = 0; i < m; ++i) {
            const int j = (i + 1) == m ? 0 : i + 1;
            const double vx = V[2 * i], vy = V[2 * i + 1];
            const double ex = V[2 * j] - vx, ey = V[2 * j + 1] - vy;
            const double c0 = ex * (Ay - vy) - ey * (Ax - vx);
            const double c1 = ex * (By - Ay) - ey * (Bx - Ax);
            if (c1 > 0) { const double t = -c0 / c1; if (t > l) l = t; }
            else if (c1 < 0) { const double t = -c0 / c1; if (t < h) h = t; }
            else if (c0 < 0) dead = true;
          }
          if (!dead && l <= h) {
            if (l > reach) skipped = true;
            else if (h > reach) { reach = h; grew = true; }
          }
        }
        if (!grew || !skipped) break;
      }
#endif
      if (!(reach >= 1.0)) return false;
    }
    return true;
  }

  // The footprint's rotation takes htp_fastm.h's sincos (explicit FMA, <= 2 ulp, the same doubles on the device
  // and the host build), not the double-double libm: only a collision boolean depends on it, and a last-bit
  // difference flips one only for a body within ~1e-15 m of a boundary (the oracle's numpy cos / sin are not
  // correctly rounded either).  Trajectory samples and grid indices keep htp_libm.h.
  // NBC: the body's vertex count as a compile-time constant (4: the planners' rectangular bodies), so the corner
  // arrays are indexed by constants and stay in registers; 0: the run-time count (scratch memory)
  template <int NBC>
  HTP_HD bool pose_hits_t(double x, double y, double yaw) const {
    const int nb = NBC ? NBC : this->nb;
    double sn, cs;
    fm::sincos(yaw, sn, cs);
    double bx[NBC ? NBC : MAXB], by[NBC ? NBC : MAXB];
    for (int k = 0; k < nb; ++k) {
      const double vx = body[2 * k], vy = body[2 * k + 1];
      bx[k] = cs * vx + (-sn) * vy + x;
      by[k] = sn * vx + cs * vy + y;
    }
    for (int p = blk0; p < blk1; ++p)
      if (sat_hit<NBC>(bx, by, p)) return true;
    if (field >= 0 && !in_field<NBC>(bx, by, field)) return true;
    if (lane1 > lane0 && !in_lanes<NBC>(bx, by)) return true;
    return false;
  }
  HTP_HD bool pose_hits(double x, double y, double yaw) const {
    return nb == 4 ? pose_hits_t<4>(x, y, yaw) : pose_hits_t<0>(x, y, yaw);
  }

};

template <class C>
struct Search {
  C& c;
  const double* prm;
  const int32_t* dsc;
  Geo g;
  Work w;
  Shared& sh;
  int nb, nmot;
  double res, yaw_res, wb, curv_max, maxsteer;
  Footprint fp;

  HTP_HD Search(C& c_, const double* p, const int32_t* d, const Geo& g_, const Work& w_, Shared& s)
      : c(c_), prm(p), dsc(d), g(g_), w(w_), sh(s) {
    res = prm[P_RES];
    yaw_res = prm[P_YAWRES];
    wb = prm[P_WB];
    curv_max = prm[P_CURV];
    maxsteer = prm[P_MAXSTEER];
    nmot = dsc[D_MOT1] - dsc[D_MOT0];
    const int b0 = g.poly_off[dsc[D_BODY]];
    nb = g.poly_off[dsc[D_BODY] + 1] - b0;
    for (int q = c.lane; q < 2 * nb; q += C::width) sh.body[q] = g.vert[2 * b0 + q];
    c.sync();
    fp = Footprint{g, sh.body, nb, dsc[D_BLK0], dsc[D_BLK1], dsc[D_FIELD], dsc[D_LANE0], dsc[D_LANE1]};
  }

  HTP_HD bool pose_hits(double x, double y, double yaw) const { return fp.pose_hits(x, y, yaw); }

  // ------------------------------------------------------------ reductions
  HTP_HD int any(int v) const { return c.isum(v ? 1 : 0) > 0; }
  // (value, index) min with the smallest index on ties; result uniform.
  HTP_HD void argmin(double& v, int& i) const {
    if (C::width == 1) return;
    sh.red_d[c.lane] = v;
    sh.red_i[c.lane] = i;
    c.sync();
    double bv = sh.red_d[0];
    int bi = sh.red_i[0];
    for (int l = 1; l < C::width; ++l) {
      const double ov = sh.red_d[l];
      const int oi = sh.red_i[l];
      if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    c.sync();
    v = bv;
    i = bi;
  }

  // ------------------------------------------------------------ heuristic
  HTP_HD double search_length(double x, double y) const {  // get_search_length :120-129
    double out = prm[P_DEFLEN];
    for (int p = dsc[D_LANE0]; p < dsc[D_LANE1]; ++p) {
      const int o = g.poly_off[p], m = g.poly_off[p + 1] - o;
      const double* V = g.vert + 2 * o;
      bool in = true;
      for (int i = 0; i < m && in; ++i) {
        const int j = (i + 1) == m ? 0 : i + 1;
        const double cr = (V[2 * j] - V[2 * i]) * (y - V[2 * i + 1]) - (V[2 * j + 1] - V[2 * i + 1]) * (x - V[2 * i]);
        in = cr > 0;
      }
      if (in) out = g.lane_len[p];
    }
    return out;
  }

  HTP_HD double heuristic(double x, double y, double yaw) {  // calculate_state_cost :131-158
    const int G0 = dsc[D_GUIDE0], G1 = dsc[D_GUIDE1];
    double best = 0.0;
    int bi = -1;
    for (int q = G0 + c.lane; q < G1; q += C::width) {
      const double d = hm::hypot(g.guide[4 * q] - x, g.guide[4 * q + 1] - y);
      if (bi < 0 || d < best) { best = d; bi = q; }
    }
    if (bi < 0) { best = __builtin_huge_val(); bi = 0x7fffffff; }
    argmin(best, bi);
    double dtp = best * 100;
    const double yaw_diff = fabs(angle_wrap(g.guide[4 * bi + 2] - yaw));
    if (dtp > 2.0) dtp = 100.0;
    const double dist_to_goal = g.guide[4 * (G1 - 1) + 3] - g.guide[4 * bi + 3];
    return dtp + yaw_diff * 0.2 + dist_to_goal * 5;
  }

  HTP_HD static double prio(double cost, double h) {
    const double b = 50 * h;
    return b > cost ? b : cost;  // Python max(cost, 50 h)
  }

  HTP_HD void index(double x, double y, double yaw, int32_t* k) const {
    k[0] = (int32_t)rint(x / res);
    k[1] = (int32_t)rint(y / res);
    k[2] = (int32_t)rint(yaw / yaw_res);
  }

  // ------------------------------------------------------------ table + heapdict
  HTP_HD int find(const int32_t* k) const {  // slot of key (existing or empty)
    uint32_t h = (uint32_t)k[0] * 73856093u ^ (uint32_t)k[1] * 19349663u ^ (uint32_t)k[2] * 83492791u;
    uint32_t m = (uint32_t)w.cap_slot - 1u;
    for (uint32_t i = h & m;; i = (i + 1) & m) {
      const Slot& s = w.slot[i];
      if (s.state == 0 || (s.kx == k[0] && s.ky == k[1] && s.kt == k[2])) return (int)i;
    }
  }
  HTP_HD void hswap(int i, int j) {
    const double vi = w.hval[i], vj = w.hval[j];
    const int32_t si = w.hslot[i], sj = w.hslot[j];
    w.hval[i] = vj; w.hslot[i] = sj;
    w.hval[j] = vi; w.hslot[j] = si;
    w.slot[sj].hpos = i;
    w.slot[si].hpos = j;
  }
  HTP_HD void decrease_key(int i) {
    while (i) {
      const int p = (i - 1) >> 1;
      if (w.hval[p] < w.hval[i]) break;
      hswap(i, p);
      i = p;
    }
  }
  HTP_HD void heapify(int i, int n) {
    for (;;) {
      const int l = 2 * i + 1, r = 2 * i + 2;
      int low = (l < n && w.hval[l] < w.hval[i]) ? l : i;
      if (r < n && w.hval[r] < w.hval[low]) low = r;
      if (low == i) break;
      hswap(i, low);
      i = low;
    }
  }
  HTP_HD int popitem(int& n) {  // -> slot
    const int s = w.hslot[0];
    if (n == 1) {
      n = 0;
    } else {
      --n;
      w.hval[0] = w.hval[n];
      w.hslot[0] = w.hslot[n];
      w.slot[w.hslot[0]].hpos = 0;
      heapify(0, n);
    }
    w.slot[s].hpos = -1;
    return s;
  }
  HTP_HD void hset(int s, double v, int& n) {  // heapdict.__setitem__
    if (w.slot[s].hpos >= 0) {
      int i = w.slot[s].hpos;
      while (i) {
        const int p = (i - 1) >> 1;
        hswap(i, p);
        i = p;
      }
      popitem(n);
    }
    w.hval[n] = v;
    w.hslot[n] = s;
    w.slot[s].hpos = n;
    ++n;
    decrease_key(n - 1);
  }

  // ------------------------------------------------------------ motion primitives
  // Lane m integrates primitive m from pose (x0, y0, yaw0) with n steps into sh.traj.
  HTP_HD void simulate(int m, double x0, double y0, double yaw0, int n) {
    const double steer = g.motion[2 * (dsc[D_MOT0] + m)], dir = g.motion[2 * (dsc[D_MOT0] + m) + 1];
    const double yaw_step = dir * res / wb * hm::tan(steer);
    const double init_yaw = angle_wrap(yaw0 + yaw_step);
    const double stop = init_yaw + yaw_step * (double)(n + 1);
    const int num = n + 2;
    const double div = (double)(n + 1);
    const double delta = stop - init_yaw;
    const double step = delta / div;
    double ax = 0.0, ay = 0.0;
    double* T = sh.traj + m * (n + 1) * 3;
    for (int i = 0; i <= n; ++i) {  // numpy linspace (step == 0 branch included), angle_wrap, cumsum
      const double yi = (step == 0) ? ((double)i / div) * delta + init_yaw : (double)i * step + init_yaw;
      const double wy = angle_wrap(yi);
      const double dx = res * hm::cos(wy) * dir;
      const double dy = res * hm::sin(wy) * dir;
      ax = (i == 0) ? dx : ax + dx;
      ay = (i == 0) ? dy : ay + dy;
      const double ni = (i + 1 == num - 1) ? stop : ((step == 0) ? ((double)(i + 1) / div) * delta + init_yaw
                                                                : (double)(i + 1) * step + init_yaw);
      T[3 * i] = x0 + ax;
      T[3 * i + 1] = y0 + ay;
      T[3 * i + 2] = angle_wrap(ni);
    }
  }

  // simulated_path_cost :306-329 for primitive m (trajectory in sh.traj)
  HTP_HD double motion_cost(int m, int n, const Node& par) const {
    const double steer = g.motion[2 * (dsc[D_MOT0] + m)], dir = g.motion[2 * (dsc[D_MOT0] + m) + 1];
    const double* T = sh.traj + m * (n + 1) * 3;
    double cost = par.cost;
    double pl = 0.0;
    for (int i = 0; i < n; ++i) {
      const double d = hm::hypot(T[3 * (i + 1)] - T[3 * i], T[3 * (i + 1) + 1] - T[3 * i + 1]);
      pl = (i == 0) ? d : pl + d;
    }
    cost += pl;
    if (dir == -1) cost += 5000;
    cost += steer * 1;
    const double sa = hm::atan(par.curv * wb);
    cost += fabs(steer - sa) * 5;
    if ((double)par.dir != dir) cost += 1000;
    return cost;
  }

  // ------------------------------------------------------------ Reeds-Shepp goal shot
  // all admissible words from (sx, sy, syaw) to the goal into sh.paths; returns n or -1 (assert/capacity)
  HTP_HD int rs_paths(double sx, double sy, double syaw) {
    const double gx = prm[P_GX], gy = prm[P_GY], gyaw = prm[P_GYAW];
    const double maxc = curv_max;
    const double dx = gx - sx, dy = gy - sy, dth = gyaw - syaw;
    const double cc = hm::cos(syaw), ss = hm::sin(syaw);
    const double x = (cc * dx + ss * dy) * maxc;
    const double y = (-ss * dx + cc * dy) * maxc;
    const double xb = x * hm::cos(dth) + y * hm::sin(dth);
    const double yb = x * hm::sin(dth) - y * hm::cos(dth);
    const rs::Cand* T = rs::cand_table();
    for (int k = c.lane; k < 46; k += C::width) {
      const rs::Cand& cd = T[k];
      const bool back = cd.arg >= 4;
      const double bx = back ? xb : x, by = back ? yb : y;
      const int am = cd.arg & 3;
      const double ax = (am == 1 || am == 3) ? -bx : bx;
      const double ay = (am == 2 || am == 3) ? -by : by;
      const double ap = (am == 1 || am == 2) ? -dth : dth;
      double t = 0, u = 0, v = 0;
      int n = 0;
      if (rs::eval_word(cd.word, ax, ay, ap, t, u, v)) n = rs::lengths_of(cd.lmode, t, u, v, sh.cand_len + 5 * k);
      sh.cand_n[k] = n;
    }
    c.sync();
    rs::PathSet S{sh.paths, 0, 0};
    for (int k = 0; k < 46; ++k)
      if (sh.cand_n[k] > 0) rs::add_path(S, sh.cand_n[k], sh.cand_len + 5 * k, T[k].ty);
    c.sync();
    if (S.err) return -1;
    // generate_local_course must not raise for any path (calc_all_paths samples all of them first)
    for (int p = 0; p < S.n; ++p)
      if (!course_ok(sh.paths[p], maxc * res)) return -1;
    return S.n;
  }

  // index-only replay of rs::local_course: true unless the reference raises IndexError
  HTP_HD static bool course_ok(const rs::Path& p, double step) {
    const int np = rs::point_num(p, step);
    int ind = 1, cur = 0;
    double d, pd = (p.len[0] > 0.0) ? step : -step, ll = 0.0;
    for (int i = 0; i < p.nseg; ++i) {
      const double l = p.len[i];
      d = (l > 0.0) ? step : -step;
      ind -= 1;
      if (i >= 1 && (p.len[i - 1] * p.len[i]) > 0) pd = -d - ll;
      else pd = d - ll;
      while (fabs(pd) <= fabs(l)) {
        ind += 1;
        if (ind != cur && ind != cur + 1) return false;
        cur = ind;
        if (ind >= np) return false;
        pd += d;
      }
      ll = l - pd - d;
      ind += 1;
      if (ind != cur && ind != cur + 1) return false;
      cur = ind;
      if (ind >= np) return false;
    }
    return true;
  }

  // Streams the samples of path p (global frame) through the collision test in
  // chunks of 64; true if any sample collides.
  HTP_HD bool rs_path_hits(const rs::Path& p, double sx, double sy, double syaw, int64_t& n_pose) {
    const double maxc = curv_max, step = maxc * res;
    const double cq = hm::cos(-syaw), sq = hm::sin(-syaw);
    // segment origins (the previous segment's end sample, zeros first)
    double ox = 0.0, oy = 0.0, oyaw = 0.0;
    for (int i = 0; i < p.nseg; ++i) {
      sh.org[3 * i] = ox; sh.org[3 * i + 1] = oy; sh.org[3 * i + 2] = oyaw;
      double px, py, pyaw, cs;
      int dir;
      rs::interp(p.len[i], p.typ[i], maxc, ox, oy, oyaw, px, py, pyaw, cs, dir);
      if (p.typ[i] == rs::SEG_S) pyaw = oyaw;
      ox = px; oy = py; oyaw = pyaw;
    }
    c.sync();
    int base = 0, top = 0;  // chunk [base, base+64), top = highest index written + 1
    bool hit = false;
    auto flush = [&](int upto) -> bool {  // test indices [base, upto)
      c.sync();
      int h = 0;
      for (int q = base + c.lane; q < upto; q += C::width) {
        const int j = q - base;
        const int si = sh.pseg[j];
        double lx, ly, lyaw, cs;
        int dir;
        if (si < 0) { lx = 0.0; ly = 0.0; lyaw = 0.0; }
        else {
          rs::interp<true>(sh.pd[j], p.typ[si], maxc, sh.org[3 * si], sh.org[3 * si + 1], sh.org[3 * si + 2], lx, ly,
                           lyaw, cs, dir);
          if (p.typ[si] == rs::SEG_S) lyaw = sh.org[3 * si + 2];
        }
        const double gx = cq * lx + sq * ly + sx;
        const double gy = -sq * lx + cq * ly + sy;
        const double gyaw = rs::pi2pi(lyaw + syaw);
        if (pose_hits(gx, gy, gyaw)) h = 1;
      }
      n_pose += upto - base;
      const int r = any(h);
      c.sync();
      return r;
    };
    auto put = [&](int k, double pdv, int si) -> bool {  // record the final writer of index k
      if (k >= base + 64) {
        if (flush(base + 64)) return true;
        base += 64;
      }
      sh.pd[k - base] = pdv;  // uniform: every lane stores the same value
      sh.pseg[k - base] = si;
      if (k + 1 > top) top = k + 1;
      return false;
    };
    if (put(0, 0.0, -1)) return true;
    int ind = 1;
    double d, pd = (p.len[0] > 0.0) ? step : -step, ll = 0.0;
    for (int i = 0; i < p.nseg && !hit; ++i) {
      const double l = p.len[i];
      d = (l > 0.0) ? step : -step;
      ind -= 1;
      if (i >= 1 && (p.len[i - 1] * p.len[i]) > 0) pd = -d - ll;
      else pd = d - ll;
      while (fabs(pd) <= fabs(l)) {
        ind += 1;
        if (put(ind, pd, i)) { hit = true; break; }
        pd += d;
      }
      if (hit) break;
      ll = l - pd - d;
      ind += 1;
      if (put(ind, l, i)) { hit = true; break; }
    }
    if (hit) return true;
    return flush(top);
  }

  // RS goal shot: index of the path taken (generation order) or -1; cost in *out_cost
  HTP_HD int goal_shot(const Node& cur, double& out_cost, int& err, int64_t& n_pose, int64_t& n_checks) {
    const int np = rs_paths(cur.x, cur.y, cur.yaw);
    if (np < 0) { err = 1; return -1; }
    if (np == 0) return -1;
    // calculate_reeds_shepp_path_cost :129-160 + heapdict insertion in path order
    int hn = 0;
    for (int k = 0; k < np; ++k) {
      const rs::Path& P = sh.paths[k];
      double cost = cur.cost;
      int nneg = 0;
      for (int j = 0; j < P.nseg; ++j) nneg += P.len[j] < 0 ? 1 : 0;
      cost += (double)(5000 * nneg + (P.nseg - nneg));
      cost += 1000.0;
      cost += maxsteer * 1 * 1;
      double ds = 0.0;
      for (int j = 0; j + 1 < P.nseg; ++j) {
        const double a = P.typ[j] == rs::SEG_R ? -maxsteer : 0.0;
        const double b = P.typ[j + 1] == rs::SEG_R ? -maxsteer : 0.0;
        ds = ds + fabs(b - a);
      }
      cost += ds;
      // heapdict __setitem__ of a new key
      int i = hn++;
      sh.rval[i] = cost;
      sh.rkey[i] = k;
      while (i) {
        const int pp = (i - 1) >> 1;
        if (sh.rval[pp] < sh.rval[i]) break;
        const double tv = sh.rval[pp]; sh.rval[pp] = sh.rval[i]; sh.rval[i] = tv;
        const int tk = sh.rkey[pp]; sh.rkey[pp] = sh.rkey[i]; sh.rkey[i] = tk;
        i = pp;
      }
    }
    while (hn > 0) {
      const int k = sh.rkey[0];
      const double v = sh.rval[0];
      if (hn == 1) hn = 0;
      else {
        --hn;
        sh.rval[0] = sh.rval[hn];
        sh.rkey[0] = sh.rkey[hn];
        int i = 0;
        for (;;) {
          const int l = 2 * i + 1, r = 2 * i + 2;
          int low = (l < hn && sh.rval[l] < sh.rval[i]) ? l : i;
          if (r < hn && sh.rval[r] < sh.rval[low]) low = r;
          if (low == i) break;
          const double tv = sh.rval[low]; sh.rval[low] = sh.rval[i]; sh.rval[i] = tv;
          const int tk = sh.rkey[low]; sh.rkey[low] = sh.rkey[i]; sh.rkey[i] = tk;
          i = low;
        }
      }
      const rs::Path& P = sh.paths[k];
      if (!(P.L / curv_max < 1000.0)) continue;  // path.L < MIN_LENGTH_TO_GOAL (checked first: same outcome)
      ++n_checks;
      if (!rs_path_hits(P, cur.x, cur.y, cur.yaw, n_pose)) {
        out_cost = v;
        return k;
      }
    }
    return -1;
  }

  // ------------------------------------------------------------ Dubins goal shot (Pawn)
  // get_dubins_path :289-304 for the pose (x0, y0, yaw0): Dubins samples + goal,
  // arc-length spline fit.  Leaves X, Y, S, DX, DY (m points) in w.dub; returns
  // the number of spline samples (np.arange(0, s_end + ds, ds)), -1 on overflow.
  HTP_HD int dubins_fit(double x0, double y0, double yaw0, int& m) {
    const int cap = w.cap_dub + 16;
    double* X = w.dub;
    double* Y = X + cap;
    double* S = Y + cap;
    double* DX = S + cap;
    double* DY = DX + cap;
    double* WK = DY + cap;
    const double q0[3] = {x0, y0, yaw0}, q1[3] = {prm[P_GX], prm[P_GY], prm[P_GYAW]};
    dub::Path P;
    if (!dub::shortest(q0, q1, 1.0 / curv_max, P)) {
#ifdef HTP_HA_DEBUG
      if (c.lane == 0) printf("dub shortest fail %.17g %.17g %.17g\n", x0, y0, yaw0);
#endif
      return -1;
    }
    const double L = dub::length(P);
    int n = 0;
    double xs = 0.0;
    while (xs < L) {  // sample_many: x = 0, step, 2 step ... (sequential sums)
      if (n >= w.cap_dub) {
#ifdef HTP_HA_DEBUG
        if (c.lane == 0) printf("dub n overflow L=%.17g\n", L);
#endif
        return -1;
      }
      S[n] = xs;
      ++n;
      xs += res;
    }
    c.sync();
    for (int k = c.lane; k < n; k += C::width) {
      double q[3];
      dub::sample(P, S[k], q);
      X[k] = q[0];
      Y[k] = q[1];
    }
    c.sync();
    X[n] = q1[0];  // uniform: every lane stores the same value
    Y[n] = q1[1];
    c.sync();
    // drop point i when point i+1 repeats it (cubic_spline.py:94-99), then s
    int mm = 0;
    for (int i = 0; i <= n; ++i) {
      const bool dup = i < n && X[i + 1] == X[i] && Y[i + 1] == Y[i];
      if (!dup) {  // uniform: every lane moves the same values
        const double xi = X[i], yi = Y[i];
        X[mm] = xi;
        Y[mm] = yi;
        ++mm;
      }
    }
    c.sync();
    S[0] = 0.0;
    for (int i = 1; i < mm; ++i) S[i] = S[i - 1] + hm::hypot(X[i] - X[i - 1], Y[i] - Y[i - 1]);
    c.sync();
    m = mm;
#ifdef HTP_HA_DEBUG
    if (c.lane == 0) printf("dub fit L=%.17g n=%d m=%d S=%.17g\n", L, n, mm, S[mm - 1]);
#endif
    if (m < 2) return -1;
    if (c.lane == 0 || C::width == 1) dub::spline_slopes(S, X, m, DX, WK);
    if (c.lane == (C::width > 1 ? 1 : 0)) dub::spline_slopes(S, Y, m, DY, WK + 4 * cap);
    c.sync();
    const double ns = ceil((S[m - 1] + res) / res);
    if (!(ns >= 1) || ns > (double)w.cap_dub) {
#ifdef HTP_HA_DEBUG
      if (c.lane == 0) printf("dub ns bad %.17g\n", ns);
#endif
      return -1;
    }
    return (int)ns;
  }

  // spline sample k: x, y, yaw (not wrapped), curvature
  HTP_HD void dubins_eval(int k, int m, double& x, double& y, double& yaw, double& kap) const {
    const int cap = w.cap_dub + 16;
    const double* X = w.dub;
    const double* Y = X + cap;
    const double* S = Y + cap;
    const double* DX = S + cap;
    const double* DY = DX + cap;
    const double v = (double)k * res;
    const int i = dub::interval(S, m, v);
    double x1, x2, y1, y2;
    dub::eval3(S, X, DX, i, v, x, x1, x2);
    dub::eval3(S, Y, DY, i, v, y, y1, y2);
    yaw = hm::atan2(y1, x1);
    kap = (y2 * x1 - x2 * y1) / hm::pow(x1 * x1 + y1 * y1, 1.5);
  }

  // _get_goal_extension_with_dubins_path :184-230: true if the shot is taken
  HTP_HD bool goal_shot_dubins(const Node& cur, int& err, int64_t& n_pose, int64_t& n_checks) {
    int m = 0;
    const int ns = dubins_fit(cur.x, cur.y, cur.yaw, m);
    if (ns < 0) { err = 1; return false; }
    const int cap = w.cap_dub + 16;
    double* XS = w.dub + 13 * cap;
    double* YS = XS + cap;
    double* YW = YS + cap;
    for (int k = c.lane; k < ns; k += C::width) {
      double x, y, yaw, kap;
      dubins_eval(k, m, x, y, yaw, kap);
      XS[k] = x;
      YS[k] = y;
      YW[k] = angle_wrap(yaw);
    }
    c.sync();
    // calculate_path_length: cumsum of hypot(diff) (sequential)
    double len = 0.0;
    for (int k = 1; k < ns; ++k) {
      const double h = hm::hypot(XS[k] - XS[k - 1], YS[k] - YS[k - 1]);
      len = (k == 1) ? h : len + h;
    }
    if (!(len < 1000.0)) return false;  // path_length < MIN_LENGTH_TO_GOAL (checked first: same outcome)
    ++n_checks;
    for (int base = 0; base < ns; base += 64) {  // collision, 64 samples at a time, early exit
      int h = 0;
      for (int k = base + c.lane; k < base + 64 && k < ns; k += C::width)
        if (pose_hits(XS[k], YS[k], YW[k])) h = 1;
      n_pose += (ns - base) < 64 ? (ns - base) : 64;
      if (any(h)) return false;
    }
    return true;
  }

  HTP_HD bool traj_hits_single(double x, double y, double yaw, int64_t& n_pose) {
    int h = 0;
    if (c.lane == 0) h = pose_hits(x, y, yaw) ? 1 : 0;
    ++n_pose;
    return any(h);
  }

  // ------------------------------------------------------------ search
  HTP_HD int new_node(int& nn) {
    if (nn >= w.cap_node) return -1;
    return nn++;
  }

  // KING: Reeds-Shepp goal shots (motion_type "King"); otherwise Dubins (Pawn).
  // The device instantiates one kernel per motion type, so neither carries the
  // other's goal-shot code (register pressure).
  HTP_HD void run(Out& o, int32_t* log, int cap_log) {
    if (dsc[D_KING]) run_t<true>(o, log, cap_log);
    else run_t<false>(o, log, cap_log);
  }

  template <bool KING>
  HTP_HD void run_t(Out& o, int32_t* log, int cap_log) {
    o = Out{};
    const int max_nodes = (int)prm[P_MAXNODES];
    for (int q = c.lane; q < w.cap_slot; q += C::width) {
      w.slot[q].state = 0;
      w.slot[q].hpos = -1;
    }
    c.sync();
    int32_t sk[3], gk[3];
    index(prm[P_SX], prm[P_SY], prm[P_SYAW], sk);
    index(prm[P_GX], prm[P_GY], prm[P_GYAW], gk);
    int nn = 0, hn = 0;
    // start node
    Node st{};
    st.x = prm[P_SX]; st.y = prm[P_SY]; st.yaw = prm[P_SYAW]; st.cost = 0.0; st.curv = 0.0;
    st.kx = sk[0]; st.ky = sk[1]; st.kt = sk[2];
    st.pkx = sk[0]; st.pky = sk[1]; st.pkt = sk[2];
    st.parent = -1; st.kind = 0; st.aux = 0; st.dir = 1;
    const double h0 = heuristic(st.x, st.y, st.yaw);
    if (traj_hits_single(st.x, st.y, st.yaw, o.n_pose) || traj_hits_single(prm[P_GX], prm[P_GY], prm[P_GYAW], o.n_pose)) {
      o.n_checks += 2;
      o.status = ST_START_GOAL_BLOCKED;
      return;
    }
    o.n_checks += 2;
    {
      const int id = new_node(nn);
      if (c.lane == 0 || C::width == 1) w.node[id] = st;
      const int s = find(sk);
      if (c.lane == 0 || C::width == 1) {
        w.slot[s].kx = sk[0]; w.slot[s].ky = sk[1]; w.slot[s].kt = sk[2];
        w.slot[s].state = 1; w.slot[s].node = id;
      }
      c.sync();
      hset(s, prio(0.0, h0), hn);
      c.sync();
    }
    int counter = 0, status = ST_NO_PATH, goal_node = -1;
    for (;;) {
      if (counter > max_nodes) { status = ST_MAX_NODES; break; }
      counter += 1;
      if (hn == 0) { status = ST_NO_PATH; break; }
      const int s = popitem(hn);
      c.sync();
      const int cid = w.slot[s].node;
      if (c.lane == 0 || C::width == 1) w.slot[s].state = 2;
      const Node cur = w.node[cid];
      if (o.n_expanded < cap_log && (c.lane == 0 || C::width == 1)) {
        log[3 * o.n_expanded] = cur.kx; log[3 * o.n_expanded + 1] = cur.ky; log[3 * o.n_expanded + 2] = cur.kt;
      }
      o.n_expanded += 1;
      c.sync();
      // goal extension
      int err = 0;
      double gcost = 0.0;
      int pk = -1;
      if constexpr (KING) {
        pk = goal_shot(cur, gcost, err, o.n_pose, o.n_checks);
        if (err) { status = ST_RS_ERROR; break; }
      } else {
        const bool shot = goal_shot_dubins(cur, err, o.n_pose, o.n_checks);
        if (err) { status = ST_CAPACITY; break; }
        pk = shot ? 0 : -1;
      }
      int gid = -1;
      if (pk >= 0) {
        gid = new_node(nn);
        if (gid < 0) { status = ST_CAPACITY; break; }
        Node gn{};
        gn.x = prm[P_GX]; gn.y = prm[P_GY]; gn.yaw = prm[P_GYAW];  // end pose (unused: never expanded)
        gn.cost = gcost; gn.curv = 0.0; gn.kx = gk[0]; gn.ky = gk[1]; gn.kt = gk[2];
        gn.pkx = cur.kx; gn.pky = cur.ky; gn.pkt = cur.kt; gn.parent = cid; gn.kind = KING ? 2 : 3;
        gn.aux = (int16_t)pk;
        gn.dir = 1;
        if (c.lane == 0 || C::width == 1) w.node[gid] = gn;
      }
      // check_the_arrival :464-495 (goal pose = goal_node.traj[0])
      if (fabs(cur.x - prm[P_GX]) < res && fabs(cur.y - prm[P_GY]) < res &&
          fabs(angle_wrap(cur.yaw - prm[P_GYAW])) < yaw_res) {
        gid = new_node(nn);
        if (gid < 0) { status = ST_CAPACITY; break; }
        Node gn = cur;
        gn.kx = gk[0]; gn.ky = gk[1]; gn.kt = gk[2];
        if (c.lane == 0 || C::width == 1) {
          w.node[gid] = gn;
          w.node[cid].kx = gk[0]; w.node[cid].ky = gk[1]; w.node[cid].kt = gk[2];
        }
      }
      c.sync();
      if (gid >= 0) {
        const int gs = find(gk);
        if (c.lane == 0 || C::width == 1) {
          w.slot[gs].kx = gk[0]; w.slot[gs].ky = gk[1]; w.slot[gs].kt = gk[2];
          w.slot[gs].state = 2; w.slot[gs].node = gid;
        }
        c.sync();
        goal_node = gid;
        status = ST_FOUND;
        break;
      }
      // expansion: all primitives share the parent's search length
      const double L = search_length(cur.x, cur.y);
      const int n = (int)rint(L / res);
      if (n < 1 || n + 1 > MAXTRAJ || nmot * (n + 1) > TRAJCAP) { status = ST_BAD_INPUT; break; }
      for (int m = c.lane; m < nmot; m += C::width) {
        simulate(m, cur.x, cur.y, cur.yaw, n);
        sh.hit[m] = 0;
      }
      c.sync();
      const int tot = nmot * (n + 1);
      for (int q = c.lane; q < tot; q += C::width) {
        const int m = q / (n + 1), i = q - m * (n + 1);
        const double* T = sh.traj + (m * (n + 1) + i) * 3;
        if (pose_hits(T[0], T[1], T[2])) sh.hit[m] = 1;
      }
      o.n_pose += tot;
      o.n_checks += nmot;
      c.sync();
      for (int m = c.lane; m < nmot; m += C::width) {
        sh.ccost[m] = motion_cost(m, n, cur);
        const double steer = g.motion[2 * (dsc[D_MOT0] + m)];
        sh.ccurv[m] = hm::tan(steer) / wb;
        const double* T = sh.traj + (m * (n + 1) + n) * 3;
        index(T[0], T[1], T[2], sh.ckey + 3 * m);
      }
      c.sync();
      bool cap = false;
      for (int m = 0; m < nmot; ++m) {
        if (sh.hit[m]) continue;
        const int32_t* k = sh.ckey + 3 * m;
        const int s2 = find(k);
        const int state = w.slot[s2].state;
        if (state == 2) continue;
        const double cost = sh.ccost[m];
        if (state == 1 && !(cost < w.node[w.slot[s2].node].cost)) continue;
        const int id = new_node(nn);
        if (id < 0) { cap = true; break; }
        const double* T = sh.traj + (m * (n + 1) + n) * 3;
        Node ch{};
        ch.x = T[0]; ch.y = T[1]; ch.yaw = T[2]; ch.cost = cost; ch.curv = sh.ccurv[m];
        ch.kx = k[0]; ch.ky = k[1]; ch.kt = k[2];
        ch.pkx = cur.kx; ch.pky = cur.ky; ch.pkt = cur.kt;
        ch.parent = cid; ch.kind = 1; ch.aux = (int16_t)m;
        ch.dir = (int32_t)g.motion[2 * (dsc[D_MOT0] + m) + 1];
        const double h = heuristic(ch.x, ch.y, ch.yaw);
        if (c.lane == 0 || C::width == 1) {
          w.node[id] = ch;
          w.slot[s2].kx = k[0]; w.slot[s2].ky = k[1]; w.slot[s2].kt = k[2];
          w.slot[s2].state = 1; w.slot[s2].node = id;
        }
        c.sync();
        hset(s2, prio(cost, h), hn);
        c.sync();
      }
      if (cap) { status = ST_CAPACITY; break; }
    }
    o.counter = counter;
    o.status = status;
    (void)goal_node;
  }

  // get_path_from_expanded_nodes :429-454 -> number of samples written (or needed)
  HTP_HD int backtrack(int32_t* chain, int cap_chain, double* px, double* py, double* pyaw, double* pdir,
                       double* pk, int cap_path, int& status) {
    return dsc[D_KING] ? backtrack_t<true>(chain, cap_chain, px, py, pyaw, pdir, pk, cap_path, status)
                       : backtrack_t<false>(chain, cap_chain, px, py, pyaw, pdir, pk, cap_path, status);
  }

  template <bool KING>
  HTP_HD int backtrack_t(int32_t* chain, int cap_chain, double* px, double* py, double* pyaw, double* pdir,
                         double* pk, int cap_path, int& status) {
    // the start node is node 0; its grid index is the goal's if the start itself
    // arrived (check_the_arrival relabels the node object, :492-493)
    const int32_t sk[3] = {w.node[0].kx, w.node[0].ky, w.node[0].kt};
    int32_t gk[3];
    index(prm[P_GX], prm[P_GY], prm[P_GYAW], gk);
    int32_t k[3] = {gk[0], gk[1], gk[2]};
    int s = find(k);
    if (w.slot[s].state != 2) return 0;
    int nc = 0;
    while (!(k[0] == sk[0] && k[1] == sk[1] && k[2] == sk[2])) {
      if (nc >= cap_chain) { status = ST_BACKTRACK; return 0; }
      const int id = w.slot[s].node;
      if (c.lane == 0 || C::width == 1) chain[nc] = id;
      ++nc;
      const Node& nd = w.node[id];
      k[0] = nd.pkx; k[1] = nd.pky; k[2] = nd.pkt;
      s = find(k);
      if (w.slot[s].state != 2) { status = ST_BACKTRACK; return 0; }  // the reference raises KeyError
    }
    c.sync();
    int off = 0;
    for (int ci = nc - 1; ci >= 0; --ci) {
      const Node nd = w.node[chain[ci]];
      if (nd.kind == 0) {
        if (off < cap_path && (c.lane == 0 || C::width == 1)) {
          px[off] = nd.x; py[off] = nd.y; pyaw[off] = nd.yaw; pdir[off] = 1.0; pk[off] = 0.0;
        }
        off += 1;
      } else if (nd.kind == 1) {
        const Node par = w.node[nd.parent];
        const double L = search_length(par.x, par.y);
        const int n = (int)rint(L / res);
        if (c.lane == 0 || C::width == 1) simulate(nd.aux, par.x, par.y, par.yaw, n);
        c.sync();
        const double dir = g.motion[2 * (dsc[D_MOT0] + nd.aux) + 1];
        const double kv = hm::tan(g.motion[2 * (dsc[D_MOT0] + nd.aux)]) / wb;
        const double* T = sh.traj + nd.aux * (n + 1) * 3;
        for (int i = c.lane; i <= n; i += C::width)
          if (off + i < cap_path) {
            px[off + i] = T[3 * i]; py[off + i] = T[3 * i + 1]; pyaw[off + i] = T[3 * i + 2];
            pdir[off + i] = dir; pk[off + i] = kv;
          }
        off += n + 1;
        c.sync();
      } else if constexpr (!KING) {
        const Node par = w.node[nd.parent];
        int m = 0;
        const int ns = dubins_fit(par.x, par.y, par.yaw, m);
        for (int k = c.lane; k < ns; k += C::width)
          if (off + k < cap_path) {
            double x, y, yaw, kap;
            dubins_eval(k, m, x, y, yaw, kap);
            px[off + k] = x; py[off + k] = y; pyaw[off + k] = angle_wrap(yaw); pdir[off + k] = 1.0; pk[off + k] = kap;
          }
        off += ns > 0 ? ns : 0;
        c.sync();
      } else {
        const Node par = w.node[nd.parent];
        (void)rs_paths(par.x, par.y, par.yaw);
        const rs::Path P = sh.paths[nd.aux];
        c.sync();
        rs::NullSink ns;
        const int cnt = rs::local_course(P, curv_max, curv_max * res, ns);
        if (cnt > 0 && off + cnt <= cap_path && (c.lane == 0 || C::width == 1)) {
          struct DSink {
            double *x, *y, *yaw, *cs, *dir;
            int limit;
            double sx, sy, syaw, cq, sq;
            HTP_HD void put(int kk, double lx, double ly, double lyaw, double cc, int d) const {
              if (kk >= limit) return;
              x[kk] = cq * lx + sq * ly + sx;
              y[kk] = -sq * lx + cq * ly + sy;
              yaw[kk] = rs::pi2pi(lyaw + syaw);
              cs[kk] = cc;
              dir[kk] = (double)d;
            }
          } gs{px + off, py + off, pyaw + off, pk + off, pdir + off, cnt, par.x, par.y, par.yaw, hm::cos(-par.yaw),
               hm::sin(-par.yaw)};
          rs::local_course(P, curv_max, curv_max * res, gs);
        }
        off += cnt > 0 ? cnt : 0;
        c.sync();
      }
    }
    return off;
  }
};

}  // namespace ha
}  // namespace htp
