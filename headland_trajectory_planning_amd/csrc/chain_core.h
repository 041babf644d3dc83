// Device-resident warm-start -> OBCA input chain for the orchard workload (synth.make_orchard_instance):
// every step between the planners' kernels and the solver runs on the device, one problem per wavefront,
// with the host generator's arithmetic (numpy's expression order, pairwise sums, np.interp / linspace /
// searchsorted semantics) so the device-built instance equals the host-built one.
//
//   prep ..... the turn's length (np.sum of np.hypot of the path steps: numpy's pairwise summation),
//              ds = L / (N - 1), desired_v = min(ds / dT, 0.9): get_init_ref_path's inputs
//              (R/obca_py/util.py:62-113 at spacing ds / 2 = L / (2 N - 2))
//   resample . the init guess at N rows of even arc length (synth._resample_rows) and the headland width
//              the warm start needs (synth._needed_headland over the footprint of both pose sets):
//              max(6, needed + margin) -> the orchard producer's headland_width
//   pack ..... get_obstacles_for_OBCA's polygons (htp_oge_obstacles_batch) split into quads with the same
//              union, the rest of the orchard when fewer than M, the M closest to the warm start
//              (separating-axis gaps, stable order), cdd-style halfspaces -> obs_A / obs_b; init_traj; params
// Sequential pieces run on lane 0 (they are short); results are written once per problem.
#pragma once
#include <cmath>
#include "htp_libm.h"
#include <cstdint>

#include "oge_core.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace htp {
namespace chain {

constexpr int MAXQ = 64;     // candidate quads per problem
constexpr int MAXPV = 8;     // vertices per vehicle polygon

// numpy pairwise_sum (contiguous doubles): 8 accumulators up to 128 elements, halves above
HTP_HD inline double pairwise_sum(const double* a, int64_t n) {
  if (n < 8) {
    double r = 0.0;   // numpy starts from -0.0 for n < 8; adding any value gives the same result
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return n == 0 ? 0.0 : r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

// np.interp(x, xp, fp) for increasing xp (ties allowed), numpy's arr_interp
HTP_HD inline double interp(double x, const double* xp, const double* fp, int n, int stride) {
  if (x >= xp[n - 1]) return x == xp[n - 1] ? fp[(int64_t)(n - 1) * stride] : fp[(int64_t)(n - 1) * stride];
  if (x < xp[0]) return fp[0];
  int lo = 0, hi = n - 1;   // largest j with xp[j] <= x
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (xp[mid] <= x) lo = mid;
    else hi = mid;
  }
  const int j = lo;
  const double yj = fp[(int64_t)j * stride], yk = fp[(int64_t)(j + 1) * stride];
  if (xp[j] == x) return yj;
  const double slope = (yk - yj) / (xp[j + 1] - xp[j]);
  double r = slope * (x - xp[j]) + yj;
  if (r != r) {
    r = slope * (x - xp[j + 1]) + yk;
    if (r != r && yj == yk) r = yj;
  }
  return r;
}

struct Vehicle {             // car-frame polygons of the footprint (body, then implements)
  int npoly;
  int nv[2];
  double v[2][MAXPV][2];
};

// the polygon `k` of the vehicle placed at pose (x, y, th) (synth._polys_at arithmetic)
HTP_HD inline void place(const Vehicle& V, int k, double x, double y, double th, double* px, double* py) {
  const double c = hm::cos(th), s = hm::sin(th);
  for (int j = 0; j < V.nv[k]; ++j) {
    px[j] = V.v[k][j][0] * c - V.v[k][j][1] * s + x;
    py[j] = V.v[k][j][0] * s + V.v[k][j][1] * c + y;
  }
}

// synth._min_sat_gap for one placed polygon F (m vertices) and a quad Q: max over the unit edge normals of
// both of the projection gap
HTP_HD inline double sat_gap(const double* fx, const double* fy, int m, const double (*Q)[2], int nq) {
  double best = -INFINITY;
  for (int side = 0; side < 2; ++side) {
    const int ne = side == 0 ? m : nq;
    for (int e = 0; e < ne; ++e) {
      double ex, ey;
      if (side == 0) { const int e1 = (e + 1) % m; ex = fx[e1] - fx[e]; ey = fy[e1] - fy[e]; }
      else { const int e1 = (e + 1) % nq; ex = Q[e1][0] - Q[e][0]; ey = Q[e1][1] - Q[e][1]; }
      double nx = ey, ny = -ex;
      const double nn = sqrt(nx * nx + ny * ny);
      nx = nx / nn;
      ny = ny / nn;
      double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
      for (int j = 0; j < m; ++j) {
        const double d = fx[j] * nx + fy[j] * ny;
        amin = d < amin ? d : amin;
        amax = d > amax ? d : amax;
      }
      for (int j = 0; j < nq; ++j) {
        const double d = Q[j][0] * nx + Q[j][1] * ny;
        bmin = d < bmin ? d : bmin;
        bmax = d > bmax ? d : bmax;
      }
      const double g1 = bmin - amax, g2 = amin - bmax;
      const double g = g1 > g2 ? g1 : g2;
      best = g > best ? g : best;
    }
  }
  return best;
}

}  // namespace chain
}  // namespace htp

namespace htp {
namespace chain {

// ---- prep: classic rows -> refpath inputs (one problem, lane 0)
HTP_HD inline void prep(const double* rows, int n, int N, double dT, double wb, double* xs, double* ys, double* dirs,
                        double* steps, double* rp_params) {
  for (int i = 0; i < n; ++i) {
    xs[i] = rows[5 * i];
    ys[i] = rows[5 * i + 1];
    dirs[i] = rows[5 * i + 4];
  }
  for (int i = 0; i + 1 < n; ++i) steps[i] = hm::hypot(rows[5 * (i + 1)] - rows[5 * i], rows[5 * (i + 1) + 1] - rows[5 * i + 1]);
  const double Lp = pairwise_sum(steps, n - 1);
  const double ds = Lp / (N - 1);
  const double dv = ds / dT;
  rp_params[0] = wb;
  rp_params[1] = dv < 0.9 ? dv : 0.9;   // min(ds / dT, 0.9)
  rp_params[2] = Lp / (2.0 * N - 2.0);   // ds / 2 (synth.make_orchard_instance)
}

// ---- resample (synth._resample_rows): init-guess rows -> N rows at even arc length (one lane)
// ref: [nr][5] init-guess rows; s: nr scratch doubles; traj: [N][5] out.
HTP_HD inline void resample(const double* ref, int nr, int N, double* s, double* traj) {
  s[0] = 0.0;
  for (int i = 1; i < nr; ++i) s[i] = s[i - 1] + hm::hypot(ref[5 * i] - ref[5 * (i - 1)], ref[5 * i + 1] - ref[5 * (i - 1) + 1]);
  const double send = s[nr - 1];
  const double tstep = send / (N - 1);
  for (int k = 0; k < N; ++k) {
    const double t = k == N - 1 ? send : (double)k * tstep + 0.0;   // np.linspace(0, s[-1], N)
    double* o = traj + 5 * k;
    o[0] = interp(t, s, ref + 0, nr, 5);
    o[1] = interp(t, s, ref + 1, nr, 5);
    o[3] = interp(t, s, ref + 3, nr, 5);
    o[4] = interp(t, s, ref + 4, nr, 5);
    int idx = 0;   // np.searchsorted(s, t, side="right"), clipped to [1, nr - 1]
    {
      int lo = 0, hi = nr;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] <= t) lo = mid + 1;
        else hi = mid;
      }
      idx = lo < 1 ? 1 : (lo > nr - 1 ? nr - 1 : lo);
    }
    double v = ref[5 * idx + 2];
    if (v == 0.0) v = ref[5 * (idx - 1) + 2];
    o[2] = v;
  }
  traj[2] = 0.0;
  traj[5 * (N - 1) + 2] = 0.0;
  traj[4] = 0.0;
}

// ---- resample + the headland width the warm start needs (lane 0).  Returns hw.
HTP_HD inline double resample_hw(const double* ref, int nr, int N, double* s, double* traj, const Vehicle& V,
                                 const oge::Scene& S, double margin) {
  resample(ref, nr, N, s, traj);
  // _needed_headland over the footprint at the N resampled poses and every init-guess row
  const double ang = oge::headland_angle(S, oge::NEAR);
  double ys[oge::MAXR], xs[oge::MAXR];
  for (int i = 0; i < S.n; ++i) { ys[i] = S.ry[i][0]; xs[i] = S.rx[i][0]; }
  double need = -INFINITY;
  for (int k = 0; k < V.npoly; ++k) {
    for (int p = 0; p < N + nr; ++p) {
      const double* r = p < N ? traj + 5 * p : ref + 5 * (p - N);
      double px[MAXPV], py[MAXPV];
      place(V, k, r[0], r[1], r[3], px, py);
      for (int j = 0; j < V.nv[k]; ++j) {
        const double d = interp(py[j], ys, xs, S.n, 1) - px[j];
        need = d > need ? d : need;
      }
    }
  }
  const double nh = need * fabs(hm::sin(ang)) + margin;
  return nh > 6.0 ? nh : 6.0;
}

// ---- pack: producer polygons -> M quads (split, orchard extension, nearest M, dummies) -> halfspaces.
// Returns 0, or 1 when a quad's hull has fewer than 4 facets / the pool overflows.
HTP_HD inline int pack(const oge::PolyOut& po, const oge::SceneIn& in, const oge::Scene& S, const double* traj, int N,
                       const double* ref, int nr, const Vehicle& V, int M, double* A, double* b) {
  double Q[MAXQ][4][2];
  int nq = 0;
  for (int p = 0; p < po.n; ++p) {   // synth._split_quads
    const int n = po.nv[p];
    if (n <= 4) {
      if (nq >= MAXQ || n != 4) return 1;
      for (int j = 0; j < 4; ++j) { Q[nq][j][0] = po.xy[p][j][0]; Q[nq][j][1] = po.xy[p][j][1]; }
      ++nq;
      continue;
    }
    int i = 1;
    for (;;) {
      const int j = i < n - 3 ? i : n - 3;
      if (nq >= MAXQ) return 1;
      const int idx[4] = {0, j, j + 1, j + 2};
      for (int t = 0; t < 4; ++t) { Q[nq][t][0] = po.xy[p][idx[t]][0]; Q[nq][t][1] = po.xy[p][idx[t]][1]; }
      ++nq;
      if (j + 2 >= n - 1) break;
      i += 2;
    }
  }
  if (nq < M) {   // the rest of the orchard: tree rows not used by get_obstacle_tree_rows, nearest first
    const double hi = in.start[1] > in.end[1] ? in.start[1] : in.end[1];
    const double lo = in.start[1] < in.end[1] ? in.start[1] : in.end[1];
    int low_idx = -1, up_idx = -1;
    for (int i = 0; i < S.n; ++i)
      if (S.ry[i][0] > lo && S.ry[i][0] < hi) { if (low_idx < 0) low_idx = i; up_idx = i; }
    int a, c;
    if (low_idx == up_idx) { a = up_idx - 2 > 0 ? up_idx - 2 : 0; c = up_idx + 2 < S.n - 1 ? up_idx + 2 : S.n - 1; }
    else { a = low_idx - 2 > 0 ? low_idx - 2 : 0; c = up_idx + 3 < S.n - 1 ? up_idx + 3 : S.n - 1; }
    const double mid = 0.5 * (in.start[1] + in.end[1]);
    int ord[oge::MAXR], no = 0;
    double key[oge::MAXR];
    for (int i = 0; i < S.n; ++i) {
      if (i >= a && i < c) continue;
      const double kv = fabs(S.ry[i][0] - mid);
      int t = no++;   // insertion by (distance, index)
      while (t > 0 && key[t - 1] > kv) { key[t] = key[t - 1]; ord[t] = ord[t - 1]; --t; }
      key[t] = kv;
      ord[t] = i;
    }
    for (int t = 0; t < no; ++t) {
      if (nq >= MAXQ) return 1;
      oge::row_rect(S, ord[t], in.tree_width, false, Q[nq]);
      ++nq;
    }
    // the other bound quad (create_boundary_polygons :336-371)
    int ui = 0, li = 0;
    for (int i = 1; i < S.n; ++i) { if (S.ry[i][0] > S.ry[ui][0]) ui = i; if (S.ry[i][0] < S.ry[li][0]) li = i; }
    const double rw = S.row_width;
    if (nq >= MAXQ) return 1;
    double (*q)[2] = Q[nq++];
    if (in.start[1] > in.end[1]) {   // the producer took the low quad: add the up quad
      q[0][0] = S.rx[ui][0] - 8; q[0][1] = S.ry[ui][0] + rw;
      q[1][0] = S.rx[ui][0] - 8; q[1][1] = S.ry[ui][0] + rw + 1;
      q[2][0] = S.rx[ui][1] + 8; q[2][1] = S.ry[ui][1] + rw + 1;
      q[3][0] = S.rx[ui][1] + 8; q[3][1] = S.ry[ui][1] + rw;
    } else {
      q[0][0] = S.rx[li][0] - 8; q[0][1] = S.ry[li][0] - rw;
      q[1][0] = S.rx[li][0] - 8; q[1][1] = S.ry[li][0] - rw - 1;
      q[2][0] = S.rx[li][1] + 8; q[2][1] = S.ry[li][1] - rw - 1;
      q[3][0] = S.rx[li][1] + 8; q[3][1] = S.ry[li][1] - rw;
    }
  }
  int keep[MAXQ], nk = 0;
  if (nq > M) {   // the M smallest gaps to the warm start's footprint (stable), in pool order
    double gap[MAXQ];
    for (int q = 0; q < nq; ++q) {
      double g = INFINITY;
      for (int k = 0; k < V.npoly; ++k) {
        double gk = INFINITY;
        for (int p = 0; p < N + nr; ++p) {
          const double* r = p < N ? traj + 5 * p : ref + 5 * (p - N);
          double px[MAXPV], py[MAXPV];
          place(V, k, r[0], r[1], r[3], px, py);
          const double v = sat_gap(px, py, V.nv[k], Q[q], 4);
          gk = v < gk ? v : gk;
        }
        g = gk < g ? gk : g;
      }
      gap[q] = g;
    }
    bool taken[MAXQ];
    for (int q = 0; q < nq; ++q) taken[q] = false;
    for (int t = 0; t < M; ++t) {
      int best = -1;
      for (int q = 0; q < nq; ++q)
        if (!taken[q] && (best < 0 || gap[q] < gap[best])) best = q;
      taken[best] = true;
    }
    for (int q = 0; q < nq; ++q) if (taken[q]) keep[nk++] = q;
  } else {
    for (int q = 0; q < nq; ++q) keep[nk++] = q;
  }
  for (int t = 0; t < M; ++t) {
    double R[4][2];
    if (t < nk) {
      for (int j = 0; j < 4; ++j) { R[j][0] = Q[keep[t]][j][0]; R[j][1] = Q[keep[t]][j][1]; }
    } else {   // far dummy quads (synth: only when the orchard has no obstacle left)
      const int k = t - nk;
      const double cx = in.start[0] + 60.0 + 5.0 * k, cy = in.start[1] + 60.0;
      R[0][0] = cx; R[0][1] = cy; R[1][0] = cx; R[1][1] = cy + 1.0;
      R[2][0] = cx + 1.0; R[2][1] = cy + 1.0; R[3][0] = cx + 1.0; R[3][1] = cy;
    }
    double Ah[2 * oge::MAXV], bh[oge::MAXV];
    if (oge::halfspaces(R, 4, Ah, bh) != 4) return 1;
    for (int j = 0; j < 4; ++j) {
      A[2 * (4 * t + j)] = Ah[2 * j];
      A[2 * (4 * t + j) + 1] = Ah[2 * j + 1];
      b[4 * t + j] = bh[j];
    }
  }
  return 0;
}

}  // namespace chain
}  // namespace htp
