// CPU baseline build of the OBCA interior-point core ("the
// build's own C++ CPU implementation of the same solver, OpenMP, one problem
// per core, on all host cores").  Same obca_core.h as the gfx950 kernel, run
// as a serial lane per OpenMP thread.  Loaded only by bench.py's cpu_baseline
// leg; the product path never calls it (there is no CPU fallback).
#include <omp.h>

#include <cstdlib>
#include <vector>

#define HTP_HD
#include "wave_ctx.h"
#include "obca_batch.h"

using namespace htp;

extern "C" int htp_cpu_threads(void) { return omp_get_max_threads(); }

// Solves problems [first, first + count) of the batch; returns 0 or < 0 on bad input.
extern "C" int htp_cpu_obca_solve_range(const htp_obca_batch* in, htp_obca_result* out, int64_t first,
                                        int64_t count, int nthreads) {
  const char* e = nullptr;
  if (check_shape(in, &e) || first < 0 || first + count > in->batch) return -1;
  Options o = default_options();
  o.wall_rate = 1e9;
  Dims D;
  make_dims(D, in->N, in->M, in->K, in->time_opt, in->obs_edges, in->body_edges);
  const Layout L = make_layout(D);
  const BatchView b{in->traj, in->obs_A, in->obs_b, in->body_G, in->body_g, in->params,
                    in->init_control, in->init_mu, in->init_lambda};
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
  {
    std::vector<double> ws((size_t)L.total);
    std::vector<double> lds(4 * NBMAX * NBMAX + 8 + 128);
    std::vector<int> ilds(2 * NBMAX);
#pragma omp for schedule(dynamic, 1)
    for (int64_t p = first; p < first + count; ++p) {
      HostLane c;
      c.lds = lds.data();
      c.ildsp = ilds.data();
      const ProblemIn pin = problem_view(b, D, p);
      ObcaSolver<HostLane, MAXE, MAXE> S(c, D, L, o, pin, ws.data());
      Result r{};
      S.run(r);
      if (out->x)
        for (int q = 0; q < D.n; ++q) out->x[(size_t)p * D.n + q] = ws[L.x + q];
      if (out->objective) out->objective[p] = r.objective;
      if (out->status) out->status[p] = r.status;
      if (out->iterations) out->iterations[p] = r.iters;
      if (out->n_factor) out->n_factor[p] = r.n_factor;
      if (out->nlp_error) out->nlp_error[p] = r.nlp_error;
      if (out->n_resto) out->n_resto[p] = r.n_resto;
    }
  }
  return 0;
}

// The point formulation (optimizer_points.py) on the host cores: the same core, FORM 1 -- the CPU baseline of
// tools/bench_points.py.
extern "C" int htp_cpu_obca_points_solve_range(const htp_obca_points_batch* in, htp_obca_result* out, int64_t first,
                                               int64_t count, int nthreads) {
  const char* e = nullptr;
  if (check_shape_points(in, &e) || first < 0 || first + count > in->batch) return -1;
  Options o = default_options();
  o.wall_rate = 1e9;
  Dims D;
  make_dims_points(D, in->N, in->M, in->n_vertices, in->obs_edges);
  const Layout L = make_layout(D);
  const BatchView b = points_view(in);
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
  {
    std::vector<double> ws((size_t)L.total);
    std::vector<double> lds(4 * NBMAX * NBMAX + 8 + 128);
    std::vector<int> ilds(2 * NBMAX);
#pragma omp for schedule(dynamic, 1)
    for (int64_t p = first; p < first + count; ++p) {
      HostLane c;
      c.lds = lds.data();
      c.ildsp = ilds.data();
      const ProblemIn pin = problem_view(b, D, p);
      ObcaSolver<HostLane, 1, MAXE, 1> S(c, D, L, o, pin, ws.data());
      Result r{};
      S.run(r);
      if (out->x)
        for (int q = 0; q < D.n; ++q) out->x[(size_t)p * D.n + q] = ws[L.x + q];
      if (out->objective) out->objective[p] = r.objective;
      if (out->status) out->status[p] = r.status;
      if (out->iterations) out->iterations[p] = r.iters;
      if (out->n_factor) out->n_factor[p] = r.n_factor;
      if (out->nlp_error) out->nlp_error[p] = r.nlp_error;
      if (out->n_resto) out->n_resto[p] = r.n_resto;
    }
  }
  return 0;
}

// Reeds-Shepp words for one pose pair on the host (rs_core.h, the same core as htp_rs_all_paths_batch).
// Used by the workload generator's fish-tail warm starts (synth.py), which run before any GPU call.
// The reference's rounding (pure-Python reeds_shepp.py): no a*b+c contraction into FMA, as the device build
// (rs_core.h's clang pragma); -march=x86-64-v3 would otherwise contract and move a sample's exact-zero pop.
#pragma GCC optimize("fp-contract=off")
#include "rs_host.h"

extern "C" int htp_cpu_rs_all_paths(const double* q, int64_t cap_paths, int64_t cap_points, int32_t* n_paths,
                                    int64_t* n_points, double* lengths, int8_t* ctypes, double* L,
                                    int64_t* point_offsets, double* x, double* y, double* yaw, double* cs,
                                    int8_t* dir) {
  return htp::rs::all_paths_host(q, cap_paths, cap_points, n_paths, n_points, lengths, ctypes, L, point_offsets, x, y,
                                 yaw, cs, dir);
}

// The planner cores' correctly rounded libm (htp_libm.h), host build: the generator's and the tests' twin of
// htp_libm_batch_device.
#include "libm_batch.h"

extern "C" int htp_cpu_libm_batch(int32_t fn, const double* x, const double* y, double* out, int64_t n) {
  if (fn < 0 || fn >= htp::hm::F_COUNT || n < 0 || (n > 0 && (!x || !out))) return -1;
  for (int64_t i = 0; i < n; ++i) out[i] = htp::hm::eval(fn, x[i], y ? y[i] : 0.0);
  return 0;
}

// The notebook chain's heuristic lowering (ychain_core.h), host build: waypoints, guide rows, lane rings and
// search lengths of one problem (tests/test_ychain_cpu.py compares it with path_planner's ReferenceLineHeuristic).
#include "ychain_core.h"

extern "C" int htp_cpu_ychain_lower(const double* rows, int32_t nrows, const double* eps, const double* start,
                                    const double* goal, double drive_row_offset, double default_len, double* wp,
                                    int32_t* n_wp, double* guide, int32_t cap_guide, int32_t* n_guide, double* rings,
                                    int32_t* n_ring, double* lengths) {
  if (nrows < 1 || nrows > htp::yc::MAXROWS) return -1;
  double w[htp::yc::MAXWP][2];
  const int n = htp::yc::waypoints(rows, nrows, eps, start, goal, drive_row_offset, w);
  if (n < 2) return 1;
  *n_wp = n;
  for (int k = 0; k < n; ++k) { wp[2 * k] = w[k][0]; wp[2 * k + 1] = w[k][1]; }
  const int m = htp::yc::guide(w, n, guide, cap_guide);
  if (m < 0) return 2;
  *n_guide = m;
  for (int k = 0; k + 1 < n; ++k) {
    double ring[htp::yc::CAPV][2];
    const int nv = htp::yc::capsule(w[k], w[k + 1], htp::yc::LANE_HALF_WIDTH, ring);
    if (nv < 3) return 3;
    n_ring[k] = nv;
    for (int j = 0; j < nv; ++j) {
      rings[(k * htp::yc::CAPV + j) * 2] = ring[j][0];
      rings[(k * htp::yc::CAPV + j) * 2 + 1] = ring[j][1];
    }
    lengths[k] = htp::yc::search_length(k, n - 1, default_len);
  }
  return 0;
}

// Hybrid A* on the host cores (hastar_core.h, the same core as htp_hastar_search_batch, fp-contract off as the
// device build): searches [first, first + count) of a batch, one search per OpenMP thread -- the CPU baseline of
// tools/bench_hastar.py.  Outputs as htp_hastar_result (path arrays may be null: no backtrack).
#include "hastar_core.h"

extern "C" int htp_cpu_hastar_range(const htp_hastar_batch* in, htp_hastar_result* out, int64_t first, int64_t count,
                                    int nthreads) {
  if (!in || !out || first < 0 || count < 0 || first + count > in->batch || in->max_nodes_cap < 0) return -1;
  using namespace htp::ha;
  if (!in->params || !in->desc || !in->poly_off || !in->vertices || !in->lane_len || !in->guide || !in->motions ||
      in->npoly < 1 || in->nvert < 1 || in->nguide < 1 || in->nmotion < 1 || in->cap_path < 0 ||
      !poly_table_ok(in->poly_off, in->npoly, in->nvert))
    return -1;
  const Pools P{in->params, in->desc, Geo{in->poly_off, in->vertices, in->lane_len, in->guide, in->motions},
                in->npoly, in->nvert, in->nguide, in->nmotion};
  if (nthreads <= 0) nthreads = omp_get_max_threads();
  const int64_t cn = 4 + (int64_t)(in->max_nodes_cap + 1) * MAXMOT + 4;
  int64_t cs = 1;
  while (cs < 2 * cn) cs <<= 1;
  const Geo g{in->poly_off, in->vertices, in->lane_len, in->guide, in->motions};
#pragma omp parallel num_threads(nthreads)
  {
    std::vector<Node> nodes((size_t)cn);
    std::vector<Slot> slots((size_t)cs);
    std::vector<double> hval((size_t)cn);
    std::vector<int32_t> hslot((size_t)cn);
    std::vector<double> dub((size_t)DUBW * (CAP_DUB + 16));
    Shared* sh = new Shared();
#pragma omp for schedule(dynamic, 1)
    for (int64_t b = first; b < first + count; ++b) {
      const double* prm = in->params + b * HTP_HA_NPARAM;
      const int32_t* d = in->desc + b * HTP_HA_NDESC;
      HostLane c;
      Work w{nodes.data(), slots.data(), hval.data(), hslot.data(), (int32_t)cn, (int32_t)cs, dub.data(), CAP_DUB};
      Out o{};
      int n_path = 0;
      if (!valid_search(P, prm, d, in->max_nodes_cap)) {   // as the device kernel: the search is not run
        o.status = ST_BAD_INPUT;
        if (out->status) out->status[b] = o.status;
        if (out->counter) out->counter[b] = 0;
        if (out->n_path) out->n_path[b] = 0;
        if (out->n_expanded) out->n_expanded[b] = 0;
        if (out->n_pose) out->n_pose[b] = 0;
        continue;
      }
      Search<HostLane> S(c, prm, d, g, w, *sh);
      S.run(o, nullptr, 0);
      if (out->x && (o.status == ST_FOUND || o.status == ST_NO_PATH || o.status == ST_MAX_NODES)) {
        const int64_t off = b * in->cap_path;
        int st = o.status;
        n_path = S.backtrack(w.hslot, w.cap_node, out->x + off, out->y + off, out->yaw + off, out->dir + off,
                             out->k + off, in->cap_path, st);
        o.status = st;
      }
      if (out->status) out->status[b] = o.status;
      if (out->counter) out->counter[b] = o.counter;
      if (out->n_path) out->n_path[b] = n_path;
      if (out->n_expanded) out->n_expanded[b] = o.n_expanded;
      if (out->n_pose) out->n_pose[b] = o.n_pose;
    }
    delete sh;
  }
  return 0;
}
