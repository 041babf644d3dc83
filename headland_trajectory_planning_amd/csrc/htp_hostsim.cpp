// TEST-ONLY host build of the solver core (serial single-lane context).
// Used by tests/ to debug the kernel logic against the oracle in a container
// without a GPU.  The product never loads this library (no CPU fallback).
#include <cstdlib>
#include <vector>

#define HTP_HD
#include "wave_ctx.h"
#include "obca_batch.h"

using namespace htp;

extern "C" int htp_hostsim_obca_solve(const htp_obca_batch* in, htp_obca_result* out, const char** names,
                                      const double* values, int nopt) {
  const char* e = nullptr;
  if (check_shape(in, &e)) return -1;
  Options o = default_options();
  o.wall_rate = 1e9;
  for (int k = 0; k < nopt; ++k)
    if (set_option(o, names[k], values[k])) return -2;
  Dims D;
  make_dims(D, in->N, in->M, in->K, in->time_opt, in->obs_edges, in->body_edges);
  Layout L = make_layout(D);
  std::vector<double> ws((size_t)L.total);
  std::vector<double> lds(4 * NBMAX * NBMAX + 8 + 128);
  std::vector<int> ilds(2 * NBMAX);
  BatchView b{in->traj, in->obs_A, in->obs_b, in->body_G, in->body_g, in->params,
              in->init_control, in->init_mu, in->init_lambda};
  for (int p = 0; p < in->batch; ++p) {
    HostLane c;
    c.lds = lds.data();
    c.ildsp = ilds.data();
    ProblemIn pin = problem_view(b, D, p);
    ObcaSolver<HostLane, MAXE, MAXE> S(c, D, L, o, pin, ws.data());
    Result r{};
    S.run(r);
    for (int q = 0; q < D.n; ++q) out->x[(size_t)p * D.n + q] = ws[L.x + q];
    if (out->objective) out->objective[p] = r.objective;
    if (out->status) out->status[p] = r.status;
    if (out->iterations) out->iterations[p] = r.iters;
    if (out->n_factor) out->n_factor[p] = r.n_factor;
    if (out->nlp_error) out->nlp_error[p] = r.nlp_error;
      if (out->n_resto) out->n_resto[p] = r.n_resto;
  }
  return 0;
}

// debug: initialize problem 0, optionally factor once (mode: 0 none, 1 normal with dw, 2 LS),
// copy the workspace out; returns sf.
extern "C" double htp_hostsim_debug_ws(const htp_obca_batch* in, int mode, double dw, double* ws_out,
                                       int64_t ws_len, int* neg_out) {
  Options o = default_options();
  o.wall_rate = 1e9;
  Dims D;
  make_dims(D, in->N, in->M, in->K, in->time_opt, in->obs_edges, in->body_edges);
  Layout L = make_layout(D);
  std::vector<double> ws((size_t)L.total);
  std::vector<double> lds(4 * NBMAX * NBMAX + 8 + 128);
  std::vector<int> ilds(2 * NBMAX);
  BatchView b{in->traj, in->obs_A, in->obs_b, in->body_G, in->body_g, in->params,
              in->init_control, in->init_mu, in->init_lambda};
  HostLane c;
  c.lds = lds.data();
  c.ildsp = ilds.data();
  ProblemIn pin = problem_view(b, D, 0);
  ObcaSolver<HostLane, MAXE, MAXE> S(c, D, L, o, pin, ws.data());
  S.initialize();
  int neg = 0, zero = 0;
  if (mode == 1) S.factorize(false, dw, 0.0, neg, zero);
  if (mode == 2) S.factorize(true, 0.0, 0.0, neg, zero);
  if (neg_out) { neg_out[0] = neg; neg_out[1] = zero; }
  for (int64_t q = 0; q < ws_len && q < L.total; ++q) ws_out[q] = ws[q];
  return S.sf;
}

// point formulation (optimizer_points.py), serial host build
extern "C" int htp_hostsim_obca_points_solve(const htp_obca_points_batch* in, htp_obca_result* out,
                                             const char** names, const double* values, int nopt) {
  const char* e = nullptr;
  if (check_shape_points(in, &e)) return -1;
  Options o = default_options();
  o.wall_rate = 1e9;
  for (int k = 0; k < nopt; ++k)
    if (set_option(o, names[k], values[k])) return -2;
  Dims D;
  make_dims_points(D, in->N, in->M, in->n_vertices, in->obs_edges);
  Layout L = make_layout(D);
  std::vector<double> ws((size_t)L.total);
  std::vector<double> lds(4 * NBMAX * NBMAX + 8 + 128);
  std::vector<int> ilds(2 * NBMAX);
  BatchView b = points_view(in);
  for (int p = 0; p < in->batch; ++p) {
    HostLane c;
    c.lds = lds.data();
    c.ildsp = ilds.data();
    ProblemIn pin = problem_view(b, D, p);
    ObcaSolver<HostLane, 1, MAXE, 1> S(c, D, L, o, pin, ws.data());
    Result r{};
    S.run(r);
    for (int q = 0; q < D.n; ++q) out->x[(size_t)p * D.n + q] = ws[L.x + q];
    if (out->objective) out->objective[p] = r.objective;
    if (out->status) out->status[p] = r.status;
    if (out->iterations) out->iterations[p] = r.iters;
    if (out->n_factor) out->n_factor[p] = r.n_factor;
    if (out->nlp_error) out->nlp_error[p] = r.nlp_error;
      if (out->n_resto) out->n_resto[p] = r.n_resto;
  }
  return 0;
}
