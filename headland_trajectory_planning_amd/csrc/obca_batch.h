// Batch <-> per-problem views and option plumbing shared by the HIP library
// and the test-only host build.
#pragma once
#include <cstring>

#include "../../include/htp.h"
#include "htp_common.h"
#include "obca_core.h"

namespace htp {

struct BatchView {  // plain copy of htp_obca_batch pointers (device or host)
  const double *traj, *obsA, *obsb, *bodyG, *bodyg, *params, *init_u, *init_mu, *init_la;
};

template <class DD>
HTP_HD inline ProblemIn problem_view(const BatchView& b, DD& D, int64_t p) {
  ProblemIn in;
  in.traj = b.traj + p * D.N * NS;
  in.obsA = b.obsA + p * D.TEo * 2;
  in.obsb = b.obsb + p * D.TEo;
  in.bodyG = b.bodyG + p * D.TEb * 2;
  in.bodyg = b.bodyg + p * D.TEb;
  in.par = b.params + p * NPARAM;
  in.init_u = b.init_u ? b.init_u + p * (D.N - 1) * NC : nullptr;
  in.init_mu = b.init_mu ? b.init_mu + p * (int64_t)D.N * D.mu_count : nullptr;
  in.init_la = b.init_la ? b.init_la + p * (int64_t)D.N * D.lam_count : nullptr;
  return in;
}

inline int check_shape(const htp_obca_batch* in, const char** err) {
  if (in->batch < 0) { *err = "[OBCA] batch must be >= 0"; return -1; }
  if (in->N < 2) { *err = "[OBCA] N must be >= 2"; return -1; }
  if (in->M < 1 || in->M > MAXM) { *err = "[OBCA] M must be in [1, 16]"; return -1; }
  if (in->K < 1 || in->K > MAXK) { *err = "[OBCA] K must be in [1, 4]"; return -1; }
  for (int m = 0; m < in->M; ++m)
    if (in->obs_edges[m] < 3 || in->obs_edges[m] > MAXE) { *err = "[OBCA] obstacle edges must be in [3, 8]"; return -1; }
  for (int k = 0; k < in->K; ++k)
    if (in->body_edges[k] < 3 || in->body_edges[k] > MAXE) { *err = "[OBCA] body edges must be in [3, 8]"; return -1; }
  return 0;
}

inline int check_shape_points(const htp_obca_points_batch* in, const char** err) {
  if (in->batch < 0) { *err = "[OBCA points] batch must be >= 0"; return -1; }
  if (in->N < 2) { *err = "[OBCA points] N must be >= 2"; return -1; }
  if (in->M < 1 || in->M > MAXM) { *err = "[OBCA points] M must be in [1, 16]"; return -1; }
  if (in->n_vertices < 3 || in->n_vertices > MAXKV) { *err = "[OBCA points] n_vertices must be in [3, 16]"; return -1; }
  for (int m = 0; m < in->M; ++m)
    if (in->obs_edges[m] < 3 || in->obs_edges[m] > MAXE) { *err = "[OBCA points] obstacle edges must be in [3, 8]"; return -1; }
  return 0;
}

// point formulation: vertices ride in the body_G slot (Dims::eb[0] = KV)
inline BatchView points_view(const htp_obca_points_batch* in) {
  return BatchView{in->traj, in->obs_A, in->obs_b, in->vertices, in->vertices, in->params,
                   in->init_control, nullptr, nullptr};
}

inline int set_option(Options& o, const char* name, double v) {
#define HTP_OPT(f) if (!std::strcmp(name, #f)) { o.f = (decltype(o.f))v; return 0; }
  HTP_OPT(tol) HTP_OPT(dual_inf_tol) HTP_OPT(constr_viol_tol) HTP_OPT(compl_inf_tol)
  HTP_OPT(acceptable_tol) HTP_OPT(acceptable_constr_viol_tol) HTP_OPT(acceptable_compl_inf_tol)
  HTP_OPT(acceptable_dual_inf_tol) HTP_OPT(acceptable_iter) HTP_OPT(max_iter) HTP_OPT(max_soc)
  HTP_OPT(bound_relax_factor) HTP_OPT(scaling_max_gradient) HTP_OPT(scaling_min_value)
  HTP_OPT(bound_push) HTP_OPT(bound_frac) HTP_OPT(bound_mult_init_val) HTP_OPT(constr_mult_init_max)
  HTP_OPT(mu_init) HTP_OPT(kappa_eps) HTP_OPT(kappa_mu) HTP_OPT(theta_mu) HTP_OPT(tau_min)
  HTP_OPT(kappa_sigma) HTP_OPT(kappa_d) HTP_OPT(s_max) HTP_OPT(gamma_theta) HTP_OPT(gamma_phi)
  HTP_OPT(delta) HTP_OPT(s_theta) HTP_OPT(s_phi) HTP_OPT(eta_phi) HTP_OPT(alpha_min_frac) HTP_OPT(kappa_soc)
  HTP_OPT(dw0) HTP_OPT(dw_min) HTP_OPT(dw_max) HTP_OPT(kw_minus) HTP_OPT(kw_plus) HTP_OPT(kw_plus_bar)
  HTP_OPT(dc_bar) HTP_OPT(kappa_c)
  HTP_OPT(obj_max_inc) HTP_OPT(tiny_step_tol) HTP_OPT(tiny_step_y_tol) HTP_OPT(soft_resto_pderror_reduction_factor)
  HTP_OPT(resto_penalty_parameter) HTP_OPT(resto_proximity_weight) HTP_OPT(required_infeasibility_reduction)
  HTP_OPT(bound_mult_reset_threshold) HTP_OPT(max_filter_resets) HTP_OPT(filter_reset_trigger)
  HTP_OPT(watchdog_shortened_iter_trigger) HTP_OPT(watchdog_trial_iter_max) HTP_OPT(max_soft_resto_iters)
  HTP_OPT(max_cpu_time)
#undef HTP_OPT
  return -1;
}

}  // namespace htp
