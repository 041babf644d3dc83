// Shared definitions for the batched OBCA interior-point solver.
//
// Problem layout follows R/obca_py/optimizer.py exactly (variables :292-354,
// constraints :356-425, objective :427-473); the algorithm is the IPOPT
// restatement documented in oracle/ipm.py (and DESIGN.md section 3).
#pragma once
#include <cstdint>

#ifndef HTP_HD
#error "define HTP_HD (__host__ __device__ or empty) before including htp_common.h"
#endif

// obca_core.h LocalStore: factored local blocks kept for the KKT solves (experiment, off; see there)
#ifndef HTP_STORE_LOCAL
#define HTP_STORE_LOCAL 0
#endif

// obca_core.h ObcaSolver::ubx / ubs: skip the loads of upper-bound data that is +inf / 0 for the whole solve
#ifndef HTP_UB_SKIP
#define HTP_UB_SKIP 0
#endif

namespace htp {

constexpr int NS = 5;       // state  [x, y, v, theta, steer]
constexpr int NC = 2;       // control [accel, steer_rate]
constexpr int MAXM = 16;    // obstacles per problem
constexpr int MAXK = 4;     // vehicle bodies per problem
constexpr int MAXE = 8;     // edges per polytope
constexpr int MAXKV = 16;   // point formulation: vehicle hull vertices
constexpr int NBMAX = 13;   // stage block: 5 multipliers + 5 x + 2 u + 1 tau

// per-problem scalar parameters (host packs them; see include/htp.h)
enum Param {
  P_DT = 0, P_Q00, P_Q01, P_Q10, P_Q11, P_R00, P_R01, P_R10, P_R11, P_W00, P_W11,
  P_WHEELBASE, P_MAXSTEER, P_MAXV, P_MAXACC, P_MAXSR, P_DMIN, P_XLO, P_XHI, P_YLO, P_YHI,
  P_HAS_INIT_CONTROL, P_HAS_INIT_DUAL, NPARAM = 24
};

// IPOPT option values (defaults in oracle/ipm.py OPTS)
struct Options {
  double tol, dual_inf_tol, constr_viol_tol, compl_inf_tol;
  double acceptable_tol, acceptable_constr_viol_tol, acceptable_compl_inf_tol, acceptable_dual_inf_tol;
  int acceptable_iter, max_iter, max_soc, pad0;
  double bound_relax_factor, scaling_max_gradient, scaling_min_value;
  double bound_push, bound_frac, bound_mult_init_val, constr_mult_init_max;
  double mu_init, kappa_eps, kappa_mu, theta_mu, tau_min, kappa_sigma, kappa_d, s_max;
  double gamma_theta, gamma_phi, delta, s_theta, s_phi, eta_phi, alpha_min_frac, kappa_soc;
  double dw0, dw_min, dw_max, kw_minus, kw_plus, kw_plus_bar, dc_bar, kappa_c;
  // line-search heuristics and the restoration phase (oracle/ipm.py docstring)
  double obj_max_inc, tiny_step_tol, tiny_step_y_tol, soft_resto_pderror_reduction_factor;
  double resto_penalty_parameter, resto_proximity_weight, required_infeasibility_reduction;
  double bound_mult_reset_threshold;
  int max_filter_resets, filter_reset_trigger, watchdog_shortened_iter_trigger, watchdog_trial_iter_max;
  int max_soft_resto_iters, pad1;
  // max_cpu_time (optimizer.py:475,486): seconds per problem, <= 0 = off; wall_rate = device wall-clock ticks/s
  double max_cpu_time, wall_rate;
};

inline Options default_options() {
  Options o{};
  o.tol = 1e-8; o.dual_inf_tol = 1.0; o.constr_viol_tol = 1e-4; o.compl_inf_tol = 1e-4;
  o.acceptable_tol = 1e-6; o.acceptable_constr_viol_tol = 1e-2; o.acceptable_compl_inf_tol = 1e-2;
  o.acceptable_dual_inf_tol = 1e10; o.acceptable_iter = 15; o.max_iter = 3000; o.max_soc = 4;
  o.bound_relax_factor = 1e-8; o.scaling_max_gradient = 100.0; o.scaling_min_value = 1e-8;
  o.bound_push = 1e-2; o.bound_frac = 1e-2; o.bound_mult_init_val = 1.0; o.constr_mult_init_max = 1e3;
  o.mu_init = 0.1; o.kappa_eps = 10.0; o.kappa_mu = 0.2; o.theta_mu = 1.5; o.tau_min = 0.99;
  o.kappa_sigma = 1e10; o.kappa_d = 1e-5; o.s_max = 100.0;
  o.gamma_theta = 1e-5; o.gamma_phi = 1e-8; o.delta = 1.0; o.s_theta = 1.1; o.s_phi = 2.3;
  o.eta_phi = 1e-8; o.alpha_min_frac = 0.05; o.kappa_soc = 0.99;
  o.dw0 = 1e-4; o.dw_min = 1e-20; o.dw_max = 1e40; o.kw_minus = 1.0 / 3.0; o.kw_plus = 8.0;
  o.kw_plus_bar = 100.0; o.dc_bar = 1e-8; o.kappa_c = 0.25;
  o.obj_max_inc = 5.0; o.tiny_step_tol = 10.0 * 2.220446049250313e-16; o.tiny_step_y_tol = 1e-2;
  o.soft_resto_pderror_reduction_factor = 0.9999; o.max_soft_resto_iters = 10;
  o.resto_penalty_parameter = 1000.0; o.resto_proximity_weight = 1.0; o.required_infeasibility_reduction = 0.9;
  o.bound_mult_reset_threshold = 1000.0;
  o.max_filter_resets = 5; o.filter_reset_trigger = 5; o.watchdog_shortened_iter_trigger = 10;
  o.watchdog_trial_iter_max = 3;
  o.max_cpu_time = 0.0; o.wall_rate = 1.0;
  return o;
}

// Batch-uniform problem shape (all problems of one launch share it).
struct Dims {
  int N, M, K, topt;
  int eo[MAXM], eb[MAXK], offo[MAXM], offb[MAXK];
  int TEo, TEb, mu_count, lam_count, P;
  int n, mc, md;               // variables, equality rows, inequality rows
  int oU, oMU, oLAM, oTAU, oS; // variable offsets (optimizer.py:292-354)
  int eDyn, eTerm, ePair;      // equality-row offsets
  int nb, nw;                  // stage block size (12 + topt), stage w size (7 + topt)
  int form;                    // 0: optimizer.py, 1: optimizer_points.py (point formulation)
  int KV;                      // point formulation: vehicle hull vertices (rows per block = 2 KV)
  int nblk;                    // blocks of the stage chain (N, or N + 1 with a hard terminal block)
};

// Offsets (in doubles) of the per-problem workspace arrays.
struct Layout {
  int64_t x, xL, xU, zL, zU, gf, dx, xt, rx, sx, dzL, dzU;   // n
  int64_t s, dL, dU, vL, vU, d, ds, st, dt, yd, scI, dyd, rs, rd, dsoc, ss, syd, dvL, dvU;  // md
  int64_t yc, c, scE, dyc, rc, ct, csoc, syc;                 // mc
  int64_t pairS, pairR;                                      // 6P, 3P
  int64_t Kst, Off, LD, fac, V, X;                           // stage storage
  int64_t ipiv;                                              // ints stored as double
  // restoration phase: n/p variables R = [n_c | p_c | n_d | p_d] (nR = 2 mc + 2 md), their trial values,
  // steps, bound multipliers and multiplier steps; per-row diagonal eR (mc + md) of the eliminated n/p;
  // folded constraint right-hand sides; the reference point x_R and D_R = 1/max(1,|x_R|) (n)
  int64_t R, Rt, dR, zR, dzR, eR, rcf, rdf, xR, dr, rRx;
  // the original iterate while the restoration phase runs; the original filter (2 FMAX); saved scalars
  int64_t ox, os, oyc, oyd, ozL, ozU, ovL, ovU, ofilt, osv;
  // watchdog reference point and direction (x, s, y, z, v, R, zR, c, d, step)
  int64_t wx, ws, wyc, wyd, wzL, wzU, wvL, wvU, wR, wzR, wc, wd, wdx, wds, wdyc, wdyd, wdR;
  int64_t ax;                                                // last acceptable iterate (x)
  int64_t plist;                                             // compacted block indices (local sweeps, pass 2)
  int64_t lfac;                                              // factored local blocks (LocalStore, P records)
  int64_t total;
};

// Everything a launch needs that is uniform over the batch (lives in
// constant memory on the device; scalar-cached).
struct Shape {
  Dims D;
  Layout L;
  Options o;
};

struct Result {            // per problem
  int32_t status, iters, n_factor, n_resto;
  double objective, final_mu, nlp_error, sf;
  int64_t cyc[8];          // shader cycles: local sweeps, assembly, stage chain, kkt solves, total,
                           // errors+grad_lag, line search, update+re-eval
};

enum Status { ST_SUCCESS = 0, ST_ACCEPTABLE = 1, ST_MAXITER = 2, ST_RESTORATION = 3, ST_STEPFAIL = 4,
              ST_BADINPUT = 5, ST_CPUTIME = 6, ST_INFEASIBLE = 7, ST_TINYSTEP = 8 };

HTP_HD inline void make_dims(Dims& d, int N, int M, int K, int topt, const int* eo, const int* eb) {
  d.N = N; d.M = M; d.K = K; d.topt = topt ? 1 : 0;
  d.TEo = 0; d.TEb = 0;
  for (int m = 0; m < M; ++m) { d.eo[m] = eo[m]; d.offo[m] = d.TEo; d.TEo += eo[m]; }
  for (int k = 0; k < K; ++k) { d.eb[k] = eb[k]; d.offb[k] = d.TEb; d.TEb += eb[k]; }
  d.mu_count = d.TEb * M;
  d.lam_count = d.TEo * K;
  d.P = N * M * K;
  d.oU = NS * N;
  d.oMU = d.oU + NC * (N - 1);
  d.oLAM = d.oMU + N * d.mu_count;
  d.oTAU = d.oLAM + N * d.lam_count;
  d.oS = d.oTAU + (d.topt ? N - 1 : 0);
  d.n = d.oS + NS;
  d.eDyn = NS;
  d.eTerm = NS + NS * (N - 1);
  d.ePair = d.eTerm + NS;
  d.mc = d.ePair + 2 * d.P;
  d.md = 2 * d.P;
  d.nw = 7 + d.topt;
  d.nb = NS + d.nw;
  d.form = 0;
  d.KV = 0;
  d.nblk = N;
}

// Point formulation (R/obca_py/optimizer_points.py): X (5N), U (2(N-1)), LAMBDA
// obstacle-major (N * sum_{j'<j} e_j' + i * e_j, :223-255); no mu, tau or terminal
// slack; equality rows X0, dynamics, X_{N-1} = end (hard, :264-278); per block
// (obstacle j, step i) 2 KV inequality rows [||A'lam||^2, (A(R v_k + t) - b).lam]
// for each hull vertex k (:282-327).  The vertices travel in the body_G slot
// (eb[0] = KV); the stage chain gets one extra block for the terminal rows.
HTP_HD inline void make_dims_points(Dims& d, int N, int M, int KV, const int* eo) {
  const int kv[1] = {KV};
  make_dims(d, N, M, 1, 0, eo, kv);
  d.form = 1;
  d.KV = KV;
  d.mu_count = 0;
  d.lam_count = d.TEo;
  d.P = N * M;
  d.oMU = d.oU + NC * (N - 1);
  d.oLAM = d.oMU;
  d.oTAU = d.oLAM + N * d.TEo;
  d.oS = d.oTAU;
  d.n = d.oS;
  d.mc = d.ePair;
  d.md = 2 * KV * d.P;
  d.nblk = N + 1;
}

inline Layout make_layout(const Dims& d) {
  Layout L{};
  int64_t o = 0;
  auto take = [&](int64_t cnt) { int64_t r = o; o += (cnt + 7) & ~int64_t(7); return r; };
  L.x = take(d.n); L.xL = take(d.n); L.xU = take(d.n); L.zL = take(d.n); L.zU = take(d.n);
  L.gf = take(d.n); L.dx = take(d.n); L.xt = take(d.n); L.rx = take(d.n); L.sx = take(d.n);
  L.dzL = take(d.n); L.dzU = take(d.n);
  L.s = take(d.md); L.dL = take(d.md); L.dU = take(d.md); L.vL = take(d.md); L.vU = take(d.md);
  L.d = take(d.md); L.ds = take(d.md); L.st = take(d.md); L.dt = take(d.md); L.yd = take(d.md);
  L.scI = take(d.md); L.dyd = take(d.md); L.rs = take(d.md); L.rd = take(d.md); L.dsoc = take(d.md);
  L.ss = take(d.md); L.syd = take(d.md); L.dvL = take(d.md); L.dvU = take(d.md);
  L.yc = take(d.mc); L.c = take(d.mc); L.scE = take(d.mc); L.dyc = take(d.mc); L.rc = take(d.mc);
  L.ct = take(d.mc); L.csoc = take(d.mc); L.syc = take(d.mc);
  L.pairS = take(6 * (int64_t)d.P); L.pairR = take(3 * (int64_t)d.P);
  const int64_t nb2 = (int64_t)d.nb * d.nb;
  L.Kst = take(d.nblk * nb2); L.Off = take(d.nblk * nb2); L.LD = take(d.nblk * nb2); L.fac = take(d.nblk * nb2);
  L.V = take((int64_t)d.nblk * d.nb); L.X = take((int64_t)d.nblk * d.nb); L.ipiv = take((int64_t)d.nblk * d.nb);
  const int64_t nR = 2 * (int64_t)d.mc + 2 * (int64_t)d.md, mcd = (int64_t)d.mc + d.md;
  L.R = take(nR); L.Rt = take(nR); L.dR = take(nR); L.zR = take(nR); L.dzR = take(nR); L.eR = take(mcd);
  L.rcf = take(d.mc); L.rdf = take(d.md); L.xR = take(d.n); L.dr = take(d.n); L.rRx = take(nR);
  L.ox = take(d.n); L.os = take(d.md); L.oyc = take(d.mc); L.oyd = take(d.md); L.ozL = take(d.n); L.ozU = take(d.n);
  L.ovL = take(d.md); L.ovU = take(d.md); L.ofilt = take(2 * 64); L.osv = take(64);
  L.wx = take(d.n); L.ws = take(d.md); L.wyc = take(d.mc); L.wyd = take(d.md); L.wzL = take(d.n); L.wzU = take(d.n);
  L.wvL = take(d.md); L.wvU = take(d.md); L.wR = take(nR); L.wzR = take(nR); L.wc = take(d.mc); L.wd = take(d.md);
  L.wdx = take(d.n); L.wds = take(d.md); L.wdyc = take(d.mc); L.wdyd = take(d.md); L.wdR = take(nR);
  L.ax = take(d.n);
  L.plist = take(d.P);
  // LocalStore<MAXE, MAXE>::COUNT fields per local block (the widest kernel instance; obca_core.h)
  constexpr int64_t LF_MAX = (2 * MAXE + 2) * (2 * MAXE + 3) / 2 + 3 * (2 * MAXE + 2) + 2 * (2 * MAXE) + 2 + 4 + 1;
  L.lfac = take(HTP_STORE_LOCAL && d.form == 0 ? LF_MAX * d.P : 0);
  L.total = o;
  return L;
}

}  // namespace htp
