// Batched OBCA interior-point solver core: one problem per wavefront.
//
// NLP: R/obca_py/optimizer.py (variables :292-354, constraints :356-425,
// objective :427-473, dynamics :9-36 / :364-377).  Algorithm: the IPOPT 3.14
// default path restated in oracle/ipm.py (that file lists every constant).
// Linear algebra: structure-exploiting Schur eliminations of DESIGN.md s.3
// (same order as oracle/structured.py):
//   inequality slacks/multipliers -> per-(stage,obstacle,body) local blocks
//   -> terminal slack block -> block-tridiagonal stage LDL^T (Bunch-Kaufman
//   per 13x13 block), giving the exact inertia by Sylvester's law.
//
// Parallel model: every "for (q = c.lane; q < n; q += c.width)" loop is a
// lane-parallel sweep with independent iterations; c.sync() separates
// sweeps; c.sum()/maxv() are wave reductions.  All control flow outside the
// sweeps is wave-uniform.
#pragma once
#include <cmath>
#include <type_traits>

#include "htp_common.h"
#include "htp_fastm.h"
#include "htp_libm.h"

// The solver's transcendental functions.  With HTP_SOLVER_DETLIBM (default) the same doubles on the device and on
// every host build, so the device solve is reproduced on the host bit for bit (emu_wave.h,
// tests/test_gpu_emulation.py): the hot ones (dynamics sin / cos / tan, the barrier's log) from htp_fastm.h
// (explicit FMA, <= 2 ulp), IPOPT's few pow updates per iteration correctly rounded (htp_libm.h).  0 takes the
// platform's (ocml on the device).
#ifndef HTP_SOLVER_DETLIBM
#define HTP_SOLVER_DETLIBM 1
#endif
namespace htp {
namespace sm {
#if HTP_SOLVER_DETLIBM
using fm::cos;
using fm::log;
using fm::sin;
using fm::sincos;
using fm::tan;
using hm::pow;
#if HTP_LOG10_PLATFORM
HTP_HD inline double log10(double x) { return ::log10(x); }
#else
HTP_HD inline double log10(double x) { return fm::log(x) * 0.43429448190325182765; }   // the obj_max_inc test
#endif
#else
HTP_HD inline double sin(double x) { return ::sin(x); }
HTP_HD inline double cos(double x) { return ::cos(x); }
HTP_HD inline double tan(double x) { return ::tan(x); }
HTP_HD inline double log(double x) { return ::log(x); }
HTP_HD inline double pow(double x, double y) { return ::pow(x, y); }
HTP_HD inline double log10(double x) { return ::log10(x); }
HTP_HD inline void sincos(double x, double& s, double& c) {
#if defined(__HIP_DEVICE_COMPILE__)
  ::sincos(x, &s, &c);
#else
  s = ::sin(x);
  c = ::cos(x);
#endif
}
#endif
}  // namespace sm
}  // namespace htp

// Contraction: a * b + c fused exactly where the source writes it within one expression (clang's llvm.fmuladd),
// never across statements -- the same fused operations in the device build and in the clang host emulation
// (emu_wave.h).  htp_libm.h above leaves contract(off) in effect; this restores it for the solver.
#if defined(__clang__)
#pragma clang fp contract(on)
#endif

#include "dyn_gen.h"
#ifdef HTP_TRACE_ON
#include <cstdio>
#endif

#ifndef HTP_UNROLL_N
#define HTP_UNROLL_N 4
#endif
// loads in flight per lane in sweep(): 8 and 12 give the fewest cycles per iteration, 4 is 4 % and 2 is 14 % slower,
// 16 is slower again (profiles/r03t_ab_sweep_unroll.txt, r03u_ab_sweep_unroll.txt; results bit-identical)
// Riccati factor: stop at the first non-positive-definite pivot (the inertia is then decided; 1) or run every stage
// (0, the round-3 kernel) -- bit-identical results, fewer cycles in inertia-correction trials
// Riccati factor: stage records staged through LDS HTP_FAC_SB stages at a time (0: one stage of register prefetch,
// the round-4 kernel; bit-identical either way)
// The Newton step's Riccati backward solve pass run inside the Riccati factor (1; exact dynamics only): the
// backward recursion of the solve needs P_{i+1}, F_i and K_i, which the factor has at stage i, so its MFMAs
// ride along with the factor's chain instead of a second pass over the stage records.  Same operands and the
// same operation order as riccati_solve_mfma_t's backward pass: bit-identical.  0: a separate pass (round 5).
// Round 6 A/B (config D 4 096, profiles/r06r_ab_D.txt): 3.45 M -> 3.36 M wave-cycles per problem-iteration.
#ifndef HTP_BWD_FUSE
#define HTP_BWD_FUSE 1
#endif
// Stage-chain loops with their invariants (workspace bases, sizes, the lane index, the relaxation flag) held in
// locals set before the loop (1), or re-read inside it (0, round 5).  The solver object's address escapes into
// the out-of-line phases, so after every wavefront fence each such read went back to memory through a pointer
// chain -- and on gfx950 a load waits for every earlier store (one in-order vmcnt counter), so a re-read right
// after a stage's stores cost the stores' full completion latency.  Values unchanged.
#ifndef HTP_HOIST
#define HTP_HOIST 1
#endif
// local sweeps: the trip loops' bound and lane index read once before the loop (1), or in every trip (0, round 5;
// each re-read is a pointer chain from the solver object issued behind the previous trip's stores)
#ifndef HTP_HOIST_TRIP
#define HTP_HOIST_TRIP 1
#endif
// pivoted local blocks: the right-hand side of each Bunch-Kaufman solve in LDS (1) or in registers via select chains
// (0, round 5)
#ifndef HTP_PIV_V_LDS
#define HTP_PIV_V_LDS 1
#endif
// Riccati forward solve pass: Rt_i^-1 rt_i for a ring block's stages solved up front, one lane per stage (1), or
// on the chain in each stage (0, round 5)
#ifndef HTP_KV_HOIST
#define HTP_KV_HOIST 1
#endif
// Riccati factor record loads without per-lane branches (1) or as conditional loads (0, round 5)
#ifndef HTP_FILL_SEL
#define HTP_FILL_SEL 1
#endif
#ifndef HTP_FAC_SB
#define HTP_FAC_SB 4
#endif
#ifndef HTP_RIC_EARLY_EXIT
#define HTP_RIC_EARLY_EXIT 1
#endif
// factor_ic's inertia scan (see ObcaSolver::ic_scan): 1 on, 0 off (every trial factorization run in full)
// NaN steps and trial values are evaluation errors (never accepted, never a tiny step): 1; 0 = round-3 behaviour
#ifndef HTP_NAN_GUARD
#define HTP_NAN_GUARD 1
#endif
#ifndef HTP_FUSE_RHS
#define HTP_FUSE_RHS 1
#endif
#ifndef HTP_IC_SCAN
#define HTP_IC_SCAN 1
#endif
#ifndef HTP_SWEEP_U
#define HTP_SWEEP_U 8
#endif
#define HTP_PRAGMA_(x) _Pragma(#x)
#define HTP_PRAGMA(x) HTP_PRAGMA_(x)
#define HTP_UNROLL HTP_PRAGMA(unroll HTP_UNROLL_N)
#ifndef HTP_FI
#define HTP_FI __attribute__((always_inline))
#endif
// IPM phases called from several sites (factorize, kkt_solve, line-search trial,
// constraint / barrier / error evaluations): one out-of-line copy each keeps the
// kernel's instruction footprint small (instruction-cache misses were a large
// share of the per-iteration latency); helpers stay force-inlined.
#ifdef HTP_OUTLINE_PHASES
#define HTP_PHASE __attribute__((noinline))
#else
#define HTP_PHASE HTP_FI
#endif
// The barrier function (a log per bounded variable and slack, 8 loads per lane in flight) is evaluated at the
// current point and at each line-search trial point from three sites; one out-of-line copy instead of three
// inlined ones removes a sixth of the kernel's instructions (tools/code_size.py).
// Cold IPM phases (watchdog, soft restoration, restoration entry / exit, pivoted local blocks on the serial
// path): out of line (the default) or force-inlined (HTP_COLD_INLINE, experiments).  Out of line, the solver
// object's address escapes into them.
#ifdef HTP_COLD_INLINE
#define HTP_COLD HTP_FI
#else
#define HTP_COLD __attribute__((noinline))
#endif
#ifndef HTP_BARRIER_INLINE
#define HTP_BARRIER_ATTR __attribute__((noinline))
#else
#define HTP_BARRIER_ATTR HTP_FI
#endif

#ifndef HTP_RELAX_RICCATI
#define HTP_RELAX_RICCATI 1   // 0: experiments only -- relaxed systems take the block LDL^T path (round 2)
#endif
#ifndef HTP_PT_RICCATI
#define HTP_PT_RICCATI 1      // 0: experiments only -- the point formulation takes the block LDL^T path
#endif
// FORM 0 with the relaxed-dynamics Riccati (HTP_RELAX_RICCATI) never takes the block LDL^T path, so its stage
// assembly stores only what the Riccati records read (the w x w Hessian block, the jerk cross terms, J_i).
#define HTP_COMPACT_STAGE HTP_RELAX_RICCATI

namespace htp {

struct ProblemIn {
  const double* traj;    // N x 5
  const double* obsA;    // TEo x 2
  const double* obsb;    // TEo
  const double* bodyG;   // TEb x 2
  const double* bodyg;   // TEb
  const double* par;     // NPARAM
  const double* init_u;  // (N-1) x 2 or null
  const double* init_mu; // N x mu_count or null
  const double* init_la; // N x lam_count or null
};

HTP_HD HTP_FI inline double sq(double a) { return a * a; }
HTP_HD inline bool finite_(double a) { return a > -1e300 && a < 1e300; }
HTP_HD inline double dmax(double a, double b) { return a > b ? a : b; }
HTP_HD inline double nmax(double a, double b) { return (b > a || b != b) ? b : a; }   // NaN-sticky max
HTP_HD inline double dmin(double a, double b) { return a < b ? a : b; }
HTP_HD inline double dabs(double a) { return a < 0 ? -a : a; }

constexpr double HTP_INF = __builtin_huge_val();

#ifdef HTP_TRACE_ON
#define HTP_TRACE(...) do { if (c.lane == 0) printf(__VA_ARGS__); } while (0)
#else
#define HTP_TRACE(...) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// Local (stage, obstacle m, body n) block:  z = [mu_mn (EN), lam_mn (EM)],
// rows c2a, c2b (equality), coupled to p = (x_i, y_i, theta_i).
// Inequality rows c1 (||A'lam||^2 in [0,1]) and c3 (distance >= dmin) are
// already eliminated (Hbar = W + Sigma + dw + Jd' E^-1 Jd).
// ---------------------------------------------------------------------------
template <int EN, int EM>
struct LocalBlock {
  static constexpr int NZ = EN + EM;
  static constexpr int NL = NZ + 2;
  static constexpr int NPK = NL * (NL + 1) / 2;
  double K[NPK];       // packed lower; becomes L (unit, strict lower) + D (diag)
  double B[NL][3];     // coupling to p = (x, y, theta)
  double Hpp[6];       // direct p-p terms: xx xy yy xt yt tt
  double J1[NZ], J3z[NZ], J3p[2];
  double E1, E3, Ds1, Ds3;
  int neg, zero;

  HTP_HD HTP_FI static int pk(int r, int c) { return r * (r + 1) / 2 + c; }

  bool piv;            // Bunch-Kaufman would interchange: use the pivoted path

  // Unpivoted LDL^T of K (inertia = signs of D), in place.  With H_zz
  // positive definite (every multiplier pivot > 0) this is a Cholesky of H_zz
  // followed by one of the negative definite 2x2 Schur complement: stable.
  // The reduced Hessian may however be indefinite on the multiplier block
  // itself (only its restriction to null(C_z) must be positive); a
  // non-positive multiplier pivot sets `piv` and the block is redone by
  // ObcaSolver::local_pivoted (Bunch-Kaufman with interchanges, exact
  // inertia, stable solves).  The common case keeps this small,
  // register-resident code.
  HTP_HD HTP_FI void factor() {
    neg = 0;
    zero = 0;
    piv = false;
    for (int k = 0; k < NL; ++k) {
      double dk = K[pk(k, k)];
      for (int j = 0; j < k; ++j) dk -= K[pk(k, j)] * K[pk(k, j)] * K[pk(j, j)];
      for (int r = k + 1; r < NL; ++r) {
        double v = K[pk(r, k)];
        for (int j = 0; j < k; ++j) v -= K[pk(r, j)] * K[pk(k, j)] * K[pk(j, j)];
        K[pk(r, k)] = v;
      }
      if (k < NZ && !(dk > 0.0)) piv = true;
      if (dk == 0.0) { zero = 1; dk = 1.0; }
      if (dk < 0.0) ++neg;
      K[pk(k, k)] = dk;
      const double idk = 1.0 / dk;  // one division per pivot, the column is scaled by multiplication
      for (int r = k + 1; r < NL; ++r) K[pk(r, k)] = K[pk(r, k)] * idk;
    }
  }
  // W = L^-1 v (unit lower forward substitution only), in place
  HTP_HD HTP_FI void forward(double* v) const {
    for (int k = 0; k < NL; ++k)
      for (int j = 0; j < k; ++j) v[k] -= K[pk(k, j)] * v[j];
  }
  HTP_HD HTP_FI void solve(double* v) const {  // in place K^-1 v
    for (int k = 0; k < NL; ++k)
      for (int j = 0; j < k; ++j) v[k] -= K[pk(k, j)] * v[j];
    for (int k = 0; k < NL; ++k) v[k] /= K[pk(k, k)];
    for (int k = NL - 1; k >= 0; --k)
      for (int r = k + 1; r < NL; ++r) v[k] -= K[pk(r, k)] * v[r];
  }
};

// Factored local blocks kept for the KKT solves (HTP_STORE_LOCAL, experiment, off): the factor sweep stores every
// unpivoted block's LDL^T factor and the rows the solves read, structure-of-arrays (field f of block p at f * P + p);
// the right-hand-side and back sweeps load them instead of rebuilding and refactoring each block.  The same doubles
// either way, but 107 extra doubles per block written and read twice per iteration cost more than the VALU they
// save: 23 % more cycles per IPM iteration on config D (profiles/r04c_ab_D.txt, base vs sl0).
template <int EN, int EM>
struct LocalStore {
  static constexpr int NZ = EN + EM, NL = NZ + 2, NPK = NL * (NL + 1) / 2;
  static constexpr int F_K = 0, F_B = NPK, F_J1 = F_B + 3 * NL, F_J3Z = F_J1 + NZ, F_J3P = F_J3Z + NZ;
  static constexpr int F_E1 = F_J3P + 2, F_E3 = F_E1 + 1, F_DS1 = F_E3 + 1, F_DS3 = F_DS1 + 1, F_PIV = F_DS3 + 1;
  static constexpr int COUNT = F_PIV + 1;
};

// ---------------------------------------------------------------------------
// Point-formulation local block (R/obca_py/optimizer_points.py:282-327):
// z = lam_ji (EM) of obstacle j at step i, no equality rows; its 2 KV
// inequality rows (||A'lam||^2 in [0,1], (A(R v_k + t) - b).lam in
// [dmin, 1e5] for every hull vertex k) are eliminated, leaving
// Hbar_zz (+ coupling to p = (x, y, theta)).  IPOPT's inertia needs Hbar_zz
// positive definite: a non-positive pivot sets `piv` and the exact counts
// come from the Bunch-Kaufman path.
// ---------------------------------------------------------------------------
template <int EM>
struct PtBlock {
  static constexpr int NZ = EM;
  static constexpr int NL = EM;
  static constexpr int NPK = NZ * (NZ + 1) / 2;
  double K[NPK];
  double B[NZ][3];
  double Hpp[6];
  int neg, zero;
  bool piv;

  HTP_HD HTP_FI static int pk(int r, int c) { return r * (r + 1) / 2 + c; }
  HTP_HD HTP_FI void factor() {
    neg = 0;
    zero = 0;
    piv = false;
    for (int k = 0; k < NL; ++k) {
      double dk = K[pk(k, k)];
      for (int j = 0; j < k; ++j) dk -= K[pk(k, j)] * K[pk(k, j)] * K[pk(j, j)];
      for (int r = k + 1; r < NL; ++r) {
        double v = K[pk(r, k)];
        for (int j = 0; j < k; ++j) v -= K[pk(r, j)] * K[pk(k, j)] * K[pk(j, j)];
        K[pk(r, k)] = v;
      }
      if (!(dk > 0.0)) piv = true;
      if (dk == 0.0) { zero = 1; dk = 1.0; }
      if (dk < 0.0) ++neg;
      K[pk(k, k)] = dk;
      for (int r = k + 1; r < NL; ++r) K[pk(r, k)] = K[pk(r, k)] / dk;
    }
  }
  HTP_HD HTP_FI void solve(double* v) const {
    for (int k = 0; k < NL; ++k)
      for (int j = 0; j < k; ++j) v[k] -= K[pk(k, j)] * v[j];
    for (int k = 0; k < NL; ++k) v[k] /= K[pk(k, k)];
    for (int k = NL - 1; k >= 0; --k)
      for (int r = k + 1; r < NL; ++r) v[k] -= K[pk(r, k)] * v[r];
  }
};

// Bunch-Kaufman LDL^T (LAPACK dsytf2 / dsytrs, lower) of a packed symmetric
// n x n matrix, for the rare local blocks that need interchanges.  Run-time
// indexing: these live in their own (not inlined) frame.
// T = double (private memory) or an LDS double (device: the pivoted blocks' lane-private LDS slice)
template <class T>
HTP_HD inline T& pk_at(T* K, int r, int c) { return r >= c ? K[r * (r + 1) / 2 + c] : K[c * (c + 1) / 2 + r]; }

template <class T>
HTP_HD inline void bk_factor_packed(T* K, int* ip, int n, int& neg, int& zero) {
  const double alpha = 0.6403882032022076;
  neg = 0;
  zero = 0;
  int k = 0;
  while (k < n) {
    int kstep = 1, kp = k;
    const double absakk = fabs(pk_at(K, k, k));
    int imax = k;
    double colmax = 0.0;
    for (int r = k + 1; r < n; ++r)
      if (fabs(pk_at(K, r, k)) > colmax) { colmax = fabs(pk_at(K, r, k)); imax = r; }
    if (!(absakk >= alpha * colmax) && !(absakk == 0.0 && colmax == 0.0)) {
      double rowmax = 0.0;
      for (int j = k; j < n; ++j)
        if (j != imax && fabs(pk_at(K, imax, j)) > rowmax) rowmax = fabs(pk_at(K, imax, j));
      if (absakk >= alpha * colmax * (colmax / rowmax)) kp = k;
      else if (fabs(pk_at(K, imax, imax)) >= alpha * rowmax) kp = imax;
      else { kp = imax; kstep = 2; }
    }
    const int kk = k + kstep - 1;
    if (kp != kk) {
      for (int j = k; j < n; ++j)
        if (j != kk && j != kp) { const double t = pk_at(K, kk, j); pk_at(K, kk, j) = pk_at(K, kp, j); pk_at(K, kp, j) = t; }
      const double t = pk_at(K, kk, kk); pk_at(K, kk, kk) = pk_at(K, kp, kp); pk_at(K, kp, kp) = t;
    }
    if (kstep == 1) {
      double d = pk_at(K, k, k);
      if (d == 0.0) { zero = 1; d = 1.0; pk_at(K, k, k) = 1.0; }
      if (d < 0.0) ++neg;
      const double id = 1.0 / d;
      for (int r = k + 1; r < n; ++r) {
        const double lr = pk_at(K, r, k) * id;
        for (int q = k + 1; q <= r; ++q) pk_at(K, r, q) -= lr * pk_at(K, q, k);
      }
      for (int r = k + 1; r < n; ++r) pk_at(K, r, k) *= id;
      ip[k] = kp;
    } else {
      const double d11 = pk_at(K, k, k), d21 = pk_at(K, k + 1, k), d22 = pk_at(K, k + 1, k + 1);
      const double det = d11 * d22 - d21 * d21;
      if (det < 0.0) neg += 1;
      else if (det > 0.0) neg += (d11 + d22 < 0.0) ? 2 : 0;
      else zero = 1;
      const double i11 = d22 / det, i22 = d11 / det, i21 = -d21 / det;
      for (int r = n - 1; r >= k + 2; --r) {  // descending: rows q < r still hold their original columns
        const double a1 = pk_at(K, r, k), a2 = pk_at(K, r, k + 1);
        const double l1 = a1 * i11 + a2 * i21, l2 = a1 * i21 + a2 * i22;
        for (int q = k + 2; q <= r; ++q) pk_at(K, r, q) -= l1 * pk_at(K, q, k) + l2 * pk_at(K, q, k + 1);
        pk_at(K, r, k) = l1;
        pk_at(K, r, k + 1) = l2;
      }
      ip[k] = -(kp + 1);
      ip[k + 1] = -(kp + 1);
    }
    k += kstep;
  }
}

template <class T>
HTP_HD inline void bk_solve_packed(T* K, const int* ip, int n, double* v) {
  int k = 0;
  while (k < n) {
    if (ip[k] >= 0) {
      const int kp = ip[k];
      if (kp != k) { const double t = v[k]; v[k] = v[kp]; v[kp] = t; }
      for (int r = k + 1; r < n; ++r) v[r] -= pk_at(K, r, k) * v[k];
      v[k] /= pk_at(K, k, k);
      k += 1;
    } else {
      const int kp = -ip[k] - 1;
      if (kp != k + 1) { const double t = v[k + 1]; v[k + 1] = v[kp]; v[kp] = t; }
      for (int r = k + 2; r < n; ++r) v[r] -= pk_at(K, r, k) * v[k] + pk_at(K, r, k + 1) * v[k + 1];
      const double d11 = pk_at(K, k, k), d21 = pk_at(K, k + 1, k), d22 = pk_at(K, k + 1, k + 1);
      const double det = d11 * d22 - d21 * d21;
      const double b1 = v[k], b2 = v[k + 1];
      v[k] = (d22 * b1 - d21 * b2) / det;
      v[k + 1] = (-d21 * b1 + d11 * b2) / det;
      k += 2;
    }
  }
  k = n - 1;
  while (k >= 0) {
    if (ip[k] >= 0) {
      for (int r = k + 1; r < n; ++r) v[k] -= pk_at(K, r, k) * v[r];
      const int kp = ip[k];
      if (kp != k) { const double t = v[k]; v[k] = v[kp]; v[kp] = t; }
      k -= 1;
    } else {
      for (int r = k + 1; r < n; ++r) {
        v[k] -= pk_at(K, r, k) * v[r];
        v[k - 1] -= pk_at(K, r, k - 1) * v[r];
      }
      const int kp = -ip[k] - 1;
      if (kp != k) { const double t = v[k]; v[k] = v[kp]; v[kp] = t; }
      k -= 2;
    }
  }
}

// The same Bunch-Kaufman factorization and solves for a compile-time n, written for SIMD execution: the lanes of
// a wavefront each factor their own block with their own pivots, so every loop runs over the full compile-time
// range with per-lane predicates (no lane-dependent trip counts or divergent loop control); element (r, q) of the
// packed block sits at K[S (r (r + 1) / 2 + q)] (S = 64: the lanes' blocks interleaved in LDS, a constant offset
// from the lane's base for constant r, q); the pivot vector and the right-hand sides live in registers (constant
// indices; the per-lane k / kp are reached through selects).  Every element sees the operations of
// bk_factor_packed / bk_solve_packed above in the same order, so factors, inertia and solutions are bit-identical.
template <int S, class T>
HTP_HD HTP_FI inline T& pkx(T* K, int r, int c) { return K[S * (r >= c ? r * (r + 1) / 2 + c : c * (c + 1) / 2 + r)]; }
// The empty asm hands each element to the select chain as a register value: without it InstCombine turns the
// chain of selects between loads v[j] into one load from a select between their addresses, a run-time index that
// keeps the whole array (pivot vector, right-hand sides) in scratch memory instead of registers.
#ifndef HTP_J8
#define HTP_J8 1
#endif
#ifndef HTP_SEL_OPAQUE
#define HTP_SEL_OPAQUE 0
#endif
#ifndef HTP_BK_BATCH
#define HTP_BK_BATCH 1
#endif
#ifndef HTP_BK_MULTI
#define HTP_BK_MULTI 0
#endif
template <class V>
HTP_HD HTP_FI inline V sel_opaque(V x) {
#if defined(__HIP_DEVICE_COMPILE__) && HTP_SEL_OPAQUE
  asm("" : "+v"(x));
#endif
  return x;
}
#ifndef HTP_SEL_MASK
#define HTP_SEL_MASK 0
#endif
template <int n, class V>
HTP_HD HTP_FI inline V sel_get(const V* v, int k) {
#if HTP_SEL_MASK
  // v[k] as an OR of masked bit patterns (exactly one mask is all ones): no select of loads for InstCombine to
  // fold into a run-time address
  using U = typename std::conditional<sizeof(V) == 8, unsigned long long, unsigned int>::type;
  U r = 0;
#pragma unroll
  for (int j = 0; j < n; ++j) r |= __builtin_bit_cast(U, v[j]) & (U)(-(long long)(k == j));
  return __builtin_bit_cast(V, r);
#else
  V r = sel_opaque(v[0]);
#pragma unroll
  for (int j = 1; j < n; ++j) r = (k == j) ? sel_opaque(v[j]) : r;
  return r;
#endif
}
template <int n>
HTP_HD HTP_FI inline void sel_set(double* v, int k, double x) {
#pragma unroll
  for (int j = 0; j < n; ++j) v[j] = (k == j) ? x : v[j];
}

template <int n, int S, class T>
HTP_HD HTP_FI inline void bk_factor_simd(T* K, int* ip, int& neg, int& zero) {
  const double alpha = 0.6403882032022076;
  neg = 0;
  zero = 0;
#pragma unroll
  for (int j = 0; j < n; ++j) ip[j] = 0;
  int k = 0;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {
    const bool act = k < n;
    const int kc = act ? k : 0;                    // a valid index for the finished lanes' (unused) loads
    int kstep = 1, kp = kc;
    const double absakk = fabs((double)K[S * (kc * (kc + 1) / 2 + kc)]);
    int imax = kc;
    double colmax = 0.0;
#pragma unroll
    for (int r = 1; r < n; ++r)
      if (r > kc) {
        const double v = fabs((double)K[S * (r * (r + 1) / 2 + kc)]);
        if (v > colmax) { colmax = v; imax = r; }
      }
    if (act && !(absakk >= alpha * colmax) && !(absakk == 0.0 && colmax == 0.0)) {
      double rowmax = 0.0;
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (j >= kc && j != imax) {
          const double v = fabs((double)pkx<S>(K, imax, j));
          if (v > rowmax) rowmax = v;
        }
      if (absakk >= alpha * colmax * (colmax / rowmax)) kp = kc;
      else if (fabs((double)K[S * (imax * (imax + 1) / 2 + imax)]) >= alpha * rowmax) kp = imax;
      else { kp = imax; kstep = 2; }
    }
    const int kk = kc + kstep - 1;
    if (act && kp != kk) {
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (j >= kc && j != kk && j != kp) {
          T& a = pkx<S>(K, kk, j);
          T& b = pkx<S>(K, kp, j);
          const double t = a; a = b; b = t;
        }
      T& a = K[S * (kk * (kk + 1) / 2 + kk)];
      T& b = K[S * (kp * (kp + 1) / 2 + kp)];
      const double t = a; a = b; b = t;
    }
    if (act && kstep == 1) {
      double d = K[S * (kc * (kc + 1) / 2 + kc)];
      if (d == 0.0) { zero = 1; d = 1.0; K[S * (kc * (kc + 1) / 2 + kc)] = 1.0; }
      if (d < 0.0) ++neg;
      const double id = 1.0 / d;
      double lr[n];
#pragma unroll
      for (int r = 0; r < n; ++r) lr[r] = (r > kc) ? (double)K[S * (r * (r + 1) / 2 + kc)] * id : 0.0;
#pragma unroll
      for (int r = 1; r < n; ++r)
#pragma unroll
        for (int q = 1; q <= r; ++q)
          if (q > kc) K[S * (r * (r + 1) / 2 + q)] -= lr[r] * K[S * (q * (q + 1) / 2 + kc)];
#pragma unroll
      for (int r = 1; r < n; ++r)
        if (r > kc) K[S * (r * (r + 1) / 2 + kc)] *= id;
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (j == kc) ip[j] = kp;
    } else if (act) {
      const double d11 = K[S * (kc * (kc + 1) / 2 + kc)], d21 = K[S * ((kc + 1) * (kc + 2) / 2 + kc)];
      const double d22 = K[S * ((kc + 1) * (kc + 2) / 2 + kc + 1)];
      const double det = d11 * d22 - d21 * d21;
      if (det < 0.0) neg += 1;
      else if (det > 0.0) neg += (d11 + d22 < 0.0) ? 2 : 0;
      else zero = 1;
      const double i11 = d22 / det, i22 = d11 / det, i21 = -d21 / det;
#pragma unroll
      for (int r = n - 1; r >= 2; --r) {  // descending: rows q < r still hold their original columns
        if (r >= kc + 2) {
          const double a1 = K[S * (r * (r + 1) / 2 + kc)], a2 = K[S * (r * (r + 1) / 2 + kc + 1)];
          const double l1 = a1 * i11 + a2 * i21, l2 = a1 * i21 + a2 * i22;
#pragma unroll
          for (int q = 2; q <= r; ++q)
            if (q >= kc + 2)
              K[S * (r * (r + 1) / 2 + q)] -= l1 * K[S * (q * (q + 1) / 2 + kc)] + l2 * K[S * (q * (q + 1) / 2 + kc + 1)];
          K[S * (r * (r + 1) / 2 + kc)] = l1;
          K[S * (r * (r + 1) / 2 + kc + 1)] = l2;
        }
      }
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (j == kc || j == kc + 1) ip[j] = -(kp + 1);
    }
    k += act ? kstep : 0;
  }
}

template <int n, int S, class T>
HTP_HD HTP_FI inline void bk_solve_simd(T* K, const int* ip, double* v) {
  int k = 0;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {          // forward: P, L, D
    const bool act = k < n;
    const int kc = act ? k : 0;
    const int ipk = sel_get<n>(ip, kc);
    if (act && ipk >= 0) {
      const int kp = ipk;
      if (kp != kc) { const double a = sel_get<n>(v, kc), b = sel_get<n>(v, kp); sel_set<n>(v, kc, b); sel_set<n>(v, kp, a); }
      const double vk = sel_get<n>(v, kc);
#pragma unroll
      for (int r = 1; r < n; ++r)
        if (r > kc) v[r] -= K[S * (r * (r + 1) / 2 + kc)] * vk;
      const double dkk = K[S * (kc * (kc + 1) / 2 + kc)];
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (j == kc) v[j] /= dkk;
      k += 1;
    } else if (act) {
      const int kp = -ipk - 1;
      if (kp != kc + 1) {
        const double a = sel_get<n>(v, kc + 1), b = sel_get<n>(v, kp);
        sel_set<n>(v, kc + 1, b);
        sel_set<n>(v, kp, a);
      }
      const double vk = sel_get<n>(v, kc), vk1 = sel_get<n>(v, kc + 1);
#pragma unroll
      for (int r = 2; r < n; ++r)
        if (r > kc + 1) v[r] -= K[S * (r * (r + 1) / 2 + kc)] * vk + K[S * (r * (r + 1) / 2 + kc + 1)] * vk1;
      const double d11 = K[S * (kc * (kc + 1) / 2 + kc)], d21 = K[S * ((kc + 1) * (kc + 2) / 2 + kc)];
      const double d22 = K[S * ((kc + 1) * (kc + 2) / 2 + kc + 1)];
      const double det = d11 * d22 - d21 * d21;
      const double b1 = vk, b2 = vk1;
      sel_set<n>(v, kc, (d22 * b1 - d21 * b2) / det);
      sel_set<n>(v, kc + 1, (-d21 * b1 + d11 * b2) / det);
      k += 2;
    }
  }
  k = n - 1;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {          // backward: L', P'
    const bool act = k >= 0;
    const int kc = act ? k : 0;
    const int ipk = sel_get<n>(ip, kc);
    if (act && ipk >= 0) {
      double t = sel_get<n>(v, kc);
#pragma unroll
      for (int r = 1; r < n; ++r)
        if (r > kc) t -= K[S * (r * (r + 1) / 2 + kc)] * v[r];
      sel_set<n>(v, kc, t);
      const int kp = ipk;
      if (kp != kc) { const double a = sel_get<n>(v, kc), b = sel_get<n>(v, kp); sel_set<n>(v, kc, b); sel_set<n>(v, kp, a); }
      k -= 1;
    } else if (act) {
      const int km = kc >= 1 ? kc - 1 : 0;
      double t = sel_get<n>(v, kc), t1 = sel_get<n>(v, km);
#pragma unroll
      for (int r = 1; r < n; ++r)
        if (r > kc) {
          t -= K[S * (r * (r + 1) / 2 + kc)] * v[r];
          t1 -= K[S * (r * (r + 1) / 2 + km)] * v[r];
        }
      sel_set<n>(v, kc, t);
      sel_set<n>(v, km, t1);
      const int kp = -ipk - 1;
      if (kp != kc) { const double a = sel_get<n>(v, kc), b = sel_get<n>(v, kp); sel_set<n>(v, kc, b); sel_set<n>(v, kp, a); }
      k -= 2;
    }
  }
}

// bk_factor_simd / bk_solve_simd with every step's loads issued together (HTP_BK_BATCH, the default).  In the
// forms above each element's read-modify-write sits under its own per-lane predicate and reads a run-time-indexed
// element (column k) that may alias the previous write, so on the device every one of the ~1 500 LDS accesses of a
// factorization waited a full LDS round trip.  Here each step first loads what it reads (column k, the rows to
// interchange), then updates constant-offset elements with select-stores; the column values are the ones the
// original loop reads (an update never writes column k, and the 2 x 2 branch's descending row order already
// read the original columns), every element gets the same expression in the same order: bit-identical.
template <int n, int S, class T>
HTP_HD HTP_FI inline void bk_factor_batch(T* K, int* ip, int& neg, int& zero) {
  const double alpha = 0.6403882032022076;
  neg = 0;
  zero = 0;
#pragma unroll
  for (int j = 0; j < n; ++j) ip[j] = 0;
  int k = 0;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {
    const bool act = k < n;
    const int kc = act ? k : 0;
    int kstep = 1, kp = kc;
    double cs[n];                                  // K(r, kc) for r > kc (r <= kc: in-bounds, unused)
#pragma unroll
    for (int r = 0; r < n; ++r) cs[r] = K[S * (r * (r + 1) / 2 + kc)];
    const double absakk = fabs((double)K[S * (kc * (kc + 1) / 2 + kc)]);
    int imax = kc;
    double colmax = 0.0;
#pragma unroll
    for (int r = 1; r < n; ++r) {
      const double v = fabs(cs[r]);
      const bool t = r > kc && v > colmax;
      colmax = t ? v : colmax;
      imax = t ? r : imax;
    }
    if (act && !(absakk >= alpha * colmax) && !(absakk == 0.0 && colmax == 0.0)) {
      double rw[n];
#pragma unroll
      for (int j = 0; j < n; ++j) rw[j] = fabs((double)pkx<S>(K, imax, j));
      const double dmax = fabs((double)K[S * (imax * (imax + 1) / 2 + imax)]);
      double rowmax = 0.0;
#pragma unroll
      for (int j = 0; j < n; ++j) rowmax = (j >= kc && j != imax && rw[j] > rowmax) ? rw[j] : rowmax;
      if (absakk >= alpha * colmax * (colmax / rowmax)) kp = kc;
      else if (dmax >= alpha * rowmax) kp = imax;
      else { kp = imax; kstep = 2; }
    }
    const int kk = kc + kstep - 1;
    if (act && kp != kk) {                         // the interchanged elements are distinct: load all, then store
      double a[n], b[n];
#pragma unroll
      for (int j = 0; j < n; ++j) { a[j] = pkx<S>(K, kk, j); b[j] = pkx<S>(K, kp, j); }
      const double dk = K[S * (kk * (kk + 1) / 2 + kk)], dp = K[S * (kp * (kp + 1) / 2 + kp)];
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (j >= kc && j != kk && j != kp) { pkx<S>(K, kk, j) = b[j]; pkx<S>(K, kp, j) = a[j]; }
      K[S * (kk * (kk + 1) / 2 + kk)] = dp;
      K[S * (kp * (kp + 1) / 2 + kp)] = dk;
    }
    if (act && kstep == 1) {
      double c[n];
#pragma unroll
      for (int r = 0; r < n; ++r) c[r] = K[S * (r * (r + 1) / 2 + kc)];
      double d = K[S * (kc * (kc + 1) / 2 + kc)];
      if (d == 0.0) { zero = 1; d = 1.0; K[S * (kc * (kc + 1) / 2 + kc)] = 1.0; }
      if (d < 0.0) ++neg;
      const double id = 1.0 / d;
      double lr[n];
#pragma unroll
      for (int r = 0; r < n; ++r) lr[r] = (r > kc) ? c[r] * id : 0.0;
#pragma unroll
      for (int r = 1; r < n; ++r)
#pragma unroll
        for (int q = 1; q <= r; ++q) {
          T& e = K[S * (r * (r + 1) / 2 + q)];
          const double kv = e;
          const double nv = kv - lr[r] * c[q];
          e = (q > kc) ? nv : kv;
        }
#pragma unroll
      for (int r = 1; r < n; ++r)
        if (r > kc) K[S * (r * (r + 1) / 2 + kc)] = c[r] * id;
#pragma unroll
      for (int j = 0; j < n; ++j) ip[j] = (j == kc) ? kp : ip[j];
    } else if (act) {
      double ca[n], cb[n];
#pragma unroll
      for (int r = 0; r < n; ++r) {
        ca[r] = K[S * (r * (r + 1) / 2 + kc)];
        cb[r] = K[S * (r * (r + 1) / 2 + (kc + 1 < n ? kc + 1 : kc))];
      }
      const double d11 = K[S * (kc * (kc + 1) / 2 + kc)], d21 = K[S * ((kc + 1) * (kc + 2) / 2 + kc)];
      const double d22 = K[S * ((kc + 1) * (kc + 2) / 2 + kc + 1)];
      const double det = d11 * d22 - d21 * d21;
      if (det < 0.0) neg += 1;
      else if (det > 0.0) neg += (d11 + d22 < 0.0) ? 2 : 0;
      else zero = 1;
      const double i11 = d22 / det, i22 = d11 / det, i21 = -d21 / det;
      double l1[n], l2[n];
#pragma unroll
      for (int r = 0; r < n; ++r) {
        const double a1 = ca[r], a2 = cb[r];
        l1[r] = a1 * i11 + a2 * i21;
        l2[r] = a1 * i21 + a2 * i22;
      }
#pragma unroll
      for (int r = 2; r < n; ++r)
#pragma unroll
        for (int q = 2; q <= r; ++q) {
          T& e = K[S * (r * (r + 1) / 2 + q)];
          const double kv = e;
          const double nv = kv - (l1[r] * ca[q] + l2[r] * cb[q]);
          e = (q >= kc + 2) ? nv : kv;
        }
#pragma unroll
      for (int r = 2; r < n; ++r)
        if (r >= kc + 2) {
          K[S * (r * (r + 1) / 2 + kc)] = l1[r];
          K[S * (r * (r + 1) / 2 + kc + 1)] = l2[r];
        }
#pragma unroll
      for (int j = 0; j < n; ++j) ip[j] = (j == kc || j == kc + 1) ? -(kp + 1) : ip[j];
    }
    k += act ? kstep : 0;
  }
}

// Bunch-Kaufman pivot vector packed into one 64-bit word (HTP_PIV_V_LDS): entry j in bits [6 j, 6 j + 6) as
// ip[j] + 32 (|ip[j]| <= n <= 16), so the run-time-indexed reads and writes are shifts on a register, not a
// private-memory array.  The same integer values as bk_factor_batch's ip.
HTP_HD HTP_FI inline unsigned long long piv_put(unsigned long long w, int j, int v) {
  return (w & ~(63ull << (6 * j))) | ((unsigned long long)(v + 32) << (6 * j));
}
HTP_HD HTP_FI inline int piv_get(unsigned long long w, int j) { return (int)((w >> (6 * j)) & 63ull) - 32; }

// bk_factor_batch with the pivot vector packed (piv_put)
template <int n, int S, class T>
HTP_HD HTP_FI inline void bk_factor_batch_p(T* K, unsigned long long& ipw, int& neg, int& zero) {
  const double alpha = 0.6403882032022076;
  neg = 0;
  zero = 0;
  ipw = 0;
#pragma unroll
  for (int j = 0; j < n; ++j) ipw |= 32ull << (6 * j);   // every pivot 0
  int k = 0;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {
    const bool act = k < n;
    const int kc = act ? k : 0;
    int kstep = 1, kp = kc;
    double cs[n];                                  // K(r, kc) for r > kc (r <= kc: in-bounds, unused)
#pragma unroll
    for (int r = 0; r < n; ++r) cs[r] = K[S * (r * (r + 1) / 2 + kc)];
    const double absakk = fabs((double)K[S * (kc * (kc + 1) / 2 + kc)]);
    int imax = kc;
    double colmax = 0.0;
#pragma unroll
    for (int r = 1; r < n; ++r) {
      const double v = fabs(cs[r]);
      const bool t = r > kc && v > colmax;
      colmax = t ? v : colmax;
      imax = t ? r : imax;
    }
    if (act && !(absakk >= alpha * colmax) && !(absakk == 0.0 && colmax == 0.0)) {
      double rw[n];
#pragma unroll
      for (int j = 0; j < n; ++j) rw[j] = fabs((double)pkx<S>(K, imax, j));
      const double dmax = fabs((double)K[S * (imax * (imax + 1) / 2 + imax)]);
      double rowmax = 0.0;
#pragma unroll
      for (int j = 0; j < n; ++j) rowmax = (j >= kc && j != imax && rw[j] > rowmax) ? rw[j] : rowmax;
      if (absakk >= alpha * colmax * (colmax / rowmax)) kp = kc;
      else if (dmax >= alpha * rowmax) kp = imax;
      else { kp = imax; kstep = 2; }
    }
    const int kk = kc + kstep - 1;
    if (act && kp != kk) {                         // the interchanged elements are distinct: load all, then store
      double a[n], b[n];
#pragma unroll
      for (int j = 0; j < n; ++j) { a[j] = pkx<S>(K, kk, j); b[j] = pkx<S>(K, kp, j); }
      const double dk = K[S * (kk * (kk + 1) / 2 + kk)], dp = K[S * (kp * (kp + 1) / 2 + kp)];
#pragma unroll
      for (int j = 0; j < n; ++j)
        if (j >= kc && j != kk && j != kp) { pkx<S>(K, kk, j) = b[j]; pkx<S>(K, kp, j) = a[j]; }
      K[S * (kk * (kk + 1) / 2 + kk)] = dp;
      K[S * (kp * (kp + 1) / 2 + kp)] = dk;
    }
    if (act && kstep == 1) {
      double c[n];
#pragma unroll
      for (int r = 0; r < n; ++r) c[r] = K[S * (r * (r + 1) / 2 + kc)];
      double d = K[S * (kc * (kc + 1) / 2 + kc)];
      if (d == 0.0) { zero = 1; d = 1.0; K[S * (kc * (kc + 1) / 2 + kc)] = 1.0; }
      if (d < 0.0) ++neg;
      const double id = 1.0 / d;
      double lr[n];
#pragma unroll
      for (int r = 0; r < n; ++r) lr[r] = (r > kc) ? c[r] * id : 0.0;
#pragma unroll
      for (int r = 1; r < n; ++r)
#pragma unroll
        for (int q = 1; q <= r; ++q) {
          T& e = K[S * (r * (r + 1) / 2 + q)];
          const double kv = e;
          const double nv = kv - lr[r] * c[q];
          e = (q > kc) ? nv : kv;
        }
#pragma unroll
      for (int r = 1; r < n; ++r)
        if (r > kc) K[S * (r * (r + 1) / 2 + kc)] = c[r] * id;
      ipw = piv_put(ipw, kc, kp);
    } else if (act) {
      double ca[n], cb[n];
#pragma unroll
      for (int r = 0; r < n; ++r) {
        ca[r] = K[S * (r * (r + 1) / 2 + kc)];
        cb[r] = K[S * (r * (r + 1) / 2 + (kc + 1 < n ? kc + 1 : kc))];
      }
      const double d11 = K[S * (kc * (kc + 1) / 2 + kc)], d21 = K[S * ((kc + 1) * (kc + 2) / 2 + kc)];
      const double d22 = K[S * ((kc + 1) * (kc + 2) / 2 + kc + 1)];
      const double det = d11 * d22 - d21 * d21;
      if (det < 0.0) neg += 1;
      else if (det > 0.0) neg += (d11 + d22 < 0.0) ? 2 : 0;
      else zero = 1;
      const double i11 = d22 / det, i22 = d11 / det, i21 = -d21 / det;
      double l1[n], l2[n];
#pragma unroll
      for (int r = 0; r < n; ++r) {
        const double a1 = ca[r], a2 = cb[r];
        l1[r] = a1 * i11 + a2 * i21;
        l2[r] = a1 * i21 + a2 * i22;
      }
#pragma unroll
      for (int r = 2; r < n; ++r)
#pragma unroll
        for (int q = 2; q <= r; ++q) {
          T& e = K[S * (r * (r + 1) / 2 + q)];
          const double kv = e;
          const double nv = kv - (l1[r] * ca[q] + l2[r] * cb[q]);
          e = (q >= kc + 2) ? nv : kv;
        }
#pragma unroll
      for (int r = 2; r < n; ++r)
        if (r >= kc + 2) {
          K[S * (r * (r + 1) / 2 + kc)] = l1[r];
          K[S * (r * (r + 1) / 2 + kc + 1)] = l2[r];
        }
      ipw = piv_put(piv_put(ipw, kc, -(kp + 1)), kc + 1, -(kp + 1));
    }
    k += act ? kstep : 0;
  }
}

template <int n, int S, class T>
HTP_HD HTP_FI inline void bk_solve_batch(const T* K, const int* ip, double* v) {
  int k = 0;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {          // forward: P, L, D
    const bool act = k < n;
    const int kc = act ? k : 0;
    const int ipk = sel_get<n>(ip, kc);
    const int kc1 = kc + 1 < n ? kc + 1 : kc;
    double ca[n], cb[n];
#pragma unroll
    for (int r = 0; r < n; ++r) { ca[r] = K[S * (r * (r + 1) / 2 + kc)]; cb[r] = K[S * (r * (r + 1) / 2 + kc1)]; }
    const double d11 = K[S * (kc * (kc + 1) / 2 + kc)], d21 = K[S * (kc1 * (kc1 + 1) / 2 + kc)];
    const double d22 = K[S * (kc1 * (kc1 + 1) / 2 + kc1)];
    if (act && ipk >= 0) {
      const int kp = ipk;
      if (kp != kc) { const double a = sel_get<n>(v, kc), b = sel_get<n>(v, kp); sel_set<n>(v, kc, b); sel_set<n>(v, kp, a); }
      const double vk = sel_get<n>(v, kc);
#pragma unroll
      for (int r = 1; r < n; ++r) {
        const double nv = v[r] - ca[r] * vk;
        v[r] = (r > kc) ? nv : v[r];
      }
#pragma unroll
      for (int j = 0; j < n; ++j) v[j] = (j == kc) ? v[j] / d11 : v[j];
      k += 1;
    } else if (act) {
      const int kp = -ipk - 1;
      if (kp != kc + 1) {
        const double a = sel_get<n>(v, kc + 1), b = sel_get<n>(v, kp);
        sel_set<n>(v, kc + 1, b);
        sel_set<n>(v, kp, a);
      }
      const double vk = sel_get<n>(v, kc), vk1 = sel_get<n>(v, kc + 1);
#pragma unroll
      for (int r = 2; r < n; ++r) {
        const double nv = v[r] - (ca[r] * vk + cb[r] * vk1);
        v[r] = (r > kc + 1) ? nv : v[r];
      }
      const double det = d11 * d22 - d21 * d21;
      const double b1 = vk, b2 = vk1;
      sel_set<n>(v, kc, (d22 * b1 - d21 * b2) / det);
      sel_set<n>(v, kc + 1, (-d21 * b1 + d11 * b2) / det);
      k += 2;
    }
  }
  k = n - 1;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {          // backward: L', P'
    const bool act = k >= 0;
    const int kc = act ? k : 0;
    const int ipk = sel_get<n>(ip, kc);
    const int km = kc >= 1 ? kc - 1 : 0;
    double ca[n], cm[n];
#pragma unroll
    for (int r = 0; r < n; ++r) { ca[r] = K[S * (r * (r + 1) / 2 + kc)]; cm[r] = K[S * (r * (r + 1) / 2 + km)]; }
    if (act && ipk >= 0) {
      double t = sel_get<n>(v, kc);
#pragma unroll
      for (int r = 1; r < n; ++r) {
        const double nt = t - ca[r] * v[r];
        t = (r > kc) ? nt : t;
      }
      sel_set<n>(v, kc, t);
      const int kp = ipk;
      if (kp != kc) { const double a = sel_get<n>(v, kc), b = sel_get<n>(v, kp); sel_set<n>(v, kc, b); sel_set<n>(v, kp, a); }
      k -= 1;
    } else if (act) {
      double t = sel_get<n>(v, kc), t1 = sel_get<n>(v, km);
#pragma unroll
      for (int r = 1; r < n; ++r) {
        const double nt = t - ca[r] * v[r];
        const double nt1 = t1 - cm[r] * v[r];
        t = (r > kc) ? nt : t;
        t1 = (r > kc) ? nt1 : t1;
      }
      sel_set<n>(v, kc, t);
      sel_set<n>(v, km, t1);
      const int kp = -ipk - 1;
      if (kp != kc) { const double a = sel_get<n>(v, kc), b = sel_get<n>(v, kp); sel_set<n>(v, kc, b); sel_set<n>(v, kp, a); }
      k -= 2;
    }
  }
}

// bk_solve_batch with the right-hand side in this lane's interleaved LDS slice (element j at v[64 j], HTP_PIV_V_LDS):
// the run-time-indexed reads and writes of v (column kc, the interchanged rows) are LDS accesses instead of select
// chains that the compiler folds into private-memory (scratch) accesses.  The same operations on the same values.
template <int n, int S, class T, class VT>
HTP_HD HTP_FI inline void bk_solve_batch_l(const T* K, unsigned long long ipw, VT* v) {
  int k = 0;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {          // forward: P, L, D
    const bool act = k < n;
    const int kc = act ? k : 0;
    const int ipk = piv_get(ipw, kc);
    const int kc1 = kc + 1 < n ? kc + 1 : kc;
    double ca[n], cb[n];
#pragma unroll
    for (int r = 0; r < n; ++r) { ca[r] = K[S * (r * (r + 1) / 2 + kc)]; cb[r] = K[S * (r * (r + 1) / 2 + kc1)]; }
    const double d11 = K[S * (kc * (kc + 1) / 2 + kc)], d21 = K[S * (kc1 * (kc1 + 1) / 2 + kc)];
    const double d22 = K[S * (kc1 * (kc1 + 1) / 2 + kc1)];
    if (act && ipk >= 0) {
      const int kp = ipk;
      if (kp != kc) { const double a = v[64 * kc], b = v[64 * kp]; v[64 * kc] = b; v[64 * kp] = a; }
      const double vk = v[64 * kc];
#pragma unroll
      for (int r = 1; r < n; ++r) {
        const double vr = v[64 * r];
        const double nv = vr - ca[r] * vk;
        v[64 * r] = (r > kc) ? nv : vr;
      }
      v[64 * kc] = v[64 * kc] / d11;
      k += 1;
    } else if (act) {
      const int kp = -ipk - 1;
      if (kp != kc + 1) {
        const double a = v[64 * (kc + 1)], b = v[64 * kp];
        v[64 * (kc + 1)] = b;
        v[64 * kp] = a;
      }
      const double vk = v[64 * kc], vk1 = v[64 * (kc + 1)];
#pragma unroll
      for (int r = 2; r < n; ++r) {
        const double vr = v[64 * r];
        const double nv = vr - (ca[r] * vk + cb[r] * vk1);
        v[64 * r] = (r > kc + 1) ? nv : vr;
      }
      const double det = d11 * d22 - d21 * d21;
      const double b1 = vk, b2 = vk1;
      v[64 * kc] = (d22 * b1 - d21 * b2) / det;
      v[64 * (kc + 1)] = (-d21 * b1 + d11 * b2) / det;
      k += 2;
    }
  }
  k = n - 1;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {          // backward: L', P'
    const bool act = k >= 0;
    const int kc = act ? k : 0;
    const int ipk = piv_get(ipw, kc);
    const int km = kc >= 1 ? kc - 1 : 0;
    double ca[n], cm[n];
#pragma unroll
    for (int r = 0; r < n; ++r) { ca[r] = K[S * (r * (r + 1) / 2 + kc)]; cm[r] = K[S * (r * (r + 1) / 2 + km)]; }
    if (act && ipk >= 0) {
      double t = v[64 * kc];
#pragma unroll
      for (int r = 1; r < n; ++r) {
        const double nt = t - ca[r] * v[64 * r];
        t = (r > kc) ? nt : t;
      }
      v[64 * kc] = t;
      const int kp = ipk;
      if (kp != kc) { const double a = v[64 * kc], b = v[64 * kp]; v[64 * kc] = b; v[64 * kp] = a; }
      k -= 1;
    } else if (act) {
      double t = v[64 * kc], t1 = v[64 * km];
#pragma unroll
      for (int r = 1; r < n; ++r) {
        const double vr = v[64 * r];
        const double nt = t - ca[r] * vr;
        const double nt1 = t1 - cm[r] * vr;
        t = (r > kc) ? nt : t;
        t1 = (r > kc) ? nt1 : t1;
      }
      v[64 * kc] = t;
      v[64 * km] = t1;
      const int kp = -ipk - 1;
      if (kp != kc) { const double a = v[64 * kc], b = v[64 * kp]; v[64 * kc] = b; v[64 * kp] = a; }
      k -= 2;
    }
  }
}

// bk_solve_batch for NR right-hand sides at once (HTP_BK_MULTI): the steps' pivot selects and LDS loads are shared
// by the columns, each column sees exactly bk_solve_batch's operations.
template <int n, int S, int NR, class T>
HTP_HD HTP_FI inline void bk_solve_batch_multi(const T* K, const int* ip, double (*v)[n]) {
  int k = 0;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {          // forward: P, L, D
    const bool act = k < n;
    const int kc = act ? k : 0;
    const int ipk = sel_get<n>(ip, kc);
    const int kc1 = kc + 1 < n ? kc + 1 : kc;
    double ca[n], cb[n];
#pragma unroll
    for (int r = 0; r < n; ++r) { ca[r] = K[S * (r * (r + 1) / 2 + kc)]; cb[r] = K[S * (r * (r + 1) / 2 + kc1)]; }
    const double d11 = K[S * (kc * (kc + 1) / 2 + kc)], d21 = K[S * (kc1 * (kc1 + 1) / 2 + kc)];
    const double d22 = K[S * (kc1 * (kc1 + 1) / 2 + kc1)];
    if (act && ipk >= 0) {
      const int kp = ipk;
#pragma unroll
      for (int c = 0; c < NR; ++c) {
        if (kp != kc) { const double a = sel_get<n>(v[c], kc), b = sel_get<n>(v[c], kp); sel_set<n>(v[c], kc, b); sel_set<n>(v[c], kp, a); }
        const double vk = sel_get<n>(v[c], kc);
#pragma unroll
        for (int r = 1; r < n; ++r) {
          const double nv = v[c][r] - ca[r] * vk;
          v[c][r] = (r > kc) ? nv : v[c][r];
        }
#pragma unroll
        for (int j = 0; j < n; ++j) v[c][j] = (j == kc) ? v[c][j] / d11 : v[c][j];
      }
      k += 1;
    } else if (act) {
      const int kp = -ipk - 1;
      const double det = d11 * d22 - d21 * d21;
#pragma unroll
      for (int c = 0; c < NR; ++c) {
        if (kp != kc + 1) {
          const double a = sel_get<n>(v[c], kc + 1), b = sel_get<n>(v[c], kp);
          sel_set<n>(v[c], kc + 1, b);
          sel_set<n>(v[c], kp, a);
        }
        const double vk = sel_get<n>(v[c], kc), vk1 = sel_get<n>(v[c], kc + 1);
#pragma unroll
        for (int r = 2; r < n; ++r) {
          const double nv = v[c][r] - (ca[r] * vk + cb[r] * vk1);
          v[c][r] = (r > kc + 1) ? nv : v[c][r];
        }
        const double b1 = vk, b2 = vk1;
        sel_set<n>(v[c], kc, (d22 * b1 - d21 * b2) / det);
        sel_set<n>(v[c], kc + 1, (-d21 * b1 + d11 * b2) / det);
      }
      k += 2;
    }
  }
  k = n - 1;
#pragma unroll 1
  for (int step = 0; step < n; ++step) {          // backward: L', P'
    const bool act = k >= 0;
    const int kc = act ? k : 0;
    const int ipk = sel_get<n>(ip, kc);
    const int km = kc >= 1 ? kc - 1 : 0;
    double ca[n], cm[n];
#pragma unroll
    for (int r = 0; r < n; ++r) { ca[r] = K[S * (r * (r + 1) / 2 + kc)]; cm[r] = K[S * (r * (r + 1) / 2 + km)]; }
    if (act && ipk >= 0) {
      const int kp = ipk;
#pragma unroll
      for (int c = 0; c < NR; ++c) {
        double t = sel_get<n>(v[c], kc);
#pragma unroll
        for (int r = 1; r < n; ++r) {
          const double nt = t - ca[r] * v[c][r];
          t = (r > kc) ? nt : t;
        }
        sel_set<n>(v[c], kc, t);
        if (kp != kc) { const double a = sel_get<n>(v[c], kc), b = sel_get<n>(v[c], kp); sel_set<n>(v[c], kc, b); sel_set<n>(v[c], kp, a); }
      }
      k -= 1;
    } else if (act) {
      const int kp = -ipk - 1;
#pragma unroll
      for (int c = 0; c < NR; ++c) {
        double t = sel_get<n>(v[c], kc), t1 = sel_get<n>(v[c], km);
#pragma unroll
        for (int r = 1; r < n; ++r) {
          const double nt = t - ca[r] * v[c][r];
          const double nt1 = t1 - cm[r] * v[c][r];
          t = (r > kc) ? nt : t;
          t1 = (r > kc) ? nt1 : t1;
        }
        sel_set<n>(v[c], kc, t);
        sel_set<n>(v[c], km, t1);
        if (kp != kc) { const double a = sel_get<n>(v[c], kc), b = sel_get<n>(v[c], kp); sel_set<n>(v[c], kc, b); sel_set<n>(v[c], kp, a); }
      }
      k -= 2;
    }
  }
}

// LDS ring of the matrix-core Riccati passes (ObcaSolver::ring_fill): RING_SB + 1 stage records of
// RS_L doubles (LD slot prefix [0, SOFF + NS), V_i, X_i) after the per-wave scratch and filter.
#ifndef HTP_RING_SB
#define HTP_RING_SB 8
#endif
// ring_fill: lane-major copy with the record sources resolved once per lane (1) or the element-major copy of the
// round-4 kernel (0); the ring receives the same values
#ifndef HTP_RING_FILL_LANE
#define HTP_RING_FILL_LANE 1
#endif
constexpr int RING_SB = HTP_RING_SB;             // stages per block
constexpr int RS_SLOT = 142;                     // LD slot prefix (P | K | chol | J | 1/sc)
constexpr int RS_V = RS_SLOT, RS_X = RS_SLOT + NBMAX;
constexpr int RS_T = RS_SLOT + 2 * NBMAX;        // T_i, Q_i of the relaxed dynamics rows (relax_P), 5 x 5 each
constexpr int RS_L = RS_T + 50;                  // doubles per stage record
constexpr int RING_OFF = 4 * NBMAX * NBMAX + 8 + 2 * 64;
constexpr int RING_DOUBLES = (RING_SB + 1) * RS_L;
// pivoted local blocks (ObcaSolver::local_pivoted) on the device: one packed 10x10 block per lane in LDS,
// over the same region as the ring (never live at the same time)
// the pivoted local blocks through the SIMD-convergent Bunch-Kaufman (1) or the per-lane serial one (0, round 4)
#ifndef HTP_BK_SIMD
#define HTP_BK_SIMD 1
#endif
#ifndef HTP_PIV_LDS
#define HTP_PIV_LDS 1   // 0: pivoted blocks in private memory (smaller LDS footprint; experiments)
#endif
constexpr int PIV_LDS_PER_LANE = HTP_PIV_LDS ? 55 : 0;
constexpr int LDS_WAVE_DOUBLES = RING_OFF + (RING_DOUBLES > 64 * PIV_LDS_PER_LANE ? RING_DOUBLES : 64 * PIV_LDS_PER_LANE);
constexpr int FAC_W_FB = 11;   // factor staging doubles per stage with the fused backward solve (HTP_BWD_FUSE)
static_assert(HTP_FAC_SB >= 0 && RING_OFF + HTP_FAC_SB * (HTP_BWD_FUSE ? FAC_W_FB : 6) * 64 <= LDS_WAVE_DOUBLES,
              "factor staging exceeds the ring");

// ---------------------------------------------------------------------------
template <class Ctx, int EN_ = 4, int EM_ = 4, int FORM_ = 0>
struct ObcaSolver {
  static constexpr bool PT = FORM_ == 1;  // point formulation (optimizer_points.py)
  using gd = typename Ctx::gd;  // workspace / input arrays (HBM)
  using ld = typename Ctx::ld;  // per-wave LDS scratch
  using li = typename Ctx::li;
  using CDims = typename Ctx::template cst<Dims>;
  using CLayout = typename Ctx::template cst<Layout>;
  using COptions = typename Ctx::template cst<Options>;
  Ctx& c;
  CDims& D;
  CLayout& L;
  COptions& o;
  const ProblemIn& in;
  double* ws;

  // scalar state (wave-uniform)
  double sf, mu, tau, dw_last;
  double theta_min, theta_max;
  int n_factor;
  bool use_ric = false;
  // Inertia scan (factor_ic, HTP_IC_SCAN): while a trial factorization's local sweep has its blocks loaded, a
  // block with the wrong inertia is re-factored at the next trial values of delta_w until it has the right one;
  // ic_skip = how many more delta_w increments factor_ic may take at once (every skipped trial is known to fail
  // on that block, with no zero pivot) -- the same delta_w sequence and the same accepted factorization.
  bool ic_scan = false;
  int ic_skip = 0;
  // HTP_FUSE_RHS: the Newton step's local right-hand-side sweep runs inside the factor sweep (the blocks are
  // built and factored there already); kkt_solve then skips it.  The same per-block arithmetic: bit-identical.
  bool fuse_rhs = false;
  // HTP_BWD_FUSE: the last factorization also ran the Newton right-hand side's Riccati backward pass (V and the
  // backward half of X are in the workspace); the next fused-rhs kkt_solve starts at the forward pass
  bool bwd_ready = false;
  // restoration phase (oracle/ipm.py RestoProblem): the iterate is [x, R] with R = [n_c | p_c | n_d | p_d] >= 0,
  // constraints c(x) + n_c - p_c = 0, d(x) + n_d - p_d - s = 0, objective rho sum R + eta/2 |D_R (x - x_R)|^2
  bool rs = false;
  double eta = 0.0;     // resto_proximity_weight * sqrt(mu) (restoration phase)
  int nR = 0;           // 2 mc + 2 md
  // objective factor of the Hessian: sf, or 0 in the restoration phase
  HTP_HD HTP_FI double hsf() const { return rs ? 0.0 : sf; }
  long long cyc[8];
#ifdef HTP_KKT_PROF  // experiments: KKT-solve sub-phases (local rhs sweep, stage Riccati solve, local back sweep)
  // HTP_KKT_PROF=2: finer -- rhs sweep, stage rhs assembly, Riccati backward pass, forward pass, scatter, back
  // sweep, and the number of KKT solves (reported in Result::cyc 0-3, 5-7)
  long long kprof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define HTP_KPROF(k, t) do { const long long t_ = c.clock(); kprof[k] += t_ - (t); (t) = t_; } while (0)
#else
#define HTP_KPROF(k, t) do { } while (0)
#endif
#ifdef HTP_LPROF  // experiments: the local factor sweep -- pass 1 / pass 2 / inertia-scan cycles, trip counts (Result::cyc)
  // HTP_LPROF=2: pass 2 split instead of pass 1 and the trip counts: build_local (slot 0), Bunch-Kaufman factor
  // (slot 2), the right-hand-side solves with their fills and outputs (slot 3)
  mutable long long lprof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  mutable long long lp2_t = 0;
#define HTP_LP(k, v) do { lprof[k] += (v); } while (0)
#if HTP_LPROF == 2
#define HTP_LP1(k, v) do { } while (0)
#define HTP_LP2(k, v) do { lprof[k] += (v); } while (0)
#else
#define HTP_LP1(k, v) do { lprof[k] += (v); } while (0)
#define HTP_LP2(k, v) do { } while (0)
#endif
#else
#define HTP_LP(k, v) do { } while (0)
#define HTP_LP1(k, v) do { } while (0)
#define HTP_LP2(k, v) do { } while (0)
#endif
#ifdef HTP_PROF_ON  // experiments: sub-step cycle counters of the stage chain (tools/build_variants.py)
  long long pcyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long spcyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // solve passes: ring fills / stage steps (tools/micro)
  long long tprof = 0, tsprof = 0;
#define HTP_PROF(k) do { const long long t_ = c.clock(); pcyc[k] += t_ - tprof; tprof = t_; } while (0)
#define HTP_PROF0() do { tprof = c.clock(); } while (0)
#define HTP_SPROF(k) do { const long long t_ = c.clock(); spcyc[k] += t_ - tsprof; tsprof = t_; } while (0)
#define HTP_SPROF0() do { tsprof = c.clock(); } while (0)
#else
#define HTP_PROF(k) do { } while (0)
#define HTP_PROF0() do { } while (0)
#define HTP_SPROF(k) do { } while (0)
#define HTP_SPROF0() do { } while (0)
#endif
  // filter (wave-uniform): entries live in per-wave LDS (c.lds + FILT_OFF)
  static constexpr int FMAX = 64;
  static constexpr int FILT_OFF = 4 * NBMAX * NBMAX + 8;
  ld* f_th;
  ld* f_ph;
  int nfilt;

  HTP_HD HTP_FI ObcaSolver(Ctx& c_, CDims& D_, CLayout& L_, COptions& o_, const ProblemIn& in_, double* ws_)
      : c(c_), D(D_), L(L_), o(o_), in(in_), ws(ws_) {
    f_th = c.lds + FILT_OFF;
    f_ph = c.lds + FILT_OFF + FMAX;
  }

  HTP_HD HTP_FI gd* A(int64_t off) const { return (gd*)(ws + off); }
  HTP_HD HTP_FI static const gd* gp(const double* p) { return (const gd*)p; }
  // a wave-uniform pointer as the compiler's uniform value (scalar registers on the device)
  template <class T>
  HTP_HD HTP_FI static T* uptr(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (T*)(((unsigned long long)hi << 32) | lo);
#else
    return p;
#endif
  }
  // HTP_HOIST: what ring_fill reads besides the stage records
  struct RingSrc { const gd* LD; const gd* fac; int N, nb, lane; bool relax; };
  HTP_HD HTP_FI RingSrc ring_src() const {
    return RingSrc{uptr((const gd*)A(L.LD)), uptr((const gd*)A(L.fac)), c.uniform_i(D.N), c.uniform_i(D.nb), (int)c.lane,
                   c.uniform_i(ric_relax ? 1 : 0) != 0};
  }
  HTP_HD HTP_FI double par(int k) const { return gp(in.par)[k]; }
  HTP_HD HTP_FI double tauv(const gd* x, int i) const { return D.topt ? x[D.oTAU + i] : 1.0; }
  // Upper bounds that exist (HTP_UB_SKIP): optimizer.py's multipliers mu, lambda ([oMU, oTAU), :292-354) have a
  // lower bound only and the distance rows c3 (odd inequality rows, :414-425) no upper bound, so x_U / d_U stay
  // +inf and z_U / dz_U / v_U stay exactly 0 for the whole solve (never relaxed, corrected or stepped).  Passes
  // over n and m_in read those arrays only where the bound exists; every value they skip is that constant.
  HTP_HD HTP_FI bool ubx(int q) const { return PT || !HTP_UB_SKIP || q < D.oMU || q >= D.oTAU; }
  HTP_HD HTP_FI bool ubs(int r) const { return PT || !HTP_UB_SKIP || (r & 1) == 0; }

  // Lane-blocked sweep over [0, n): per trip a lane takes SW_U indices q_k = b + k*width.
  // ld(q, k) gathers element q into register slot k with the index clamped into range,
  // so all loads of a trip issue before any use (a plain unrolled loop puts a bound
  // check, and the elementwise bound tests, between them and waits one memory round trip
  // per element).  op(q, k) then consumes the in-range slots in ascending k -- the
  // plain loop's per-lane order, so reductions are bit-identical.
  static constexpr int SW_U = HTP_SWEEP_U;
  template <class Ld, class Op>
  HTP_HD HTP_FI void sweep(int n, Ld&& ld_, Op&& op_) const {
    for (int b = c.lane; b < n; b += SW_U * c.width) {
      HTP_PRAGMA(unroll)
      for (int k = 0; k < SW_U; ++k) { const int q = b + k * c.width; ld_(q < n ? q : n - 1, k); }
      HTP_PRAGMA(unroll)
      for (int k = 0; k < SW_U; ++k) { const int q = b + k * c.width; if (q < n) op_(q, k); }
    }
  }

  // pair p -> (i, m, n) and variable offsets
  HTP_HD HTP_FI void pair_index(int p, int& i, int& m, int& n, int& mu0, int& la0) const {
    if constexpr (PT) {  // block p = (obstacle m, step i), obstacle-major
      m = p / D.N;
      i = p - m * D.N;
      n = 0;
      la0 = D.oLAM + D.N * D.offo[m] + i * D.eo[m];
      mu0 = la0;
      return;
    }
    n = p % D.K;
    int t = p / D.K;
    m = t % D.M;
    i = t / D.M;
    mu0 = D.oMU + i * D.mu_count + m * D.TEb + D.offb[n];
    la0 = D.oLAM + i * D.lam_count + n * D.TEo + D.offo[m];
  }

  // local block q of stage i, and the number of local blocks per stage
  HTP_HD HTP_FI int blk(int i, int q) const { return PT ? q * D.N + i : i * (D.M * D.K) + q; }
  HTP_HD HTP_FI int blocks_per_stage() const { return PT ? D.M : D.M * D.K; }

  // stage w = [x_i (5), u_i (2), tau_i]
  HTP_HD HTP_FI void stage_w(const gd* x, int i, double* w) const {
    for (int k = 0; k < NS; ++k) w[k] = x[NS * i + k];
    w[5] = x[D.oU + NC * i];
    w[6] = x[D.oU + NC * i + 1];
    if (D.topt) w[7] = x[D.oTAU + i];
  }
  HTP_HD HTP_FI void dynF(const double* w, double* F) const {
    if (D.topt) dyn_F_rk2(w, par(P_DT), par(P_WHEELBASE), F);
    else dyn_F_euler(w, par(P_DT), par(P_WHEELBASE), F);
  }
  HTP_HD HTP_FI void dynJ(const double* w, double* J) const {
    if (D.topt) dyn_J_rk2(w, par(P_DT), par(P_WHEELBASE), J);
    else dyn_J_euler(w, par(P_DT), par(P_WHEELBASE), J);
  }
  // The same Jacobian at a fixed row stride of 8 (J8[k * 8 + j], j < D.nw; the rest 0): constant offsets for any
  // nw, so the array stays in registers (a run-time stride D.nw sends it to scratch memory).
  HTP_HD HTP_FI void dynJ8(const double* w, double* J8) const {
#if !HTP_J8
    double J[40];
    dynJ(w, J);
    for (int k = 0; k < NS; ++k)
      for (int j = 0; j < 8; ++j) J8[k * 8 + j] = j < D.nw ? J[k * D.nw + j] : 0.0;
    return;
#endif
    if (D.topt) {
      dyn_J_rk2(w, par(P_DT), par(P_WHEELBASE), J8);
    } else {
      double J7[NS * 7];
      dyn_J_euler(w, par(P_DT), par(P_WHEELBASE), J7);
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) J8[k * 8 + j] = j < 7 ? J7[k * 7 + j] : 0.0;
    }
  }
  HTP_HD HTP_FI void dynH(const double* w, const double* y, double* H) const {
    if (D.topt) dyn_H_rk2(w, par(P_DT), par(P_WHEELBASE), y, H);
    else dyn_H_euler(w, par(P_DT), par(P_WHEELBASE), y, H);
  }

  // ======================================================== objective
  // f (unscaled) -- optimizer.py:447-473
  HTP_HD HTP_FI double stage_obj(const gd* x, int i) const {
    const int N = D.N;
    const double dT = par(P_DT);
    double f = 0.0;
    if constexpr (PT) {  // optimizer_points.py generate_object :193-227
      if (i < N - 1) {
        if (i < N - 2) {
          const double dsr = x[D.oU + NC * (i + 1) + 1] - x[D.oU + NC * i + 1];
          const double dv = x[D.oU + NC * (i + 1)] - x[D.oU + NC * i];
          f += dsr * dsr + dv * dv;
        }
        f += sq(x[NS * i + 2] * dT) * 20.0;
      }
      return f;
    }
    if (i < N - 1) {
      const double h = dT * tauv(x, i);
      const double a = x[D.oU + NC * i], w = x[D.oU + NC * i + 1];
      if (D.topt) f += h * par(P_W11);
      f += a * (par(P_Q00) * a + par(P_Q01) * w) + w * (par(P_Q10) * a + par(P_Q11) * w);
      if (i < N - 2) {
        const double ja = (x[D.oU + NC * (i + 1)] - a) / h, jw = (x[D.oU + NC * (i + 1) + 1] - w) / h;
        f += ja * (par(P_R00) * ja + par(P_R01) * jw) + jw * (par(P_R10) * ja + par(P_R11) * jw);
      }
      f += sq(x[NS * i + 2] * h) * par(P_W00);
    }
    if (i == 0)
      for (int k = 0; k < NS; ++k) f += 5000.0 * sq(x[D.oS + k]);
    return f;
  }
  HTP_HD HTP_PHASE double eval_f(const gd* x) const {
    double f = 0.0, v_[SW_U];
    sweep(D.N, [&](int i, int k) { v_[k] = stage_obj(x, i); }, [&](int, int k) { f += v_[k]; });
    return c.sum(f);
  }
  // scaled gradient (sf * grad f) into g (all n entries written)
  HTP_HD HTP_PHASE void eval_grad_f(const gd* x, gd* g, double scale) const {
    const int N = D.N;
    const double dT = par(P_DT);
    const double Qs00 = 2 * par(P_Q00), Qs01 = par(P_Q01) + par(P_Q10), Qs11 = 2 * par(P_Q11);
    const double Rs00 = 2 * par(P_R00), Rs01 = par(P_R01) + par(P_R10), Rs11 = 2 * par(P_R11);
    HTP_UNROLL
    for (int q = c.lane; q < D.n; q += c.width) g[q] = 0.0;
    c.sync();
    if constexpr (PT) {
      for (int i = c.lane; i < N - 1; i += c.width) {
        const double a = x[D.oU + NC * i], w = x[D.oU + NC * i + 1];
        double ga = 0.0, gw = 0.0;
        if (i < N - 2) {
          ga -= 2.0 * (x[D.oU + NC * (i + 1)] - a);
          gw -= 2.0 * (x[D.oU + NC * (i + 1) + 1] - w);
        }
        if (i >= 1) {
          ga += 2.0 * (a - x[D.oU + NC * (i - 1)]);
          gw += 2.0 * (w - x[D.oU + NC * (i - 1) + 1]);
        }
        g[NS * i + 2] = scale * (40.0 * x[NS * i + 2] * dT * dT);
        g[D.oU + NC * i] = scale * ga;
        g[D.oU + NC * i + 1] = scale * gw;
      }
      c.sync();
      return;
    }
    for (int i = c.lane; i < N - 1; i += c.width) {
      const double tau = tauv(x, i), h = dT * tau;
      const double a = x[D.oU + NC * i], w = x[D.oU + NC * i + 1];
      double ga = Qs00 * a + Qs01 * w, gw = Qs01 * a + Qs11 * w;
      double gt = D.topt ? dT * par(P_W11) : 0.0;
      if (i < N - 2) {
        const double da = x[D.oU + NC * (i + 1)] - a, dw_ = x[D.oU + NC * (i + 1) + 1] - w;
        ga -= (Rs00 * da + Rs01 * dw_) / (h * h);
        gw -= (Rs01 * da + Rs11 * dw_) / (h * h);
        const double Jv = (da * (par(P_R00) * da + par(P_R01) * dw_) + dw_ * (par(P_R10) * da + par(P_R11) * dw_)) / (h * h);
        gt += -2.0 * Jv / tau;
      }
      if (i >= 1) {
        const double hp = dT * tauv(x, i - 1);
        const double da = a - x[D.oU + NC * (i - 1)], dw_ = w - x[D.oU + NC * (i - 1) + 1];
        ga += (Rs00 * da + Rs01 * dw_) / (hp * hp);
        gw += (Rs01 * da + Rs11 * dw_) / (hp * hp);
      }
      const double v = x[NS * i + 2];
      g[NS * i + 2] = scale * 2.0 * par(P_W00) * v * h * h;
      if (D.topt) gt += 2.0 * par(P_W00) * v * v * dT * dT * tau;
      g[D.oU + NC * i] = scale * ga;
      g[D.oU + NC * i + 1] = scale * gw;
      if (D.topt) g[D.oTAU + i] = scale * gt;
    }
    if (c.lane == 0)
      for (int k = 0; k < NS; ++k) g[D.oS + k] = scale * 10000.0 * x[D.oS + k];
    c.sync();
  }

  // ======================================================== constraints
  // scaled c (equality) and d (inequality) at x (optimizer.py:356-425)
  HTP_HD HTP_FI void pair_geom(const gd* x, int p, double* w, double& cs, double& sn,
                        int& i, int& m, int& n, int& mu0, int& la0) const {
    pair_index(p, i, m, n, mu0, la0);
    const int em = D.eo[m];
    const gd* Am = gp(in.obsA) + 2 * D.offo[m];
    // loads first (indices clamped), then the em-term sums in the plain order
    double a0[EM_], a1[EM_], lx[EM_];
    for (int j = 0; j < EM_; ++j) {
      const int jj = j < em ? j : 0;
      a0[j] = Am[2 * jj];
      a1[j] = Am[2 * jj + 1];
      lx[j] = x[la0 + jj];
    }
    const double th = x[NS * i + 3];
    w[0] = w[1] = 0.0;
    for (int j = 0; j < EM_; ++j) {
      if (j < em) {
        w[0] += a0[j] * lx[j];
        w[1] += a1[j] * lx[j];
      }
    }
    dyn_sincos(th, sn, cs);
  }

  // point formulation: obstacle halfspaces, lam, w = A'lam and the pose of block p
  struct PtGeom {
    double A0[EM_], A1[EM_], bb[EM_], lam[EM_];
    double w0, w1, cs, sn, tx, ty;
    int i, m, em, la0;
  };
  HTP_HD HTP_FI void pt_geom(const gd* x, int p, PtGeom& G) const {
    int n_, mu0_;
    pair_index(p, G.i, G.m, n_, mu0_, G.la0);
    G.em = D.eo[G.m];
    const gd* Am = gp(in.obsA) + 2 * D.offo[G.m];
    const gd* bm = gp(in.obsb) + D.offo[G.m];
    G.w0 = 0.0;
    G.w1 = 0.0;
    for (int j = 0; j < EM_; ++j) {
      const bool on = j < G.em;
      G.A0[j] = on ? Am[2 * j] : 0.0;
      G.A1[j] = on ? Am[2 * j + 1] : 0.0;
      G.bb[j] = on ? bm[j] : 0.0;
      G.lam[j] = on ? x[G.la0 + j] : 0.0;
      G.w0 += G.A0[j] * G.lam[j];
      G.w1 += G.A1[j] * G.lam[j];
    }
    const double th = x[NS * G.i + 3];
    dyn_sincos(th, G.sn, G.cs);
    G.tx = x[NS * G.i];
    G.ty = x[NS * G.i + 1];
  }
  // hull vertex k of the body frame: moved vertex vt = R v + t, dR/dth v, R v
  HTP_HD HTP_FI void pt_vertex(const PtGeom& G, int k, double* vt, double* dv, double* rv) const {
    const gd* V = gp(in.bodyG);
    const double v0 = V[2 * k], v1 = V[2 * k + 1];
    rv[0] = G.cs * v0 - G.sn * v1;
    rv[1] = G.sn * v0 + G.cs * v1;
    vt[0] = rv[0] + G.tx;
    vt[1] = rv[1] + G.ty;
    dv[0] = -G.sn * v0 - G.cs * v1;
    dv[1] = G.cs * v0 - G.sn * v1;
  }

  HTP_HD HTP_FI void pair_cons(const gd* x, int p, double* out4) const {
    double w[2], cs, sn;
    int i, m, n, mu0, la0;
    pair_geom(x, p, w, cs, sn, i, m, n, mu0, la0);
    const int em = D.eo[m], en = D.eb[n];
    const gd* Am = gp(in.obsA) + 2 * D.offo[m];
    const gd* bm = gp(in.obsb) + D.offo[m];
    const gd* Gn = gp(in.bodyG) + 2 * D.offb[n];
    const gd* gn = gp(in.bodyg) + D.offb[n];
    // loads first (indices clamped), then the plain-order sums over the en / em live entries
    double muj[EN_], g0[EN_], g1[EN_], gj[EN_];
    for (int j = 0; j < EN_; ++j) {
      const int jj = j < en ? j : 0;
      muj[j] = x[mu0 + jj]; g0[j] = Gn[2 * jj]; g1[j] = Gn[2 * jj + 1]; gj[j] = gn[jj];
    }
    double a0[EM_], a1[EM_], bj[EM_], lj[EM_];
    for (int j = 0; j < EM_; ++j) {
      const int jj = j < em ? j : 0;
      a0[j] = Am[2 * jj]; a1[j] = Am[2 * jj + 1]; bj[j] = bm[jj]; lj[j] = x[la0 + jj];
    }
    const double tx = x[NS * i], ty = x[NS * i + 1];
    double c2a = cs * w[0] + sn * w[1], c2b = -sn * w[0] + cs * w[1], c3 = 0.0;
    for (int j = 0; j < EN_; ++j) {
      if (j < en) {
        c2a += g0[j] * muj[j];
        c2b += g1[j] * muj[j];
        c3 -= gj[j] * muj[j];
      }
    }
    for (int j = 0; j < EM_; ++j)
      if (j < em) c3 += (a0[j] * tx + a1[j] * ty - bj[j]) * lj[j];
    out4[0] = w[0] * w[0] + w[1] * w[1];
    out4[1] = c2a;
    out4[2] = c2b;
    out4[3] = c3;
  }

  HTP_HD HTP_PHASE void eval_cons(const gd* x, gd* cc, gd* dd) const {
    const int N = D.N;
    const gd* scE = A(L.scE);
    const gd* scI = A(L.scI);
    for (int i = c.lane; i < N; i += c.width) {
#if HTP_HOIST
      // every load of the stage before its first store (a load issued after a store waits for it)
      double e0[NS], x0[NS], t0[NS];
      if (i == 0)
        for (int k = 0; k < NS; ++k) { e0[k] = scE[k]; x0[k] = x[k]; t0[k] = gp(in.traj)[k]; }
      if (i < N - 1) {
        double w[8], F[5], ek[NS], xk[NS];
        stage_w(x, i, w);
        for (int k = 0; k < NS; ++k) {
          ek[k] = scE[D.eDyn + NS * i + k];
          xk[k] = x[NS * (i + 1) + k];
        }
        dynF(w, F);
        if (i == 0)
          for (int k = 0; k < NS; ++k) cc[k] = e0[k] * (x0[k] - t0[k]);
        for (int k = 0; k < NS; ++k) cc[D.eDyn + NS * i + k] = ek[k] * (xk[k] - F[k]);
      } else {
#else
      if (i == 0)
        for (int k = 0; k < NS; ++k) cc[k] = scE[k] * (x[k] - gp(in.traj)[k]);
      if (i < N - 1) {
        double w[8], F[5];
        stage_w(x, i, w);
        dynF(w, F);
        for (int k = 0; k < NS; ++k) {
          const int r = D.eDyn + NS * i + k;
          cc[r] = scE[r] * (x[NS * (i + 1) + k] - F[k]);
        }
      } else {
#endif
#if HTP_HOIST
        double ek[NS], xk[NS], tk[NS], sk[NS];
        for (int k = 0; k < NS; ++k) {
          ek[k] = scE[D.eTerm + k];
          xk[k] = x[NS * i + k];
          tk[k] = gp(in.traj)[NS * i + k];
          sk[k] = PT ? 0.0 : x[D.oS + k];
        }
        for (int k = 0; k < NS; ++k) {
          if constexpr (PT) cc[D.eTerm + k] = ek[k] * (xk[k] - tk[k]);
          else cc[D.eTerm + k] = ek[k] * (xk[k] - tk[k] + sk[k]);
        }
#else
        for (int k = 0; k < NS; ++k) {
          const int r = D.eTerm + k;
          if constexpr (PT) cc[r] = scE[r] * (x[NS * i + k] - gp(in.traj)[NS * i + k]);
          else cc[r] = scE[r] * (x[NS * i + k] - gp(in.traj)[NS * i + k] + x[D.oS + k]);
        }
#endif
      }
    }
    if constexpr (PT) {
      const int KV = D.KV;
      for (int p = c.lane; p < D.P; p += c.width) {
        PtGeom G;
        pt_geom(x, p, G);
        for (int k = 0; k < KV; ++k) {
          double vt[2], dv[2], rv[2];
          pt_vertex(G, k, vt, dv, rv);
          double dist = 0.0;
          for (int j = 0; j < EM_; ++j) dist += (G.A0[j] * vt[0] + G.A1[j] * vt[1] - G.bb[j]) * G.lam[j];
          const int r = 2 * (KV * p + k);
          dd[r] = scI[r] * (G.w0 * G.w0 + G.w1 * G.w1);
          dd[r + 1] = scI[r + 1] * dist;
        }
      }
      c.sync();
      return;
    }
    for (int p = c.lane; p < D.P; p += c.width) {
      double v[4];
      const int re = D.ePair + 2 * p;
#if HTP_HOIST
      const double sa = scE[re], sb = scE[re + 1], s1 = scI[2 * p], s3 = scI[2 * p + 1];
      pair_cons(x, p, v);
      cc[re] = sa * v[1];
      cc[re + 1] = sb * v[2];
      dd[2 * p] = s1 * v[0];
      dd[2 * p + 1] = s3 * v[3];
#else
      pair_cons(x, p, v);
      cc[re] = scE[re] * v[1];
      cc[re + 1] = scE[re + 1] * v[2];
      dd[2 * p] = scI[2 * p] * v[0];
      dd[2 * p + 1] = scI[2 * p + 1] * v[3];
#endif
    }
    c.sync();
  }

  // J_c' yc + J_d' yd (x part) into out (scaled rows; yc, yd multipliers of scaled rows)
  HTP_HD HTP_PHASE void eval_jt(const gd* x, const gd* yc, const gd* yd, gd* out) {
    const int N = D.N;
    const gd* scE = A(L.scE);
    const gd* scI = A(L.scI);
    gd* pr = A(L.pairR);
    HTP_UNROLL
    for (int q = c.lane; q < D.n; q += c.width) out[q] = 0.0;
    c.sync();
    if constexpr (PT) {
      const int KV = D.KV;
      for (int p = c.lane; p < D.P; p += c.width) {
        PtGeom G;
        pt_geom(x, p, G);
        double ol[EM_];
        for (int j = 0; j < EM_; ++j) ol[j] = 0.0;
        double px = 0.0, py = 0.0, pt = 0.0;
        for (int k = 0; k < KV; ++k) {
          const int r = 2 * (KV * p + k);
          const double y1 = scI[r] * yd[r], y3 = scI[r + 1] * yd[r + 1];
          double vt[2], dv[2], rv[2];
          pt_vertex(G, k, vt, dv, rv);
          for (int j = 0; j < EM_; ++j)
            ol[j] += 2.0 * (G.A0[j] * G.w0 + G.A1[j] * G.w1) * y1 + (G.A0[j] * vt[0] + G.A1[j] * vt[1] - G.bb[j]) * y3;
          px += G.w0 * y3;
          py += G.w1 * y3;
          pt += (G.w0 * dv[0] + G.w1 * dv[1]) * y3;
        }
        for (int j = 0; j < EM_; ++j)
          if (j < G.em) out[G.la0 + j] = ol[j];
        pr[3 * p + 0] = px;
        pr[3 * p + 1] = py;
        pr[3 * p + 2] = pt;
      }
    } else
    for (int p = c.lane; p < D.P; p += c.width) {
      double w[2], cs, sn;
      int i, m, n, mu0, la0;
      pair_geom(x, p, w, cs, sn, i, m, n, mu0, la0);
      const int em = D.eo[m], en = D.eb[n];
      const gd* Am = gp(in.obsA) + 2 * D.offo[m];
      const gd* bm = gp(in.obsb) + D.offo[m];
      const gd* Gn = gp(in.bodyG) + 2 * D.offb[n];
      const gd* gn = gp(in.bodyg) + D.offb[n];
      const int re = D.ePair + 2 * p;
      // loads first (indices clamped), stores after
      double g0[EN_], g1[EN_], gj[EN_];
      for (int j = 0; j < EN_; ++j) {
        const int jj = j < en ? j : 0;
        g0[j] = Gn[2 * jj]; g1[j] = Gn[2 * jj + 1]; gj[j] = gn[jj];
      }
      double a0v[EM_], a1v[EM_], bj[EM_];
      for (int j = 0; j < EM_; ++j) {
        const int jj = j < em ? j : 0;
        a0v[j] = Am[2 * jj]; a1v[j] = Am[2 * jj + 1]; bj[j] = bm[jj];
      }
      const double ya = scE[re] * yc[re], yb = scE[re + 1] * yc[re + 1];
      const double y1 = scI[2 * p] * yd[2 * p], y3 = scI[2 * p + 1] * yd[2 * p + 1];
      const double tx = x[NS * i], ty = x[NS * i + 1];
      for (int j = 0; j < EN_; ++j)
        if (j < en) out[mu0 + j] = g0[j] * ya + g1[j] * yb - gj[j] * y3;
      for (int j = 0; j < EM_; ++j) {
        if (j < em) {
          const double a0 = a0v[j], a1 = a1v[j];
          out[la0 + j] = (cs * a0 + sn * a1) * ya + (-sn * a0 + cs * a1) * yb + 2.0 * (a0 * w[0] + a1 * w[1]) * y1 +
                         (a0 * tx + a1 * ty - bj[j]) * y3;
        }
      }
      pr[3 * p + 0] = w[0] * y3;
      pr[3 * p + 1] = w[1] * y3;
      pr[3 * p + 2] = (-sn * w[0] + cs * w[1]) * ya + (-cs * w[0] - sn * w[1]) * yb;
    }
    c.sync();
    const int MK = blocks_per_stage();
    for (int i = c.lane; i < N; i += c.width) {
      double gx[5] = {0, 0, 0, 0, 0};
      if (i == 0)
        for (int k = 0; k < NS; ++k) gx[k] += scE[k] * yc[k];
      else
        for (int k = 0; k < NS; ++k) gx[k] += scE[D.eDyn + NS * (i - 1) + k] * yc[D.eDyn + NS * (i - 1) + k];
      // every store of the stage goes after its last load (the pairR gathers)
      double tt[NS], gw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (i == N - 1) {
        for (int k = 0; k < NS; ++k) {
          tt[k] = scE[D.eTerm + k] * yc[D.eTerm + k];
          gx[k] += tt[k];
        }
      } else {
        double w[8], J[40], yy[5];
        stage_w(x, i, w);
        dynJ8(w, J);
        for (int k = 0; k < NS; ++k) yy[k] = scE[D.eDyn + NS * i + k] * yc[D.eDyn + NS * i + k];
#pragma unroll
        for (int k = 0; k < NS; ++k)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < D.nw) gw[j] -= J[k * 8 + j] * yy[k];
        for (int k = 0; k < NS; ++k) gx[k] += gw[k];
      }
      for (int q = 0; q < MK; ++q) {
        const int p = blk(i, q);
        gx[0] += pr[3 * p];
        gx[1] += pr[3 * p + 1];
        gx[3] += pr[3 * p + 2];
      }
      if (i == N - 1) {
        if constexpr (!PT)
          for (int k = 0; k < NS; ++k) out[D.oS + k] = tt[k];
      } else {
        out[D.oU + NC * i] = gw[5];
        out[D.oU + NC * i + 1] = gw[6];
        if (D.topt) out[D.oTAU + i] = gw[7];
      }
      for (int k = 0; k < NS; ++k) out[NS * i + k] = gx[k];
    }
    c.sync();
  }

  // ======================================================== setup
  HTP_HD HTP_FI void set_bounds_and_x0() {
    const int N = D.N;
    gd* x = A(L.x);
    gd* xL = A(L.xL);
    gd* xU = A(L.xU);
    const double vmax = dabs(par(P_MAXV)), smax = dabs(par(P_MAXSTEER));
    const double amax = dabs(par(P_MAXACC)), wmax = dabs(par(P_MAXSR));
    const double twopi = 2.0 * M_PI;
    HTP_UNROLL
    for (int q = c.lane; q < D.n; q += c.width) {
      double lo = -HTP_INF, hi = HTP_INF, v0 = 0.0;
      if (q < D.oU) {
        const int i = q / NS, k = q % NS;
        v0 = gp(in.traj)[q];
        if (k == 0) { lo = par(P_XLO); hi = par(P_XHI); }
        if (k == 1) { lo = par(P_YLO); hi = par(P_YHI); }
        if (k == 2) { lo = -vmax; hi = vmax; }
        if (k == 3) { lo = -twopi; hi = twopi; }
        if (k == 4) { lo = -smax; hi = smax; }
        (void)i;
      } else if (q < D.oMU) {
        const int j = q - D.oU;
        v0 = in.init_u ? gp(in.init_u)[j] : 0.0;
        if (j % 2 == 0) { lo = -amax; hi = amax; } else { lo = -wmax; hi = wmax; }
      } else if (q < D.oLAM) {
        v0 = in.init_mu ? gp(in.init_mu)[q - D.oMU] : 0.1;
        lo = 0.0;
      } else if (q < D.oTAU) {
        if constexpr (PT) {  // optimizer_points.py:101-104 (init_dual_var unused), :252-255
          v0 = 0.1;
          lo = 0.0;
          hi = 100000.0;
        } else {
          v0 = in.init_la ? gp(in.init_la)[q - D.oLAM] : 0.1;
          lo = 0.0;
        }
      } else if (q < D.oS) {
        v0 = 1.0;
        lo = 0.05 / par(P_DT);
        hi = 1.0;
      }
      x[q] = v0;
      xL[q] = lo;
      xU[q] = hi;
    }
    c.sync();
  }

  // gradient-based scaling at the user x0 (IPOPT nlp_scaling_method default)
  HTP_HD HTP_FI void compute_scaling() {
    const int N = D.N;
    const gd* x = A(L.x);
    gd* g = A(L.gf);
    eval_grad_f(x, g, 1.0);
    double mg = 0.0;
    HTP_UNROLL
    for (int q = c.lane; q < D.n; q += c.width) mg = dmax(mg, dabs(g[q]));
    mg = c.maxv(mg);
    sf = mg > o.scaling_max_gradient ? dmax(o.scaling_min_value, o.scaling_max_gradient / mg) : 1.0;
    gd* scE = A(L.scE);
    gd* scI = A(L.scI);
    auto scl = [&](double rm) {
      return rm > o.scaling_max_gradient ? dmax(o.scaling_min_value, o.scaling_max_gradient / rm) : 1.0;
    };
    for (int i = c.lane; i < N; i += c.width) {
      if (i == 0)
        for (int k = 0; k < NS; ++k) scE[k] = 1.0;
      if (i < N - 1) {
        double w[8], J[40];
        stage_w(x, i, w);
        dynJ8(w, J);
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          double rm = 1.0;  // +1 at x_{i+1,k}
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < D.nw) rm = dmax(rm, dabs(J[k * 8 + j]));
          scE[D.eDyn + NS * i + k] = scl(rm);
        }
      } else {
        for (int k = 0; k < NS; ++k) scE[D.eTerm + k] = 1.0;
      }
    }
    if constexpr (PT) {
      const int KV = D.KV;
      for (int p = c.lane; p < D.P; p += c.width) {
        PtGeom G;
        pt_geom(x, p, G);
        double r1 = 0.0;
        for (int j = 0; j < EM_; ++j) r1 = dmax(r1, dabs(2.0 * (G.A0[j] * G.w0 + G.A1[j] * G.w1)));
        for (int k = 0; k < KV; ++k) {
          double vt[2], dv[2], rv[2];
          pt_vertex(G, k, vt, dv, rv);
          double r3 = dmax(dabs(G.w0), dabs(G.w1));
          r3 = dmax(r3, dabs(G.w0 * dv[0] + G.w1 * dv[1]));
          for (int j = 0; j < EM_; ++j) r3 = dmax(r3, dabs(G.A0[j] * vt[0] + G.A1[j] * vt[1] - G.bb[j]));
          const int r = 2 * (KV * p + k);
          scI[r] = scl(r1);
          scI[r + 1] = scl(r3);
        }
      }
      c.sync();
      return;
    }
    for (int p = c.lane; p < D.P; p += c.width) {
      double w[2], cs, sn;
      int i, m, n, mu0, la0;
      pair_geom(x, p, w, cs, sn, i, m, n, mu0, la0);
      const int em = D.eo[m], en = D.eb[n];
      const gd* Am = gp(in.obsA) + 2 * D.offo[m];
      const gd* bm = gp(in.obsb) + D.offo[m];
      const gd* Gn = gp(in.bodyG) + 2 * D.offb[n];
      const gd* gn = gp(in.bodyg) + D.offb[n];
      double r1 = 0, ra = 0, rb = 0, r3 = 0;
      const double tx = x[NS * i], ty = x[NS * i + 1];
      for (int j = 0; j < em; ++j) {
        const double a0 = Am[2 * j], a1 = Am[2 * j + 1];
        r1 = dmax(r1, dabs(2.0 * (a0 * w[0] + a1 * w[1])));
        ra = dmax(ra, dabs(cs * a0 + sn * a1));
        rb = dmax(rb, dabs(-sn * a0 + cs * a1));
        r3 = dmax(r3, dabs(a0 * tx + a1 * ty - bm[j]));
      }
      for (int j = 0; j < en; ++j) {
        ra = dmax(ra, dabs(Gn[2 * j]));
        rb = dmax(rb, dabs(Gn[2 * j + 1]));
        r3 = dmax(r3, dabs(gn[j]));
      }
      ra = dmax(ra, dabs(-sn * w[0] + cs * w[1]));
      rb = dmax(rb, dabs(-cs * w[0] - sn * w[1]));
      r3 = dmax(r3, dmax(dabs(w[0]), dabs(w[1])));
      scE[D.ePair + 2 * p] = scl(ra);
      scE[D.ePair + 2 * p + 1] = scl(rb);
      scI[2 * p] = scl(r1);
      scI[2 * p + 1] = scl(r3);
    }
    c.sync();
  }

  HTP_HD HTP_FI void relax_and_push() {
    gd* x = A(L.x);
    gd* xL = A(L.xL);
    gd* xU = A(L.xU);
    const double rf = o.bound_relax_factor;
    HTP_UNROLL
    for (int q = c.lane; q < D.n; q += c.width) {
      double lo = xL[q], hi = xU[q];
      const bool hl = finite_(lo), hu = finite_(hi);
      if (hl) lo -= rf * dmax(1.0, dabs(lo));
      if (hu) hi += rf * dmax(1.0, dabs(hi));
      xL[q] = lo;
      xU[q] = hi;
      x[q] = push(x[q], lo, hi, hl, hu);
    }
    c.sync();
  }

  HTP_HD HTP_FI double push(double v, double lo, double hi, bool hl, bool hu) const {
    double pl = hl ? o.bound_push * dmax(1.0, dabs(lo)) : 0.0;
    double pu = hu ? o.bound_push * dmax(1.0, dabs(hi)) : 0.0;
    if (hl && hu) {
      pl = dmin(pl, o.bound_frac * (hi - lo));
      pu = dmin(pu, o.bound_frac * (hi - lo));
    }
    if (hl) v = dmax(v, lo + pl);
    if (hu) v = dmin(v, hi - pu);
    return v;
  }

  // inequality-row bounds: c1 in [0,1], c3 in [dmin, inf), relaxed and scaled
  HTP_HD HTP_FI void set_slack_bounds_and_push() {
    const double rf = o.bound_relax_factor;
    double dmn = par(P_DMIN);
    gd* s = A(L.s);
    gd* dL = A(L.dL);
    gd* dU = A(L.dU);
    const gd* d = A(L.d);
    const gd* scI = A(L.scI);
    HTP_UNROLL
    for (int r = c.lane; r < D.md; r += c.width) {
      double lo, hi;
      if ((r & 1) == 0) { lo = 0.0; hi = 1.0; } else { lo = dmn; hi = PT ? 100000.0 : HTP_INF; }
      const bool hl = true, hu = finite_(hi);
      lo -= rf * dmax(1.0, dabs(lo));
      if (hu) hi += rf * dmax(1.0, dabs(hi));
      lo *= scI[r];
      if (hu) hi *= scI[r];
      dL[r] = lo;
      dU[r] = hi;
      s[r] = push(d[r], lo, hi, hl, hu);
    }
    c.sync();
  }

  // ======================================================== KKT assembly
  // mode_ls: least-squares multiplier system (W=0, identity x/s blocks)
  template <int EN, int EM>
  HTP_HD HTP_FI void build_local(LocalBlock<EN, EM>& B, int p, bool ls, double dw, double dc) const {
    const gd* x = A(L.x);
    double w[2], cs, sn;
    int i, m, n, mu0, la0;
    pair_geom(x, p, w, cs, sn, i, m, n, mu0, la0);
    const int em = D.eo[m], en = D.eb[n];
    const gd* Am = gp(in.obsA) + 2 * D.offo[m];
    const gd* bm = gp(in.obsb) + D.offo[m];
    const gd* Gn = gp(in.bodyG) + 2 * D.offb[n];
    const gd* gn = gp(in.bodyg) + D.offb[n];
    const gd* scE = A(L.scE);
    const gd* scI = A(L.scI);
    const gd* yc = A(L.yc);
    const gd* yd = A(L.yd);
    const gd* xL = A(L.xL);
    const gd* zL = A(L.zL);
    const gd* s = A(L.s);
    const gd* dL = A(L.dL);
    const gd* dU = A(L.dU);
    const gd* vL = A(L.vL);
    const gd* vU = A(L.vU);
    constexpr int NZ = LocalBlock<EN, EM>::NZ;
    constexpr int NL = LocalBlock<EN, EM>::NL;
    const int re = D.ePair + 2 * p;
    // every load of the block issues here, unconditionally (indices clamped into range)
    const int r1 = 2 * p, r3 = 2 * p + 1;
    const double vL1 = vL[r1], sv1 = s[r1], dL1 = dL[r1], vU1 = vU[r1], dU1 = dU[r1];
    const double vL3 = vL[r3], sv3 = s[r3], dL3 = dL[r3];
    double zq[NZ], xq[NZ], xlq[NZ];
    for (int j = 0; j < NZ; ++j) {
      const bool is_mu = j < EN;
      const int jj = is_mu ? j : j - EN;
      const bool on = is_mu ? (jj < en) : (jj < em);
      const int vi = on ? (is_mu ? mu0 + jj : la0 + jj) : mu0;
      zq[j] = zL[vi];
      xq[j] = x[vi];
      xlq[j] = xL[vi];
    }
    double Am0[EM], Am1[EM], bmj[EM];
    for (int j = 0; j < EM; ++j) {
      const int jj = j < em ? j : 0;
      Am0[j] = Am[2 * jj];
      Am1[j] = Am[2 * jj + 1];
      bmj[j] = bm[jj];
    }
    double Gn0[EN], Gn1[EN], gnj[EN];
    for (int j = 0; j < EN; ++j) {
      const int jj = j < en ? j : 0;
      Gn0[j] = Gn[2 * jj];
      Gn1[j] = Gn[2 * jj + 1];
      gnj[j] = gn[jj];
    }
    const double sa = scE[re], sb = scE[re + 1], s1 = scI[2 * p], s3 = scI[2 * p + 1];
    const double ya = sa * yc[re], yb = sb * yc[re + 1], y1 = s1 * yd[2 * p], y3 = s3 * yd[2 * p + 1];
    const double tx = x[NS * i], ty = x[NS * i + 1];
    // restoration phase: rows carry the eliminated n/p diagonal, variables the proximity term
    double ea = 0.0, eb = 0.0, e1 = 0.0, e3 = 0.0, prox[NZ];
    for (int j = 0; j < NZ; ++j) prox[j] = 0.0;
    if (rs) {
      const gd* eR = A(L.eR);
      ea = eR[re]; eb = eR[re + 1]; e1 = eR[D.mc + 2 * p]; e3 = eR[D.mc + 2 * p + 1];
      if (!ls) {
        const gd* dr = A(L.dr);
        for (int j = 0; j < NZ; ++j) {
          const bool is_mu = j < EN;
          const int jj = is_mu ? j : j - EN;
          const bool on = is_mu ? (jj < en) : (jj < em);
          const int vi = is_mu ? mu0 + jj : la0 + jj;
          prox[j] = on ? eta * dr[vi] * dr[vi] : 0.0;
        }
      }
    }
    // inequality slack elimination
    if (ls) {
      B.Ds1 = 1.0;
      B.Ds3 = 1.0;
    } else {
      B.Ds1 = vL1 / (sv1 - dL1) + vU1 / (dU1 - sv1) + dw;
      B.Ds3 = vL3 / (sv3 - dL3) + dw;
    }
    B.E1 = 1.0 / B.Ds1 + dc + e1;
    B.E3 = 1.0 / B.Ds3 + dc + e3;
    // Jacobian rows (z ordering: mu[0..EN), lam[0..EM)); padded entries are 0
    double Aw[EM], Atb[EM], A0[EM], A1[EM];
    for (int j = 0; j < EM; ++j) {
      const bool on = j < em;
      A0[j] = on ? Am0[j] : 0.0;
      A1[j] = on ? Am1[j] : 0.0;
      Aw[j] = A0[j] * w[0] + A1[j] * w[1];
      Atb[j] = on ? A0[j] * tx + A1[j] * ty - bmj[j] : 0.0;
    }
    double G0[EN], G1[EN], gg[EN];
    for (int j = 0; j < EN; ++j) {
      const bool on = j < en;
      G0[j] = on ? Gn0[j] : 0.0;
      G1[j] = on ? Gn1[j] : 0.0;
      gg[j] = on ? gnj[j] : 0.0;
    }
    for (int j = 0; j < EN; ++j) {
      B.J1[j] = 0.0;
      B.J3z[j] = -s3 * gg[j];
    }
    for (int j = 0; j < EM; ++j) {
      B.J1[EN + j] = s1 * 2.0 * Aw[j];
      B.J3z[EN + j] = s3 * Atb[j];
    }
    B.J3p[0] = s3 * w[0];
    B.J3p[1] = s3 * w[1];
    const double iE1 = 1.0 / B.E1, iE3 = 1.0 / B.E3;
    // Hbar_zz
    for (int r = 0; r < NZ; ++r)
      for (int q = 0; q <= r; ++q)
        B.K[B.pk(r, q)] = B.J1[r] * B.J1[q] * iE1 + B.J3z[r] * B.J3z[q] * iE3;
    for (int j = 0; j < NZ; ++j) {
      const bool is_mu = j < EN;
      const int jj = is_mu ? j : j - EN;
      const bool on = is_mu ? (jj < en) : (jj < em);
      double dg;
      if (!on) {
        dg = 1.0;  // padding
        for (int q = 0; q < NZ; ++q) {
          if (q <= j) B.K[B.pk(j, q)] = 0.0;
          else B.K[B.pk(q, j)] = 0.0;
        }
      } else if (ls) {
        dg = 1.0;
      } else {
        dg = zq[j] / (xq[j] - xlq[j]) + dw + prox[j];
      }
      B.K[B.pk(j, j)] += dg;
    }
    if (!ls) {
      for (int r = 0; r < EM; ++r)
        for (int q = 0; q <= r; ++q)
          B.K[B.pk(EN + r, EN + q)] += y1 * 2.0 * (A0[r] * A0[q] + A1[r] * A1[q]);
    }
    // constraint rows c2a, c2b
    for (int j = 0; j < EN; ++j) {
      B.K[B.pk(NZ, j)] = sa * G0[j];
      B.K[B.pk(NZ + 1, j)] = sb * G1[j];
    }
    for (int j = 0; j < EM; ++j) {
      B.K[B.pk(NZ, EN + j)] = sa * (cs * A0[j] + sn * A1[j]);
      B.K[B.pk(NZ + 1, EN + j)] = sb * (-sn * A0[j] + cs * A1[j]);
    }
    B.K[B.pk(NZ, NZ)] = -(dc + ea);
    B.K[B.pk(NZ + 1, NZ)] = 0.0;
    B.K[B.pk(NZ + 1, NZ + 1)] = -(dc + eb);
    // coupling B = [Hbar_zp; Cp]
    const double dRa = -sn * ya - cs * yb, dRb = cs * ya - sn * yb;  // dR^T/dth' y2
    for (int r = 0; r < NZ; ++r) {
      B.B[r][0] = B.J3z[r] * B.J3p[0] * iE3;
      B.B[r][1] = B.J3z[r] * B.J3p[1] * iE3;
      B.B[r][2] = 0.0;
    }
    if (!ls) {
      for (int j = 0; j < EM; ++j) {
        B.B[EN + j][0] += y3 * A0[j];
        B.B[EN + j][1] += y3 * A1[j];
        B.B[EN + j][2] += A0[j] * dRa + A1[j] * dRb;
      }
    }
    B.B[NZ][0] = 0.0;
    B.B[NZ][1] = 0.0;
    B.B[NZ][2] = sa * (-sn * w[0] + cs * w[1]);
    B.B[NZ + 1][0] = 0.0;
    B.B[NZ + 1][1] = 0.0;
    B.B[NZ + 1][2] = sb * (-cs * w[0] - sn * w[1]);
    // direct p-p terms
    B.Hpp[0] = B.J3p[0] * B.J3p[0] * iE3;
    B.Hpp[1] = B.J3p[0] * B.J3p[1] * iE3;
    B.Hpp[2] = B.J3p[1] * B.J3p[1] * iE3;
    B.Hpp[3] = 0.0;
    B.Hpp[4] = 0.0;
    B.Hpp[5] = ls ? 0.0 : -(ya * (cs * w[0] + sn * w[1]) + yb * (-sn * w[0] + cs * w[1]));
    (void)NL;
  }

  // Local block p with Bunch-Kaufman interchanges (rare): rebuild, factor,
  // solve the nrhs right-hand sides V[k*NL ...] in place.
  template <int EN, int EM>
  HTP_COLD HTP_HD void local_pivoted(int p, bool ls, double dw, double dc, double* V, int nrhs,
                                                      int* inertia) const {
    constexpr int NL = LocalBlock<EN, EM>::NL;
    constexpr int NPK = LocalBlock<EN, EM>::NPK;
    LocalBlock<EN, EM> B;
    build_local<EN, EM>(B, p, ls, dw, dc);
    int ip[NL];
#if defined(__HIPCC__)
    // Device, 4-edge blocks: dsytf2 on this lane's LDS slice instead of a runtime-indexed private
    // array (every update a scratch read-modify-write).  Free here: the slice overlaps only the
    // Riccati ring, which no local sweep uses.  Same arithmetic, bit-identical.
    if constexpr (Ctx::kMfma && HTP_PIV_LDS && NPK <= PIV_LDS_PER_LANE) {
      ld* K = c.lds + RING_OFF + c.lane * NPK;
      for (int q = 0; q < NPK; ++q) K[q] = B.K[q];
      bk_factor_packed(K, ip, NL, inertia[0], inertia[1]);
      for (int k = 0; k < nrhs; ++k) bk_solve_packed(K, ip, NL, V + k * NL);
      return;
    }
#endif
    bk_factor_packed(B.K, ip, NL, inertia[0], inertia[1]);
    for (int k = 0; k < nrhs; ++k) bk_solve_packed(B.K, ip, NL, V + k * NL);
  }

  // local_pivoted as SIMD-convergent code (bk_factor_simd / bk_solve_simd), inlined; on the device the block goes
  // to this lane's interleaved slice of the LDS ring region (element e at lds[RING_OFF + 64 e + lane]).  The NRHS
  // right-hand sides are solved one at a time: col(k, v, false) fills v with column k, col(k, v, true) consumes
  // its solution, so only one column is live in registers (all four at once pushed the kernel into spills).
  // Bit-identical to local_pivoted.  B: the block as build_local returned it (not factored).
  template <int EN, int EM, int NRHS, class Col>
  HTP_HD HTP_FI void local_pivoted_v(const LocalBlock<EN, EM>& B, Col&& col, int* inertia) const {
    constexpr int NL = LocalBlock<EN, EM>::NL;
    constexpr int NPK = LocalBlock<EN, EM>::NPK;
    int ip[NL];
#if defined(__HIPCC__) || defined(HTP_EMU_WAVE)
#if HTP_PIV_V_LDS && HTP_BK_BATCH && defined(__HIPCC__)
    if constexpr (Ctx::kMfma && HTP_PIV_LDS && NPK <= PIV_LDS_PER_LANE) {
      // pivots packed in a register, each right-hand side in this lane's slice of the stage-LDL scratch [0, 64 NL)
      // (free during the local sweeps): no private-memory arrays on the pivoted path.  Device only: the host
      // emulation keeps the register form below, the same operations on the same values (its 64 lane threads
      // writing interleaved LDS doubles would share cache lines on every step)
      static_assert(64 * NL <= 4 * NBMAX * NBMAX, "pivoted right-hand sides exceed the stage-LDL scratch");
      ld* K = c.lds + RING_OFF + c.lane;
#pragma unroll
      for (int q = 0; q < NPK; ++q) K[64 * q] = B.K[q];
      unsigned long long ipw;
      bk_factor_batch_p<NL, 64>(K, ipw, inertia[0], inertia[1]);
#if defined(HTP_LPROF) && HTP_LPROF == 2
      lp2_t = c.clock();
#endif
      ld* vl = c.lds + c.lane;
#pragma unroll
      for (int k = 0; k < NRHS; ++k) {
        double v[NL];
        col(k, v, false);
#pragma unroll
        for (int j = 0; j < NL; ++j) vl[64 * j] = v[j];
        bk_solve_batch_l<NL, 64>(K, ipw, vl);
#pragma unroll
        for (int j = 0; j < NL; ++j) v[j] = vl[64 * j];
        col(k, v, true);
      }
      (void)ip;
      return;
    }
#endif
    if constexpr (Ctx::kMfma && HTP_PIV_LDS && NPK <= PIV_LDS_PER_LANE) {
      ld* K = c.lds + RING_OFF + c.lane;
#pragma unroll
      for (int q = 0; q < NPK; ++q) K[64 * q] = B.K[q];
#if HTP_BK_BATCH
      bk_factor_batch<NL, 64>(K, ip, inertia[0], inertia[1]);
#else
      bk_factor_simd<NL, 64>(K, ip, inertia[0], inertia[1]);
#endif
#if defined(HTP_LPROF) && HTP_LPROF == 2
      lp2_t = c.clock();
#endif
#if HTP_BK_MULTI && HTP_BK_BATCH
      if constexpr (NRHS > 1) {
        double v[NRHS][NL];
#pragma unroll
        for (int k = 0; k < NRHS; ++k) col(k, v[k], false);
        bk_solve_batch_multi<NL, 64, NRHS>(K, ip, v);
#pragma unroll
        for (int k = 0; k < NRHS; ++k) col(k, v[k], true);
        return;
      }
#endif
#pragma unroll
      for (int k = 0; k < NRHS; ++k) {
        double v[NL];
        col(k, v, false);
#if HTP_BK_BATCH
        bk_solve_batch<NL, 64>(K, ip, v);
#else
        bk_solve_simd<NL, 64>(K, ip, v);
#endif
        col(k, v, true);
      }
      return;
    }
#endif
    double K[NPK];
#pragma unroll
    for (int q = 0; q < NPK; ++q) K[q] = B.K[q];
#if HTP_BK_BATCH
    bk_factor_batch<NL, 1>(K, ip, inertia[0], inertia[1]);
#else
    bk_factor_simd<NL, 1>(K, ip, inertia[0], inertia[1]);
#endif
#pragma unroll
    for (int k = 0; k < NRHS; ++k) {
      double v[NL];
      col(k, v, false);
#if HTP_BK_BATCH
      bk_solve_batch<NL, 1>(K, ip, v);
#else
      bk_solve_simd<NL, 1>(K, ip, v);
#endif
      col(k, v, true);
    }
  }

  // LocalStore record of block p (HTP_STORE_LOCAL): written by the factor sweep, read by the solve sweeps
  template <int EN, int EM>
  HTP_HD HTP_FI void store_local(const LocalBlock<EN, EM>& B, int p, bool piv) {
    using S = LocalStore<EN, EM>;
    gd* F = A(L.lfac) + p;
    const int64_t P = D.P;
    F[S::F_PIV * P] = piv ? 1.0 : 0.0;
    if (piv) return;
    for (int q = 0; q < S::NPK; ++q) F[(S::F_K + q) * P] = B.K[q];
    for (int r = 0; r < S::NL; ++r)
      for (int col = 0; col < 3; ++col) F[(S::F_B + 3 * r + col) * P] = B.B[r][col];
    for (int j = 0; j < S::NZ; ++j) {
      F[(S::F_J1 + j) * P] = B.J1[j];
      F[(S::F_J3Z + j) * P] = B.J3z[j];
    }
    F[S::F_J3P * P] = B.J3p[0];
    F[(S::F_J3P + 1) * P] = B.J3p[1];
    F[S::F_E1 * P] = B.E1;
    F[S::F_E3 * P] = B.E3;
    F[S::F_DS1 * P] = B.Ds1;
    F[S::F_DS3 * P] = B.Ds3;
  }
  // true: block p took the pivoted path (its record holds only the flag)
  template <int EN, int EM>
  HTP_HD HTP_FI bool load_local(LocalBlock<EN, EM>& B, int p) const {
    using S = LocalStore<EN, EM>;
    const gd* F = A(L.lfac) + p;
    const int64_t P = D.P;
    if (F[S::F_PIV * P] != 0.0) return true;
    for (int q = 0; q < S::NPK; ++q) B.K[q] = F[(S::F_K + q) * P];
    for (int r = 0; r < S::NL; ++r)
      for (int col = 0; col < 3; ++col) B.B[r][col] = F[(S::F_B + 3 * r + col) * P];
    for (int j = 0; j < S::NZ; ++j) {
      B.J1[j] = F[(S::F_J1 + j) * P];
      B.J3z[j] = F[(S::F_J3Z + j) * P];
    }
    B.J3p[0] = F[S::F_J3P * P];
    B.J3p[1] = F[(S::F_J3P + 1) * P];
    B.E1 = F[S::F_E1 * P];
    B.E3 = F[S::F_E3 * P];
    B.Ds1 = F[S::F_DS1 * P];
    B.Ds3 = F[S::F_DS3 * P];
    return false;
  }

  // The three local sweeps run in two passes.  Pass 1: lane-parallel over the blocks; a block whose
  // unpivoted LDL^T meets a non-positive multiplier pivot (B.piv: ~11 % of the blocks of config D)
  // is only recorded, its index compacted into L.plist (ballot rank).  Pass 2: the recorded blocks,
  // one per lane, through the Bunch-Kaufman path (local_pivoted).  Before, a 64-block trip holding
  // any pivoted block ran that path for the whole wave -- nearly every trip.  Each block's
  // arithmetic is unchanged, so the results are bit-identical.
  // block p's right-hand side v (before the solve) and the eliminated rows' q3 (local_rhs_sweep)
  template <int EN, int EM>
  HTP_HD HTP_FI void local_rhs_vec(int p, const LocalBlock<EN, EM>& B, const gd* bx, const gd* bs, const gd* bc,
                                   const gd* bd, double* v, double& q3) const {
    constexpr int NZ = LocalBlock<EN, EM>::NZ;
    int i, m, n, mu0, la0;
    pair_index(p, i, m, n, mu0, la0);
    const int em = D.eo[m], en = D.eb[n];
    const int re = D.ePair + 2 * p;
    const double bd1 = bd[2 * p], bs1 = bs[2 * p], bd3 = bd[2 * p + 1], bs3 = bs[2 * p + 1];
    const double bc0 = bc[re], bc1 = bc[re + 1];
    double bxz[NZ];
    for (int j = 0; j < EN; ++j) bxz[j] = bx[mu0 + (j < en ? j : 0)];
    for (int j = 0; j < EM; ++j) bxz[EN + j] = bx[la0 + (j < em ? j : 0)];
    const double q1 = (bd1 + bs1 / B.Ds1) / B.E1;
    q3 = (bd3 + bs3 / B.Ds3) / B.E3;
    for (int j = 0; j < EN; ++j) v[j] = (j < en ? bxz[j] : 0.0) + B.J1[j] * q1 + B.J3z[j] * q3;
    for (int j = 0; j < EM; ++j) v[EN + j] = (j < em ? bxz[EN + j] : 0.0) + B.J1[EN + j] * q1 + B.J3z[EN + j] * q3;
    v[NZ] = bc0;
    v[NZ + 1] = bc1;
  }
  // block p's stage contribution from its solved v (local_rhs_sweep)
  template <int EN, int EM>
  HTP_HD HTP_FI void local_rhs_out(int p, const LocalBlock<EN, EM>& B, const double* v, double q3, gd* PR) const {
    constexpr int NL = LocalBlock<EN, EM>::NL;
    for (int col = 0; col < 3; ++col) {
      double acc = 0.0;
      for (int r = 0; r < NL; ++r) acc += B.B[r][col] * v[r];
      PR[3 * p + col] = -acc + (col < 2 ? B.J3p[col] * q3 : 0.0);
    }
  }

  template <int EN, int EM>
  // inertia of local block p at (dw, dc), exactly as local_factor_sweep decides it (LDL^T, or Bunch-Kaufman when
  // that needs pivoting)
  HTP_HD HTP_FI void block_inertia(int p, bool ls, double dw, double dc, int& nb, int& zb) {
    LocalBlock<EN, EM> B;
    build_local<EN, EM>(B, p, ls, dw, dc);
    B.factor();
    if (!B.piv) { nb = B.neg; zb = B.zero ? 1 : 0; return; }
    int pn[2];
#if HTP_BK_SIMD
    build_local<EN, EM>(B, p, ls, dw, dc);   // B.factor() overwrote the block
    local_pivoted_v<EN, EM, 0>(B, [](int, double*, bool) {}, pn);
#else
    local_pivoted<EN, EM>(p, ls, dw, dc, nullptr, 0, pn);
#endif
    nb = pn[0];
    zb = pn[1] ? 1 : 0;
  }
  template <int EN, int EM>
  HTP_HD HTP_FI void local_factor_sweep(bool ls, double dw, double dc, int& neg, int& zero) {
    if constexpr (PT) {
      local_factor_sweep_pt(ls, dw, dc, neg, zero);
      return;
    }
    gd* PS = A(L.pairS);
    gd* PL = A(L.plist);
    constexpr int NL = LocalBlock<EN, EM>::NL;
    auto sidx = [](int row, int col) {  // (row, col) -> xx0 xy1 yy2 xt3 yt4 tt5
      return (col == 0) ? 0 : (col == 1 ? (row == 0 ? 1 : 2) : (row == 0 ? 3 : (row == 1 ? 4 : 5)));
    };
    int npiv = 0;  // wave-uniform
    // inertia scan (ic_scan): this lane's latest first-right candidate and earliest zero-pivot candidate
    int sc_pass = 0, sc_zero = 1 << 20;
    auto scan = [&](int p, int neg_b, int zero_b) {
      if (neg_b == 2 && !zero_b) return;
      if (zero_b && dc == 0.0) { sc_zero = 0; return; }   // (the trial's own dc event: no scan needed)
      double dwj = dw;
      for (int j = 1; j <= 64; ++j) {
        dwj = next_dw(dwj);
        if (!(dwj <= o.dw_max)) { sc_pass = sc_pass > j ? sc_pass : j; return; }
        int nb_, zb_;
        block_inertia<EN, EM>(p, ls, dwj, dc, nb_, zb_);
        if (zb_ && dc == 0.0) { sc_zero = sc_zero < j ? sc_zero : j; return; }
        if (nb_ == 2 && !zb_) { sc_pass = sc_pass > j ? sc_pass : j; return; }
      }
      sc_pass = 64;
    };
#ifdef HTP_LPROF
    long long lt0 = c.clock(), lscan = 0;
#endif
#if HTP_HOIST_TRIP
    const int nblk_ = c.uniform_i(D.P), lane_ = c.lane;   // loop bound and lane read once, not behind every trip's stores
#else
    const int nblk_ = D.P, lane_ = 0;
#endif
    for (int b0 = 0; b0 < (HTP_HOIST_TRIP ? nblk_ : D.P); b0 += c.width) {
      const int p = b0 + (HTP_HOIST_TRIP ? lane_ : (int)c.lane);
      bool piv = false;
      HTP_LP1(2, 1);
      if (p < D.P) {
        LocalBlock<EN, EM> B;
        build_local<EN, EM>(B, p, ls, dw, dc);
        B.factor();
        piv = B.piv;
#if HTP_STORE_LOCAL
        store_local<EN, EM>(B, p, piv);
#endif
        if (!piv) {
          neg += B.neg;
          zero |= B.zero;
          const int nb0 = B.neg, zb0 = B.zero ? 1 : 0;
          // B' K^-1 B = W' D^-1 W with W = L^-1 B: forward substitutions only
          double W[3][NL];
          for (int col = 0; col < 3; ++col) {
            for (int r = 0; r < NL; ++r) W[col][r] = B.B[r][col];
            B.forward(W[col]);
          }
          double id[NL];
          for (int r = 0; r < NL; ++r) id[r] = 1.0 / B.K[B.pk(r, r)];
          double S[6];
          for (int col = 0; col < 3; ++col)
            for (int row = 0; row <= col; ++row) {
              double acc = 0.0;
              for (int r = 0; r < NL; ++r) acc += W[row][r] * (W[col][r] * id[r]);
              S[sidx(row, col)] = acc;
            }
#if HTP_HOIST
          // the fused right-hand side's loads before the block's first store (a load waits for earlier stores)
          if (fuse_rhs) {   // the Newton step's right-hand side (kkt_solve's local_rhs_sweep, fused)
            double v[NL], q3;
            local_rhs_vec<EN, EM>(p, B, A(L.xt), A(L.rs), A(L.rc), A(L.rd), v, q3);
            B.solve(v);
            for (int k = 0; k < 6; ++k) PS[6 * p + k] = B.Hpp[k] - S[k];
            local_rhs_out<EN, EM>(p, B, v, q3, A(L.pairR));
          } else {
            for (int k = 0; k < 6; ++k) PS[6 * p + k] = B.Hpp[k] - S[k];
          }
#else
          for (int k = 0; k < 6; ++k) PS[6 * p + k] = B.Hpp[k] - S[k];
          if (fuse_rhs) {   // the Newton step's right-hand side (kkt_solve's local_rhs_sweep, fused)
            double v[NL], q3;
            local_rhs_vec<EN, EM>(p, B, A(L.xt), A(L.rs), A(L.rc), A(L.rd), v, q3);
            B.solve(v);
            local_rhs_out<EN, EM>(p, B, v, q3, A(L.pairR));
          }
#endif
#ifdef HTP_LPROF
          const long long ls0 = c.clock();
#endif
          if (ic_scan) scan(p, nb0, zb0);   // after the block is dead (registers)
#ifdef HTP_LPROF
          lscan += c.clock() - ls0;
#endif
        }
      }
      int cnt;
      const int r = c.rank(piv, cnt);
      if (piv) PL[npiv + r] = (double)p;
      npiv += cnt;
    }
    c.sync();
#ifdef HTP_LPROF
    const long long lt1 = c.clock();
    HTP_LP1(0, lt1 - lt0);
    HTP_LP(4, (long long)c.maxv((double)lscan));
    HTP_LP(5, npiv);
    HTP_LP(6, 1);
#endif
    for (int b0 = 0; b0 < npiv; b0 += c.width) {
      const int q = b0 + (HTP_HOIST_TRIP ? lane_ : (int)c.lane);
      HTP_LP1(3, 1);
      if (q < npiv) {
        const int p = (int)PL[q];
        LocalBlock<EN, EM> B;
#if defined(HTP_LPROF) && HTP_LPROF == 2
        const long long q0 = c.clock();
#endif
        build_local<EN, EM>(B, p, ls, dw, dc);
#if defined(HTP_LPROF) && HTP_LPROF == 2
        const long long q1 = c.clock();
        HTP_LP2(0, q1 - q0);
#endif
        int pn[2];
        double S[6];
#if HTP_BK_SIMD
        double q3 = 0.0;
        auto colf = [&](int col, double* v, bool done) {
          if (col < 3) {
            if (!done) {
              for (int r = 0; r < NL; ++r) v[r] = B.B[r][col];
            } else {
              for (int row = 0; row <= col; ++row) {  // S(:,col) = B' K^-1 B(:,col)
                double acc = 0.0;
                for (int r = 0; r < NL; ++r) acc += B.B[r][row] * v[r];
                S[sidx(row, col)] = acc;
              }
            }
          } else if (!done) {
            local_rhs_vec<EN, EM>(p, B, A(L.xt), A(L.rs), A(L.rc), A(L.rd), v, q3);
          } else {
            local_rhs_out<EN, EM>(p, B, v, q3, A(L.pairR));
          }
        };
        if (fuse_rhs) local_pivoted_v<EN, EM, 4>(B, colf, pn);
        else local_pivoted_v<EN, EM, 3>(B, colf, pn);
#if defined(HTP_LPROF) && HTP_LPROF == 2
        const long long q2 = c.clock();
        HTP_LP2(2, lp2_t - q1);
        HTP_LP2(3, q2 - lp2_t);
#endif
#else
        double Vp[4 * NL], q3 = 0.0;
        for (int col = 0; col < 3; ++col)
          for (int r = 0; r < NL; ++r) Vp[col * NL + r] = B.B[r][col];
        if (fuse_rhs) local_rhs_vec<EN, EM>(p, B, A(L.xt), A(L.rs), A(L.rc), A(L.rd), Vp + 3 * NL, q3);
        local_pivoted<EN, EM>(p, ls, dw, dc, Vp, fuse_rhs ? 4 : 3, pn);
        if (fuse_rhs) local_rhs_out<EN, EM>(p, B, Vp + 3 * NL, q3, A(L.pairR));
        for (int col = 0; col < 3; ++col)
          for (int row = 0; row <= col; ++row) {  // S(:,col) = B' K^-1 B(:,col)
            double acc = 0.0;
            for (int r = 0; r < NL; ++r) acc += B.B[r][row] * Vp[col * NL + r];
            S[sidx(row, col)] = acc;
          }
#endif
        neg += pn[0];
        zero |= pn[1];
        for (int k = 0; k < 6; ++k) PS[6 * p + k] = B.Hpp[k] - S[k];
        if (ic_scan) scan(p, pn[0], pn[1]);
      }
    }
#ifdef HTP_LPROF
    HTP_LP(1, c.clock() - lt1);
#endif
    if (ic_scan) {   // every trial before min(latest first-right, earliest zero) fails without a zero pivot
      const int pass = (int)c.maxv((double)sc_pass), zr = (int)c.minv((double)sc_zero);
      const int first = pass < zr ? pass : zr;
      ic_skip = first > 1 ? first - 1 : 0;
    }
  }

  // rhs sweep: bx (x part), bs, bc, bd -> pairR (stage contributions)
  template <int EN, int EM>
  HTP_HD HTP_FI void local_rhs_sweep(bool ls, double dw, double dc, const gd* bx, const gd* bs,
                              const gd* bc, const gd* bd) {
    if constexpr (PT) {
      local_rhs_sweep_pt(ls, dw, dc, bx, bs, bd);
      return;
    }
    gd* PR = A(L.pairR);
    gd* PL = A(L.plist);
    constexpr int NL = LocalBlock<EN, EM>::NL;
    auto rhs = [&](int p, const LocalBlock<EN, EM>& B, double* v, double& q3) {
      local_rhs_vec<EN, EM>(p, B, bx, bs, bc, bd, v, q3);
    };
    auto out = [&](int p, const LocalBlock<EN, EM>& B, const double* v, double q3) {
      local_rhs_out<EN, EM>(p, B, v, q3, PR);
    };
    int npiv = 0;
#if HTP_HOIST_TRIP
    const int nblk_ = c.uniform_i(D.P), lane_ = c.lane;   // loop bound and lane read once, not behind every trip's stores
#else
    const int nblk_ = D.P, lane_ = 0;
#endif
    for (int b0 = 0; b0 < (HTP_HOIST_TRIP ? nblk_ : D.P); b0 += c.width) {
      const int p = b0 + (HTP_HOIST_TRIP ? lane_ : (int)c.lane);
      bool piv = false;
      if (p < D.P) {
        LocalBlock<EN, EM> B;
#if HTP_STORE_LOCAL
        piv = load_local<EN, EM>(B, p);
#else
        build_local<EN, EM>(B, p, ls, dw, dc);
        B.factor();
        piv = B.piv;
#endif
        if (!piv) {
          double v[NL], q3;
          rhs(p, B, v, q3);
          B.solve(v);
          out(p, B, v, q3);
        }
      }
      int cnt;
      const int r = c.rank(piv, cnt);
      if (piv) PL[npiv + r] = (double)p;
      npiv += cnt;
    }
    c.sync();
    for (int b0 = 0; b0 < npiv; b0 += c.width) {
      const int q = b0 + (HTP_HOIST_TRIP ? lane_ : (int)c.lane);
      if (q < npiv) {
        const int p = (int)PL[q];
        LocalBlock<EN, EM> B;
        build_local<EN, EM>(B, p, ls, dw, dc);
        int pn[2];
#if HTP_BK_SIMD
        double q3;
        local_pivoted_v<EN, EM, 1>(B, [&](int, double* v, bool done) {
          if (!done) rhs(p, B, v, q3);
          else out(p, B, v, q3);
        }, pn);
#else
        double v[NL], q3;
        rhs(p, B, v, q3);
        local_pivoted<EN, EM>(p, ls, dw, dc, v, 1, pn);
        out(p, B, v, q3);
#endif
      }
    }
  }

  template <int EN, int EM>
  HTP_HD HTP_FI void local_back_sweep(bool ls, double dw, double dc, const gd* bx, const gd* bs,
                               const gd* bc, const gd* bd, gd* ox, gd* os, gd* oc,
                               gd* od) {
    if constexpr (PT) {
      local_back_sweep_pt(ls, dw, dc, bx, bs, bd, ox, os, od);
      return;
    }
    gd* PL = A(L.plist);
    constexpr int NZ = LocalBlock<EN, EM>::NZ;
    constexpr int NL = LocalBlock<EN, EM>::NL;
    // block p's right-hand side minus its coupling to the stage step dp = (dx, dy, dtheta), before the solve
    auto rhs = [&](int p, const LocalBlock<EN, EM>& B, double* v, double& dpx, double& dpy) {
      int i, m, n, mu0, la0;
      pair_index(p, i, m, n, mu0, la0);
      const int em = D.eo[m], en = D.eb[n];
      const int re = D.ePair + 2 * p;
      const double bd1 = bd[2 * p], bs1 = bs[2 * p], bd3 = bd[2 * p + 1], bs3 = bs[2 * p + 1];
      const double bc0 = bc[re], bc1 = bc[re + 1];
      dpx = ox[NS * i];
      dpy = ox[NS * i + 1];
      const double dth = ox[NS * i + 3];
      double bxz[NZ];
      for (int j = 0; j < EN; ++j) bxz[j] = bx[mu0 + (j < en ? j : 0)];
      for (int j = 0; j < EM; ++j) bxz[EN + j] = bx[la0 + (j < em ? j : 0)];
      const double q1 = (bd1 + bs1 / B.Ds1) / B.E1;
      const double q3 = (bd3 + bs3 / B.Ds3) / B.E3;
      for (int j = 0; j < EN; ++j) v[j] = (j < en ? bxz[j] : 0.0) + B.J1[j] * q1 + B.J3z[j] * q3;
      for (int j = 0; j < EM; ++j) v[EN + j] = (j < em ? bxz[EN + j] : 0.0) + B.J1[EN + j] * q1 + B.J3z[EN + j] * q3;
      v[NZ] = bc0;
      v[NZ + 1] = bc1;
      for (int r = 0; r < NL; ++r) v[r] -= B.B[r][0] * dpx + B.B[r][1] * dpy + B.B[r][2] * dth;
    };
    auto out = [&](int p, const LocalBlock<EN, EM>& B, const double* v, double dpx, double dpy) {
      int i, m, n, mu0, la0;
      pair_index(p, i, m, n, mu0, la0);
      const int em = D.eo[m], en = D.eb[n];
      const int re = D.ePair + 2 * p;
      const double bd1 = bd[2 * p], bs1 = bs[2 * p], bd3 = bd[2 * p + 1], bs3 = bs[2 * p + 1];
      for (int j = 0; j < en; ++j) ox[mu0 + j] = v[j];
      for (int j = 0; j < em; ++j) ox[la0 + j] = v[EN + j];
      oc[re] = v[NZ];
      oc[re + 1] = v[NZ + 1];
      double j1 = 0.0, j3 = B.J3p[0] * dpx + B.J3p[1] * dpy;
      for (int r = 0; r < NZ; ++r) {
        j1 += B.J1[r] * v[r];
        j3 += B.J3z[r] * v[r];
      }
      const double y1 = (j1 - bd1 - bs1 / B.Ds1) / B.E1;
      const double y3 = (j3 - bd3 - bs3 / B.Ds3) / B.E3;
      od[2 * p] = y1;
      od[2 * p + 1] = y3;
      os[2 * p] = (bs1 + y1) / B.Ds1;
      os[2 * p + 1] = (bs3 + y3) / B.Ds3;
    };
    int npiv = 0;
#if HTP_HOIST_TRIP
    const int nblk_ = c.uniform_i(D.P), lane_ = c.lane;   // loop bound and lane read once, not behind every trip's stores
#else
    const int nblk_ = D.P, lane_ = 0;
#endif
    for (int b0 = 0; b0 < (HTP_HOIST_TRIP ? nblk_ : D.P); b0 += c.width) {
      const int p = b0 + (HTP_HOIST_TRIP ? lane_ : (int)c.lane);
      bool piv = false;
      if (p < D.P) {
        LocalBlock<EN, EM> B;
#if HTP_STORE_LOCAL
        piv = load_local<EN, EM>(B, p);
#else
        build_local<EN, EM>(B, p, ls, dw, dc);
        B.factor();
        piv = B.piv;
#endif
        if (!piv) {
          double v[NL], dpx, dpy;
          rhs(p, B, v, dpx, dpy);
          B.solve(v);
          out(p, B, v, dpx, dpy);
        }
      }
      int cnt;
      const int r = c.rank(piv, cnt);
      if (piv) PL[npiv + r] = (double)p;
      npiv += cnt;
    }
    c.sync();
    for (int b0 = 0; b0 < npiv; b0 += c.width) {
      const int q = b0 + (HTP_HOIST_TRIP ? lane_ : (int)c.lane);
      if (q < npiv) {
        const int p = (int)PL[q];
        LocalBlock<EN, EM> B;
        build_local<EN, EM>(B, p, ls, dw, dc);
        int pn[2];
#if HTP_BK_SIMD
        double dpx, dpy;
        local_pivoted_v<EN, EM, 1>(B, [&](int, double* v, bool done) {
          if (!done) rhs(p, B, v, dpx, dpy);
          else out(p, B, v, dpx, dpy);
        }, pn);
#else
        double v[NL], dpx, dpy;
        rhs(p, B, v, dpx, dpy);
        local_pivoted<EN, EM>(p, ls, dw, dc, v, 1, pn);
        out(p, B, v, dpx, dpy);
#endif
      }
    }
  }

  // ---------------------------------------------------- point-formulation blocks
  // eliminated inequality rows of block p, vertex k: diagonal Ds and E = 1/Ds + dc
  HTP_HD HTP_FI void pt_row_e(int p, int k, bool ls, double dw, double dc, double& Ds1, double& E1, double& Ds3,
                              double& E3) const {
    const int r1 = 2 * (D.KV * p + k), r3 = r1 + 1;
    if (ls) {
      Ds1 = 1.0;
      Ds3 = 1.0;
    } else {
      const gd* s = A(L.s); const gd* dL = A(L.dL); const gd* dU = A(L.dU);
      const gd* vL = A(L.vL); const gd* vU = A(L.vU);
      Ds1 = vL[r1] / (s[r1] - dL[r1]) + vU[r1] / (dU[r1] - s[r1]) + dw;
      Ds3 = vL[r3] / (s[r3] - dL[r3]) + vU[r3] / (dU[r3] - s[r3]) + dw;
    }
    E1 = 1.0 / Ds1 + dc;
    E3 = 1.0 / Ds3 + dc;
    if (rs) {
      const gd* eR = A(L.eR);
      E1 += eR[D.mc + r1];
      E3 += eR[D.mc + r3];
    }
  }
  // scaled Jacobian rows of block p, vertex k: J1 = s1 2 A w (z only), J3 = [J3z | J3p]
  HTP_HD HTP_FI void pt_row_jac(const PtGeom& G, int p, int k, double& s1, double* J3z, double* J3p, double* dv,
                                double* rv) const {
    const gd* scI = A(L.scI);
    const int r1 = 2 * (D.KV * p + k);
    s1 = scI[r1];
    const double s3 = scI[r1 + 1];
    double vt[2];
    pt_vertex(G, k, vt, dv, rv);
    for (int j = 0; j < EM_; ++j) J3z[j] = s3 * (G.A0[j] * vt[0] + G.A1[j] * vt[1] - G.bb[j]);
    J3p[0] = s3 * G.w0;
    J3p[1] = s3 * G.w1;
    J3p[2] = s3 * (G.w0 * dv[0] + G.w1 * dv[1]);
  }

  HTP_HD HTP_FI void build_local_pt(PtBlock<EM_>& B, const PtGeom& G, int p, bool ls, double dw, double dc) const {
    const gd* x = A(L.x); const gd* xL = A(L.xL); const gd* xU = A(L.xU);
    const gd* zL = A(L.zL); const gd* zU = A(L.zU);
    const gd* scI = A(L.scI); const gd* yd = A(L.yd);
    constexpr int NZ = EM_;
    for (int q = 0; q < PtBlock<EM_>::NPK; ++q) B.K[q] = 0.0;
    for (int r = 0; r < NZ; ++r) B.B[r][0] = B.B[r][1] = B.B[r][2] = 0.0;
    for (int q = 0; q < 6; ++q) B.Hpp[q] = 0.0;
    double Aw2[EM_];
    for (int j = 0; j < EM_; ++j) Aw2[j] = 2.0 * (G.A0[j] * G.w0 + G.A1[j] * G.w1);
    double y1sum = 0.0;
    for (int k = 0; k < D.KV; ++k) {
      double Ds1, E1, Ds3, E3, s1, J3z[EM_], J3p[3], dv[2], rv[2];
      pt_row_e(p, k, ls, dw, dc, Ds1, E1, Ds3, E3);
      pt_row_jac(G, p, k, s1, J3z, J3p, dv, rv);
      const double iE3 = 1.0 / E3, c1 = s1 * s1 / E1;
      for (int r = 0; r < NZ; ++r)
        for (int q = 0; q <= r; ++q) B.K[B.pk(r, q)] += c1 * Aw2[r] * Aw2[q] + J3z[r] * J3z[q] * iE3;
      for (int r = 0; r < NZ; ++r)
        for (int col = 0; col < 3; ++col) B.B[r][col] += J3z[r] * J3p[col] * iE3;
      B.Hpp[0] += J3p[0] * J3p[0] * iE3;
      B.Hpp[1] += J3p[0] * J3p[1] * iE3;
      B.Hpp[2] += J3p[1] * J3p[1] * iE3;
      B.Hpp[3] += J3p[0] * J3p[2] * iE3;
      B.Hpp[4] += J3p[1] * J3p[2] * iE3;
      B.Hpp[5] += J3p[2] * J3p[2] * iE3;
      if (!ls) {  // multiplier-weighted constraint Hessians
        const int r1 = 2 * (D.KV * p + k);
        const double y1 = s1 * yd[r1], y3 = scI[r1 + 1] * yd[r1 + 1];
        y1sum += y1;
        for (int j = 0; j < NZ; ++j) {
          B.B[j][0] += y3 * G.A0[j];
          B.B[j][1] += y3 * G.A1[j];
          B.B[j][2] += y3 * (G.A0[j] * dv[0] + G.A1[j] * dv[1]);
        }
        B.Hpp[5] -= y3 * (G.w0 * rv[0] + G.w1 * rv[1]);
      }
    }
    if (!ls)
      for (int r = 0; r < NZ; ++r)
        for (int q = 0; q <= r; ++q) B.K[B.pk(r, q)] += y1sum * 2.0 * (G.A0[r] * G.A0[q] + G.A1[r] * G.A1[q]);
    for (int j = 0; j < NZ; ++j) {
      double dg;
      if (j >= G.em || ls) {
        dg = 1.0;  // padding / least-squares identity
      } else {
        const int vi = G.la0 + j;
        dg = zL[vi] / (x[vi] - xL[vi]) + zU[vi] / (xU[vi] - x[vi]) + dw;
        if (rs) dg += eta * A(L.dr)[vi] * A(L.dr)[vi];
      }
      B.K[B.pk(j, j)] += dg;
    }
  }

  HTP_COLD HTP_HD void local_pivoted_pt(int p, bool ls, double dw, double dc, double* V, int nrhs,
                                                         int* inertia) const {
    PtGeom G;
    pt_geom(A(L.x), p, G);
    PtBlock<EM_> B;
    build_local_pt(B, G, p, ls, dw, dc);
    int ip[EM_];
    bk_factor_packed(B.K, ip, EM_, inertia[0], inertia[1]);
    for (int k = 0; k < nrhs; ++k) bk_solve_packed(B.K, ip, EM_, V + k * EM_);
  }

  HTP_HD HTP_FI void local_factor_sweep_pt(bool ls, double dw, double dc, int& neg, int& zero) {
    gd* PS = A(L.pairS);
    const gd* x = A(L.x);
    constexpr int NZ = EM_;
    for (int p = c.lane; p < D.P; p += c.width) {
      PtGeom G;
      pt_geom(x, p, G);
      PtBlock<EM_> B;
      build_local_pt(B, G, p, ls, dw, dc);
      B.factor();
      double Vp[3 * NZ];
      int bneg = B.neg, bzero = B.zero;
      if (B.piv) {
        for (int col = 0; col < 3; ++col)
          for (int r = 0; r < NZ; ++r) Vp[col * NZ + r] = B.B[r][col];
        int pn[2];
        local_pivoted_pt(p, ls, dw, dc, Vp, 3, pn);
        bneg = pn[0];
        bzero = pn[1];
      }
      neg += bneg;
      zero |= bzero;
      double S[6] = {0, 0, 0, 0, 0, 0};
      for (int col = 0; col < 3; ++col) {
        double v[NZ];
        for (int r = 0; r < NZ; ++r) v[r] = B.piv ? Vp[col * NZ + r] : B.B[r][col];
        if (!B.piv) B.solve(v);
        for (int row = 0; row <= col; ++row) {
          double acc = 0.0;
          for (int r = 0; r < NZ; ++r) acc += B.B[r][row] * v[r];
          const int idx = (col == 0) ? 0 : (col == 1 ? (row == 0 ? 1 : 2) : (row == 0 ? 3 : (row == 1 ? 4 : 5)));
          S[idx] = acc;
        }
      }
      for (int k = 0; k < 6; ++k) PS[6 * p + k] = B.Hpp[k] - S[k];
    }
  }

  // z-part rhs of block p: bx + sum_rows J_z q_r (q_r = (bd + bs/Ds)/E); J3p q3 summed into pp
  HTP_HD HTP_FI void pt_rhs(const PtGeom& G, int p, bool ls, double dw, double dc, const gd* bx, const gd* bs,
                            const gd* bd, double* v, double* pp) const {
    for (int j = 0; j < EM_; ++j) v[j] = (j < G.em) ? bx[G.la0 + j] : 0.0;
    pp[0] = pp[1] = pp[2] = 0.0;
    double Aw2[EM_];
    for (int j = 0; j < EM_; ++j) Aw2[j] = 2.0 * (G.A0[j] * G.w0 + G.A1[j] * G.w1);
    for (int k = 0; k < D.KV; ++k) {
      double Ds1, E1, Ds3, E3, s1, J3z[EM_], J3p[3], dv[2], rv[2];
      pt_row_e(p, k, ls, dw, dc, Ds1, E1, Ds3, E3);
      pt_row_jac(G, p, k, s1, J3z, J3p, dv, rv);
      const int r1 = 2 * (D.KV * p + k), r3 = r1 + 1;
      const double q1 = (bd[r1] + bs[r1] / Ds1) / E1;
      const double q3 = (bd[r3] + bs[r3] / Ds3) / E3;
      for (int j = 0; j < EM_; ++j) v[j] += s1 * Aw2[j] * q1 + J3z[j] * q3;
      for (int col = 0; col < 3; ++col) pp[col] += J3p[col] * q3;
    }
  }

  HTP_HD HTP_FI void local_rhs_sweep_pt(bool ls, double dw, double dc, const gd* bx, const gd* bs, const gd* bd) {
    gd* PR = A(L.pairR);
    const gd* x = A(L.x);
    constexpr int NZ = EM_;
    for (int p = c.lane; p < D.P; p += c.width) {
      PtGeom G;
      pt_geom(x, p, G);
      PtBlock<EM_> B;
      build_local_pt(B, G, p, ls, dw, dc);
      B.factor();
      double v[NZ], pp[3];
      pt_rhs(G, p, ls, dw, dc, bx, bs, bd, v, pp);
      if (B.piv) {
        int pn[2];
        local_pivoted_pt(p, ls, dw, dc, v, 1, pn);
      } else {
        B.solve(v);
      }
      for (int col = 0; col < 3; ++col) {
        double acc = 0.0;
        for (int r = 0; r < NZ; ++r) acc += B.B[r][col] * v[r];
        PR[3 * p + col] = -acc + pp[col];
      }
    }
  }

  HTP_HD HTP_FI void local_back_sweep_pt(bool ls, double dw, double dc, const gd* bx, const gd* bs, const gd* bd,
                                         gd* ox, gd* os, gd* od) {
    const gd* x = A(L.x);
    constexpr int NZ = EM_;
    for (int p = c.lane; p < D.P; p += c.width) {
      PtGeom G;
      pt_geom(x, p, G);
      PtBlock<EM_> B;
      build_local_pt(B, G, p, ls, dw, dc);
      B.factor();
      double v[NZ], pp[3];
      pt_rhs(G, p, ls, dw, dc, bx, bs, bd, v, pp);
      const double dp[3] = {ox[NS * G.i], ox[NS * G.i + 1], ox[NS * G.i + 3]};
      for (int r = 0; r < NZ; ++r) v[r] -= B.B[r][0] * dp[0] + B.B[r][1] * dp[1] + B.B[r][2] * dp[2];
      if (B.piv) {
        int pn[2];
        local_pivoted_pt(p, ls, dw, dc, v, 1, pn);
      } else {
        B.solve(v);
      }
      for (int j = 0; j < EM_; ++j)
        if (j < G.em) ox[G.la0 + j] = v[j];
      double Aw2[EM_];
      for (int j = 0; j < EM_; ++j) Aw2[j] = 2.0 * (G.A0[j] * G.w0 + G.A1[j] * G.w1);
      for (int k = 0; k < D.KV; ++k) {
        double Ds1, E1, Ds3, E3, s1, J3z[EM_], J3p[3], dv[2], rv[2];
        pt_row_e(p, k, ls, dw, dc, Ds1, E1, Ds3, E3);
        pt_row_jac(G, p, k, s1, J3z, J3p, dv, rv);
        const int r1 = 2 * (D.KV * p + k), r3 = r1 + 1;
        double j1 = 0.0, j3 = J3p[0] * dp[0] + J3p[1] * dp[1] + J3p[2] * dp[2];
        for (int j = 0; j < EM_; ++j) {
          j1 += s1 * Aw2[j] * v[j];
          j3 += J3z[j] * v[j];
        }
        const double y1 = (j1 - bd[r1] - bs[r1] / Ds1) / E1;
        const double y3 = (j3 - bd[r3] - bs[r3] / Ds3) / E3;
        od[r1] = y1;
        od[r3] = y3;
        os[r1] = (bs[r1] + y1) / Ds1;
        os[r3] = (bs[r3] + y3) / Ds3;
      }
    }
  }

  // terminal block of the point formulation (stage-chain block N): rows
  // X_{N-1} - end = 0 (optimizer_points.py:273-278), coupled to x_{N-1}
  HTP_HD HTP_FI void assemble_term_pt(double dc) {
    const int N = D.N, nb = D.nb;
    const gd* scE = A(L.scE);
    gd* K = A(L.Kst) + (int64_t)N * nb * nb;
    gd* O = A(L.Off) + (int64_t)N * nb * nb;
    const gd* eR = A(L.eR);
    for (int q = c.lane; q < nb * nb; q += c.width) {
      const int r = q / nb, cc = q % nb;
      K[q] = (r == cc) ? (r < NS ? -(dc + (rs ? eR[D.eTerm + r] : 0.0)) : 1.0) : 0.0;
      O[q] = (r < NS && cc == NS + r) ? scE[D.eTerm + r] : 0.0;
    }
  }

  // terminal slack s_k (free, objective 5000 s_k^2): Hs = 10000 sf + dw (+ eta D_R^2 in the restoration phase),
  // and the eliminated terminal row's Et = dc (+ eR) + st^2 / Hs
  HTP_HD HTP_FI double term_H(int k, bool ls, double dw) const {
    if (ls) return 1.0;
    double h = 10000.0 * hsf() + dw;
    if (rs) h += eta * A(L.dr)[D.oS + k] * A(L.dr)[D.oS + k];
    return h;
  }
  HTP_HD HTP_FI double term_E(int k, bool ls, double dw, double dc) const {
    const double st = A(L.scE)[D.eTerm + k];
    double e = dc + st * st / term_H(k, ls, dw);
    if (rs) e += A(L.eR)[D.eTerm + k];
    return e;
  }

  HTP_HD HTP_FI bool uniform44() const {
    for (int m = 0; m < D.M; ++m)
      if (D.eo[m] != 4) return false;
    for (int k = 0; k < D.K; ++k)
      if (D.eb[k] != 4) return false;
    return true;
  }

  // ---------------------------------------------------------- stage blocks
  // block layout: [y 0..4 | x 5..9 | u 10,11 | tau 12]
  HTP_HD HTP_FI void assemble_stage(int i, bool ls, double dw, double dc) {
    const int N = D.N, nb = D.nb;
    const gd* x = A(L.x);
    const gd* xL = A(L.xL);
    const gd* xU = A(L.xU);
    const gd* zL = A(L.zL);
    const gd* zU = A(L.zU);
    const gd* scE = A(L.scE);
    const gd* yc = A(L.yc);
    const gd* PS = A(L.pairS);
    gd* K = A(L.Kst) + (int64_t)i * nb * nb;
    const double dT = par(P_DT);
    // The block is accumulated in registers (lower triangle, compile-time indices: every
    // add() site is unrolled) and stored once at the end: a read-modify-write of K in HBM
    // per contribution cost one memory round trip each.  (r, q) and (q, r) receive the
    // same adds in the same order, so the mirrored store is the plain accumulation.
    constexpr int NT = NBMAX * (NBMAX + 1) / 2;
    double Kl[NT];
    for (int e = 0; e < NT; ++e) Kl[e] = 0.0;
    auto add = [&](int r, int q, double v) {
      const int hi = r >= q ? r : q, lo = r >= q ? q : r;
      Kl[hi * (hi + 1) / 2 + lo] += v;
    };
    const int rowbase = (i == 0) ? 0 : D.eDyn + NS * (i - 1);
    // variables of this block; their bound data load up front (indices clamped)
    int vidx[8];
    int nv = (i < N - 1) ? D.nw : NS;
    for (int k = 0; k < NS; ++k) vidx[k] = NS * i + k;
    vidx[5] = vidx[6] = vidx[7] = NS * i;
    if (i < N - 1) {
      vidx[5] = D.oU + NC * i;
      vidx[6] = D.oU + NC * i + 1;
      if (D.topt) vidx[7] = D.oTAU + i;
    }
    double xq[8], xlq[8], xuq[8], zlq[8], zuq[8], sce[NS];
    for (int a = 0; a < 8; ++a) {
      const int q = vidx[a];
      xq[a] = x[q]; xlq[a] = xL[q]; xuq[a] = xU[q]; zlq[a] = zL[q]; zuq[a] = zU[q];
    }
    for (int k = 0; k < NS; ++k) sce[k] = scE[rowbase + k];
    double er[NS] = {0.0, 0.0, 0.0, 0.0, 0.0}, pr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rs) {
      const gd* eR = A(L.eR);
      const gd* dr = A(L.dr);
      for (int k = 0; k < NS; ++k) er[k] = eR[rowbase + k];
      if (!ls)
        for (int a = 0; a < 8; ++a) pr[a] = eta * dr[vidx[a]] * dr[vidx[a]];
    }
    const double hs = hsf();
    for (int k = 0; k < NS; ++k) add(k, k, -(dc + er[k]));
    for (int k = 0; k < NS; ++k) add(k, NS + k, sce[k]);
    for (int a = 0; a < 8; ++a) {
      if (a < nv) {
        double dg;
        if (ls) dg = 1.0;
        else {
          dg = dw + pr[a];
          if (finite_(xlq[a])) dg += zlq[a] / (xq[a] - xlq[a]);
          if (finite_(xuq[a])) dg += zuq[a] / (xuq[a] - xq[a]);
        }
        add(NS + a, NS + a, dg);
      }
    }
    for (int a = 0; a < 8; ++a)
      if (a >= nv && a < D.nw) add(NS + a, NS + a, 1.0);  // padding (last stage)
    if (PT && !ls && i < N - 1) {  // optimizer_points.py objective: 20 (v dT)^2, (u_{i+1} - u_i)^2
      const int U0 = NS + 5, V0 = NS + 2;
      add(V0, V0, hs * 40.0 * dT * dT);
      if (i < N - 2) {
        add(U0, U0, hs * 2.0);
        add(U0 + 1, U0 + 1, hs * 2.0);
      }
      if (i >= 1) {
        add(U0, U0, hs * 2.0);
        add(U0 + 1, U0 + 1, hs * 2.0);
      }
    }
    if (!ls && i < N - 1) {
      if constexpr (!PT) {
      const double tau = tauv(x, i), h = dT * tau;
      const double Qs00 = 2 * par(P_Q00), Qs01 = par(P_Q01) + par(P_Q10), Qs11 = 2 * par(P_Q11);
      const double Rs00 = 2 * par(P_R00), Rs01 = par(P_R01) + par(P_R10), Rs11 = 2 * par(P_R11);
      const int U0 = NS + 5, T0 = NS + 7, V0 = NS + 2;
      add(U0, U0, hs * Qs00);
      add(U0 + 1, U0, hs * Qs01);
      add(U0 + 1, U0 + 1, hs * Qs11);
      const double v = x[NS * i + 2];
      add(V0, V0, hs * 2.0 * par(P_W00) * h * h);
      if (D.topt) {
        add(T0, T0, hs * 2.0 * par(P_W00) * v * v * dT * dT);
        add(V0, T0, hs * 4.0 * par(P_W00) * v * dT * dT * tau);
      }
      if (i < N - 2) {
        const double ih2 = 1.0 / (h * h);
        add(U0, U0, hs * Rs00 * ih2);
        add(U0 + 1, U0, hs * Rs01 * ih2);
        add(U0 + 1, U0 + 1, hs * Rs11 * ih2);
        if (D.topt) {
          const double da = x[D.oU + NC * (i + 1)] - x[D.oU + NC * i];
          const double dw_ = x[D.oU + NC * (i + 1) + 1] - x[D.oU + NC * i + 1];
          const double Jv = (da * (par(P_R00) * da + par(P_R01) * dw_) + dw_ * (par(P_R10) * da + par(P_R11) * dw_)) * ih2;
          add(T0, T0, hs * 6.0 * Jv / (tau * tau));
          const double k2 = 2.0 * ih2 / tau;
          add(U0, T0, hs * k2 * (Rs00 * da + Rs01 * dw_));
          add(U0 + 1, T0, hs * k2 * (Rs01 * da + Rs11 * dw_));
        }
      }
      if (i >= 1 && i - 1 < N - 2) {  // jerk_{i-1} on (u_i,u_i)
        const double hp = dT * tauv(x, i - 1), ih2 = 1.0 / (hp * hp);
        add(U0, U0, hs * Rs00 * ih2);
        add(U0 + 1, U0, hs * Rs01 * ih2);
        add(U0 + 1, U0 + 1, hs * Rs11 * ih2);
      }
      }
      // dynamics Hessian of interval i:  sum_k (-yhat_k) d2F_k
      double w[8], H[36], yy[5];
      stage_w(x, i, w);
      for (int k = 0; k < NS; ++k) yy[k] = -scE[D.eDyn + NS * i + k] * yc[D.eDyn + NS * i + k];
      dynH(w, yy, H);
      for (int r = 0; r < 8; ++r)
        if (r < D.nw)
          for (int q = 0; q <= r; ++q) add(NS + r, NS + q, H[r * (r + 1) / 2 + q]);
    } else if (!ls && i >= 1 && i - 1 < N - 2) {
      // last stage has no u; nothing else
    }
    // local-block Schur complements on (x, y, theta)
    const int MK = blocks_per_stage();
    for (int q = 0; q < MK; ++q) {
      const gd* S = PS + 6 * blk(i, q);
      add(NS + 0, NS + 0, S[0]);
      add(NS + 1, NS + 0, S[1]);
      add(NS + 1, NS + 1, S[2]);
      add(NS + 3, NS + 0, S[3]);
      add(NS + 3, NS + 1, S[4]);
      add(NS + 3, NS + 3, S[5]);
    }
    // terminal slack block (i == N-1): Hs = 10000 sf + dw (+ proximity), Et = dc (+ eR) + st^2 / Hs
    if (!PT && i == N - 1) {
      for (int k = 0; k < NS; ++k) {
        const double st = scE[D.eTerm + k];
        const double Et = term_E(k, ls, dw, dc);
        add(NS + k, NS + k, st * st / Et);
      }
    }
    // the Riccati path reads only the w x w block [NS, nb)^2 of K (riccati_factor[_mfma]); the block LDL^T
    // path (point formulation, experiments) reads all of it
    constexpr int R0 = (!PT && HTP_COMPACT_STAGE) ? NS : 0;
    for (int r = R0; r < NBMAX; ++r)
      for (int q = R0; q < NBMAX; ++q)
        if (r < nb && q < nb) K[r * nb + q] = Kl[r >= q ? r * (r + 1) / 2 + q : q * (q + 1) / 2 + r];
    // Riccati records: reciprocal scaling of this stage's multiplier rows
    {
      gd* Ss = A(L.LD) + (int64_t)i * nb * nb + SOFF;
      const int yb = (i == 0) ? 0 : D.eDyn + NS * (i - 1);
      for (int k = 0; k < NS; ++k) Ss[k] = 1.0 / scE[yb + k];
    }
    // off-diagonal block for i+1 (rows of block i+1, cols of block i)
    if (i < N - 1) {
      gd* O = A(L.Off) + (int64_t)(i + 1) * nb * nb;
      constexpr bool compact = !PT && HTP_COMPACT_STAGE;
      if (compact) {   // the Riccati reads only the jerk cross terms C (rows U0, U0+1; columns U0, U0+1, T0) of Off
        const int U0 = NS + 5;
        for (int a = 0; a < 2; ++a)
          for (int b = 0; b < 3; ++b) O[(U0 + a) * nb + U0 + b] = 0.0;
      } else {
        for (int q = 0; q < nb * nb; ++q) O[q] = 0.0;
      }
      double w[8], J[40];
      stage_w(x, i, w);
      dynJ8(w, J);
      gd* Js = A(L.LD) + (int64_t)i * nb * nb + JOFF;  // unscaled J_i (stride 8) for the Riccati records
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const double s_ = scE[D.eDyn + NS * i + k];
        if (!compact)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < D.nw) O[k * nb + NS + j] = -s_ * J[k * 8 + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) Js[k * 8 + j] = J[k * 8 + j];
      }
      if (PT && !ls && i < N - 2) {
        const int U0 = NS + 5;
        O[U0 * nb + U0] = -hs * 2.0;
        O[(U0 + 1) * nb + U0 + 1] = -hs * 2.0;
      }
      if (!PT && !ls && i < N - 2) {
        const double tau = tauv(x, i), h = dT * tau, ih2 = 1.0 / (h * h);
        const double Rs00 = 2 * par(P_R00), Rs01 = par(P_R01) + par(P_R10), Rs11 = 2 * par(P_R11);
        const int U0 = NS + 5, T0 = NS + 7;
        O[U0 * nb + U0] = -hs * Rs00 * ih2;
        O[U0 * nb + U0 + 1] = -hs * Rs01 * ih2;
        O[(U0 + 1) * nb + U0] = -hs * Rs01 * ih2;
        O[(U0 + 1) * nb + U0 + 1] = -hs * Rs11 * ih2;
        if (D.topt) {
          const double da = x[D.oU + NC * (i + 1)] - x[D.oU + NC * i];
          const double dw_ = x[D.oU + NC * (i + 1) + 1] - x[D.oU + NC * i + 1];
          const double k2 = -2.0 * ih2 / tau;
          O[U0 * nb + T0] = hs * k2 * (Rs00 * da + Rs01 * dw_);
          O[(U0 + 1) * nb + T0] = hs * k2 * (Rs01 * da + Rs11 * dw_);
        }
      }
    }
  }

  // ----------------------------------------- Bunch-Kaufman on an LDS block
  // a: n x n symmetric (full storage, row-major, stride nb); ip: pivots.
  // On exit: unit L in the strict lower part, D on the (sub)diagonal,
  // ip[k] >= 0: 1x1 pivot swapped with ip[k]; ip[k] = ip[k+1] = -(r+1): 2x2.
  HTP_HD HTP_FI void bk_factor(ld* a, li* ip, int n, int& neg, int& zero) {
    const int nb = D.nb;
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    ld* sh = c.lds + 4 * NBMAX * NBMAX;  // scalars
    int k = 0;
    while (k < n) {
      int kstep = 1, kp = k;
      if (c.lane == 0) {
        const double absakk = dabs(a[k * nb + k]);
        int imax = k;
        double colmax = 0.0;
        for (int r = k + 1; r < n; ++r)
          if (dabs(a[r * nb + k]) > colmax) { colmax = dabs(a[r * nb + k]); imax = r; }
        if (dmax(absakk, colmax) == 0.0) {
          kp = k; kstep = 1;
        } else if (absakk >= alpha * colmax) {
          kp = k; kstep = 1;
        } else {
          double rowmax = 0.0;
          for (int j = k; j < n; ++j)
            if (j != imax) rowmax = dmax(rowmax, dabs(a[imax * nb + j]));
          if (absakk >= alpha * colmax * (colmax / rowmax)) { kp = k; kstep = 1; }
          else if (dabs(a[imax * nb + imax]) >= alpha * rowmax) { kp = imax; kstep = 1; }
          else { kp = imax; kstep = 2; }
        }
        sh[0] = kp;
        sh[1] = kstep;
      }
      c.sync();
      kp = c.uniform_i((int)sh[0]);
      kstep = c.uniform_i((int)sh[1]);
      c.sync();
      const int kk = k + kstep - 1;
      if (kp != kk) {  // LAPACK-style interchange of rows/cols kk, kp inside the trailing block A(k:n,k:n)
        for (int j = k + c.lane; j < n; j += c.width) {
          const double t = a[kk * nb + j];
          a[kk * nb + j] = a[kp * nb + j];
          a[kp * nb + j] = t;
        }
        c.sync();
        for (int j = k + c.lane; j < n; j += c.width) {
          const double t = a[j * nb + kk];
          a[j * nb + kk] = a[j * nb + kp];
          a[j * nb + kp] = t;
        }
        c.sync();
      }
      if (kstep == 1) {
        const double d = a[k * nb + k];
        if (d == 0.0) zero = 1;
        if (d < 0.0) ++neg;
        const double id = d != 0.0 ? 1.0 / d : 0.0;
        const int m = n - k - 1;
        for (int e = c.lane; e < m * m; e += c.width) {
          const int r = k + 1 + e / m, q = k + 1 + e % m;
          a[r * nb + q] -= a[r * nb + k] * a[q * nb + k] * id;
        }
        c.sync();
        for (int r = k + 1 + c.lane; r < n; r += c.width) {
          a[r * nb + k] *= id;
          a[k * nb + r] = a[r * nb + k];
        }
        c.sync();
      } else {
        const double d11 = a[k * nb + k], d21 = a[(k + 1) * nb + k], d22 = a[(k + 1) * nb + k + 1];
        const double det = d11 * d22 - d21 * d21;
        if (det < 0.0) neg += 1;
        else if (det > 0.0) neg += (d11 + d22 < 0.0) ? 2 : 0;
        else zero = 1;
        const double i11 = d22 / det, i22 = d11 / det, i21 = -d21 / det;
        const int m = n - k - 2;
        for (int e = c.lane; e < m * m; e += c.width) {
          const int r = k + 2 + e / m, q = k + 2 + e % m;
          const double ar1 = a[r * nb + k], ar2 = a[r * nb + k + 1];
          const double aq1 = a[q * nb + k], aq2 = a[q * nb + k + 1];
          const double l1 = ar1 * i11 + ar2 * i21, l2 = ar1 * i21 + ar2 * i22;
          a[r * nb + q] -= l1 * aq1 + l2 * aq2;
        }
        c.sync();
        for (int r = k + 2 + c.lane; r < n; r += c.width) {
          const double ar1 = a[r * nb + k], ar2 = a[r * nb + k + 1];
          const double l1 = ar1 * i11 + ar2 * i21, l2 = ar1 * i21 + ar2 * i22;
          a[r * nb + k] = l1;
          a[r * nb + k + 1] = l2;
          a[k * nb + r] = l1;
          a[(k + 1) * nb + r] = l2;
        }
        c.sync();
      }
      if (c.lane == 0) {
        if (kstep == 1) ip[k] = kp;
        else { ip[k] = -(kp + 1); ip[k + 1] = -(kp + 1); }
      }
      c.sync();
      k += kstep;
    }
  }

  // out = A^{-1} from a BK factor (lane-parallel over (row, col) entries)
  HTP_HD HTP_FI void bk_inverse(const ld* a, const li* ip, int n, ld* out) {
    const int nb = D.nb;
    for (int e = c.lane; e < nb * nb; e += c.width) out[e] = ((e / nb) == (e % nb) && e / nb < n) ? 1.0 : 0.0;
    c.sync();
    int k = 0;
    while (k < n) {  // P then L^-1 on all columns
      if (ip[k] >= 0) {
        const int kp = ip[k];
        if (kp != k) {
          for (int q = c.lane; q < n; q += c.width) { const double t = out[k * nb + q]; out[k * nb + q] = out[kp * nb + q]; out[kp * nb + q] = t; }
          c.sync();
        }
        const int m = n - k - 1;
        for (int e = c.lane; e < m * n; e += c.width) {
          const int r = k + 1 + e / n, q = e % n;
          out[r * nb + q] -= a[r * nb + k] * out[k * nb + q];
        }
        c.sync();
        k += 1;
      } else {
        const int kp = -ip[k] - 1;
        if (kp != k + 1) {
          for (int q = c.lane; q < n; q += c.width) { const double t = out[(k + 1) * nb + q]; out[(k + 1) * nb + q] = out[kp * nb + q]; out[kp * nb + q] = t; }
          c.sync();
        }
        const int m = n - k - 2;
        for (int e = c.lane; e < m * n; e += c.width) {
          const int r = k + 2 + e / n, q = e % n;
          out[r * nb + q] -= a[r * nb + k] * out[k * nb + q] + a[r * nb + k + 1] * out[(k + 1) * nb + q];
        }
        c.sync();
        k += 2;
      }
    }
    // D^-1 (row operations, independent per column)
    for (int q = c.lane; q < n; q += c.width) {
      int kk = 0;
      while (kk < n) {
        if (ip[kk] >= 0) {
          out[kk * nb + q] /= a[kk * nb + kk];
          kk += 1;
        } else {
          const double d11 = a[kk * nb + kk], d21 = a[(kk + 1) * nb + kk], d22 = a[(kk + 1) * nb + kk + 1];
          const double det = d11 * d22 - d21 * d21;
          const double b1 = out[kk * nb + q], b2 = out[(kk + 1) * nb + q];
          out[kk * nb + q] = (d22 * b1 - d21 * b2) / det;
          out[(kk + 1) * nb + q] = (-d21 * b1 + d11 * b2) / det;
          kk += 2;
        }
      }
    }
    c.sync();
    k = n - 1;
    while (k >= 0) {  // L^-T then P^T
      if (ip[k] >= 0) {
        for (int q = c.lane; q < n; q += c.width) {
          double acc = out[k * nb + q];
          for (int r = k + 1; r < n; ++r) acc -= a[r * nb + k] * out[r * nb + q];
          out[k * nb + q] = acc;
        }
        c.sync();
        const int kp = ip[k];
        if (kp != k) {
          for (int q = c.lane; q < n; q += c.width) { const double t = out[k * nb + q]; out[k * nb + q] = out[kp * nb + q]; out[kp * nb + q] = t; }
          c.sync();
        }
        k -= 1;
      } else {
        for (int q = c.lane; q < n; q += c.width) {
          double a1 = out[k * nb + q], a0 = out[(k - 1) * nb + q];
          for (int r = k + 1; r < n; ++r) {
            a1 -= a[r * nb + k] * out[r * nb + q];
            a0 -= a[r * nb + k - 1] * out[r * nb + q];
          }
          out[k * nb + q] = a1;
          out[(k - 1) * nb + q] = a0;
        }
        c.sync();
        const int kp = -ip[k] - 1;
        if (kp != k) {
          for (int q = c.lane; q < n; q += c.width) { const double t = out[k * nb + q]; out[k * nb + q] = out[kp * nb + q]; out[kp * nb + q] = t; }
          c.sync();
        }
        k -= 2;
      }
    }
  }


  // ---------------------------------------------------------- Riccati path
  // Stage system with exact dynamics (dc == 0), written on the augmented state
  // z_i = [x_i, u_{i-1}, tau_{i-1}] and control v_i = [u_i, tau_i] so the jerk
  // coupling (optimizer.py:461-465) becomes stage-local.  Backward recursion
  //   Rt = R + B'PB, St = S + B'PA, K = -Rt^-1 St, P <- Q + A'PA + St'K.
  // The block-tridiagonal KKT system has IPOPT's inertia iff every Rt is
  // positive definite (Rt are the pivot blocks of the reduced Hessian).
  // Per-stage storage (slot i of L.LD): P_i [0,64), K_i [64,88).
  // Cholesky of the leading nv x nv (nv <= 3) block of R (stride 3).  Lc holds
  // the lower factor with the RECIPROCAL of each pivot on its diagonal, so the
  // solves multiply instead of divide.  Loops run to 3 with `j < nv` guards:
  // static register indices (no dynamic-index select chains).
  HTP_HD HTP_FI static bool chol3(const double* R, int nv, double* Lc) {
    for (int k = 0; k < 9; ++k) Lc[k] = 0.0;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j < nv) {
        double d = R[j * 3 + j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= Lc[j * 3 + k] * Lc[j * 3 + k];
        if (!(d > 0.0)) ok = false;
        const double id = 1.0 / sqrt(d);
        Lc[j * 3 + j] = id;
#pragma unroll
        for (int r = j + 1; r < 3; ++r) {
          if (r < nv) {
            double v = R[r * 3 + j];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= Lc[r * 3 + k] * Lc[j * 3 + k];
            Lc[r * 3 + j] = v * id;
          }
        }
      }
    }
    return ok;
  }
  HTP_HD HTP_FI static void chol3_solve(const double* Lc, int nv, double* b) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j < nv) {
#pragma unroll
        for (int k = 0; k < j; ++k) b[j] -= Lc[j * 3 + k] * b[k];
        b[j] *= Lc[j * 3 + j];
      }
    }
#pragma unroll
    for (int j = 2; j >= 0; --j) {
      if (j < nv) {
#pragma unroll
        for (int k = j + 1; k < 3; ++k)
          if (k < nv) b[j] -= Lc[k * 3 + j] * b[k];
        b[j] *= Lc[j * 3 + j];
      }
    }
  }

  // ---------------------------------------------- relaxed dynamics rows (restoration, delta_c > 0)
  // With delta_c > 0 or in the restoration phase (eliminated n/p: e_R on the diagonal) the y rows of
  // stage block i read  s (x_i - xh_i) - E y_i = b  (xh_i = F_{i-1} u_{i-1} + e_i the nominal state),
  // i.e.  x_i = xh_i + Eh yh_i  with  Eh = E / s^2  and  yh = s y.  Eliminating y_i (pivot -E: its 5
  // negative eigenvalues) and then x_i (pivot P_xx + Eh^-1, which must be positive definite for
  // IPOPT's inertia) turns the cost-to-go (P, p) over z_i into one over the NOMINAL zh_i.  With
  // S = Eh^1/2, A = S P_xx S, Mi = (I + A)^-1 (Cholesky L L' = I + A):
  //   P~[x,:] = S^-1 Mi S P[x,:],   P~[c,c] = P[c,c] - W_c' W_c  (W = L^-1 S P[x,:]),
  //   T = S Mi S = (P_xx + Eh^-1)^-1,   Q = S^-1 Mi S = (I + P_xx Eh)^-1;
  // no term is a difference of nearly equal numbers whether Eh is tiny (delta_c) or huge (restoration
  // rows whose n/p are far from their bounds: P~_xx -> Eh^-1, T -> P_xx^-1).  The solve passes use
  //   backward  w_x = Q r_x,  w_c = r_c - P[c,x] T r_x       (r = p - P e, the exact-dynamics w),
  //   forward   x_i = xh_i + T r_x,  yh_i = Q r_x             (r = p - P zh).
  // Exact inertia (Sylvester): every (I + A) and every Rt positive definite.  E = 0 (the
  // exact-dynamics iterations) is the plain recursion.
  HTP_HD HTP_FI void stage_Eh(int i, double dc, double* Eh) const {
    const gd* scE = A(L.scE);
    const int rowbase = (i == 0) ? 0 : D.eDyn + NS * (i - 1);
    for (int k = 0; k < NS; ++k) {
      const double e = dc + (rs ? A(L.eR)[rowbase + k] : 0.0);
      const double sc = scE[rowbase + k];
      Eh[k] = dmax(e / (sc * sc), 1e-300);
    }
  }
  // Cholesky of a symmetric 5x5 (row-major) into packed lower Lc (15) with RECIPROCAL pivots
  HTP_HD HTP_FI static bool chol5(const double* Am, double* Lc) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      double d = Am[j * NS + j];
#pragma unroll
      for (int k = 0; k < j; ++k) d -= Lc[j * (j + 1) / 2 + k] * Lc[j * (j + 1) / 2 + k];
      if (!(d > 0.0)) { ok = false; d = 1.0; }
      const double id = 1.0 / sqrt(d);
      Lc[j * (j + 1) / 2 + j] = id;
#pragma unroll
      for (int r = j + 1; r < NS; ++r) {
        double v = Am[r * NS + j];
#pragma unroll
        for (int k = 0; k < j; ++k) v -= Lc[r * (r + 1) / 2 + k] * Lc[j * (j + 1) / 2 + k];
        Lc[r * (r + 1) / 2 + j] = v * id;
      }
    }
    return ok;
  }
  HTP_HD HTP_FI static void chol5_fwd(const double* Lc, double* b) {  // b <- L^-1 b
#pragma unroll
    for (int j = 0; j < NS; ++j) {
#pragma unroll
      for (int k = 0; k < j; ++k) b[j] -= Lc[j * (j + 1) / 2 + k] * b[k];
      b[j] *= Lc[j * (j + 1) / 2 + j];
    }
  }
  HTP_HD HTP_FI static void chol5_bwd(const double* Lc, double* b) {  // b <- L^-T b
#pragma unroll
    for (int j = NS - 1; j >= 0; --j) {
#pragma unroll
      for (int k = j + 1; k < NS; ++k) b[j] -= Lc[k * (k + 1) / 2 + j] * b[k];
      b[j] *= Lc[j * (j + 1) / 2 + j];
    }
  }
  // P8 (LDS, 8 x 8 stride 8, symmetric): cost-to-go of stage block i -> its relaxed form P~ (in place,
  // symmetric); T_i to Trec[0, 25) and Q_i to Trec[25, 50) (global) for the solve passes.
  // Wl: LDS scratch (105 doubles).  Returns false if I + S P_xx S is not positive definite.
  HTP_HD HTP_FI bool relax_P(ld* P8, int i, double dc, ld* Wl, gd* Trec) {
    double Eh[NS], S[NS], Am[NS * NS], Lc[15];
    stage_Eh(i, dc, Eh);
    for (int k = 0; k < NS; ++k) S[k] = sqrt(Eh[k]);
    for (int a = 0; a < NS; ++a)
      for (int b = 0; b < NS; ++b) Am[a * NS + b] = (a == b ? 1.0 : 0.0) + S[a] * P8[a * 8 + b] * S[b];
    const bool ok = chol5(Am, Lc);
    ld* Wm = Wl;         // 5 x 8: W = L^-1 S P[x,:]
    ld* Ym = Wl + 40;    // 5 x 8: Y = Mi S P[x,:]
    ld* Mm = Wl + 80;    // 5 x 5: Mi
    for (int q = c.lane; q < 8 + NS; q += c.width) {   // column q of S P[x,:] (q < 8) or of I (q >= 8)
      double v[NS];
      for (int a = 0; a < NS; ++a) v[a] = (q < 8) ? S[a] * P8[a * 8 + q] : (a == q - 8 ? 1.0 : 0.0);
      chol5_fwd(Lc, v);
      if (q < 8)
        for (int a = 0; a < NS; ++a) Wm[a * 8 + q] = v[a];
      chol5_bwd(Lc, v);
      for (int a = 0; a < NS; ++a) {
        if (q < 8) Ym[a * 8 + q] = v[a];
        else Mm[a * NS + (q - 8)] = v[a];
      }
    }
    c.sync();
    constexpr int PE = (64 + Ctx::width - 1) / Ctx::width;
    double pn[PE];
    {
      int u = 0;
      for (int e = c.lane; e < 64; e += c.width, ++u) {
        const int r = e / 8, q = e % 8;
        double v;
        if (r < NS && q < NS) v = 0.5 * (Ym[r * 8 + q] / S[r] + Ym[q * 8 + r] / S[q]);
        else if (r < NS) v = Ym[r * 8 + q] / S[r];
        else if (q < NS) v = Ym[q * 8 + r] / S[q];
        else {
          v = P8[e];
          for (int a = 0; a < NS; ++a) v -= Wm[a * 8 + r] * Wm[a * 8 + q];
        }
        pn[u] = v;
      }
    }
    for (int e = c.lane; e < 2 * NS * NS; e += c.width) {
      const int f = e < NS * NS ? e : e - NS * NS, a = f / NS, b = f % NS;
      const double mi = 0.5 * (Mm[a * NS + b] + Mm[b * NS + a]);
      Trec[e] = e < NS * NS ? S[a] * mi * S[b] : mi * S[b] / S[a];
    }
    c.sync();
    {
      int u = 0;
      for (int e = c.lane; e < 64; e += c.width, ++u) P8[e] = pn[u];
    }
    c.sync();
    return ok;
  }
  HTP_HD HTP_FI gd* trec(int i) const { return A(L.fac) + (int64_t)i * D.nb * D.nb; }
  bool ric_relax = false;   // the current stage factor uses relaxed dynamics rows (T records valid)

  // returns number of stages whose Rt is not positive definite
  HTP_HD HTP_FI int riccati_factor(double dc) {
    const int N = D.N, nb = D.nb, nv = D.nw - NS, nz = NS + nv;
    ld* Pc = c.lds;          // 8x8 (stride 8): P_{i+1}
    ld* Pn = c.lds + 64;     // 8x8: P_i
    ld* Hw = c.lds + 128;    // 8x8 stage Hessian over w
    ld* Jm = c.lds + 192;    // 5x8 unscaled dF/dw
    ld* Cb = c.lds + 232;    // 2x3 jerk cross C_{i-1}
    ld* PJx = c.lds + 240;   // 8x5
    ld* PB = c.lds + 280;    // 8x3
    ld* Rt = c.lds + 304;    // 3x3
    ld* St = c.lds + 313;    // 3x8
    ld* AtPA = c.lds + 337;  // 5x5
    ld* Kl = c.lds + 362;    // 3x8
    int bad = 0;             // relax_P scratch: c.lds + 240 .. 345 (PJx .. AtPA, dead between stages)
    // stage N-1: P = [[H_xx, 0], [0, 0]]
    {
      const gd* Kst = A(L.Kst) + (int64_t)(N - 1) * nb * nb;
      for (int e = c.lane; e < 64; e += c.width) {
        const int r = e / 8, q = e % 8;
        Pc[e] = (r < NS && q < NS) ? Kst[(NS + r) * nb + NS + q] : 0.0;
      }
      gd* Ps = A(L.LD) + (int64_t)(N - 1) * nb * nb;
      c.sync();
      for (int e = c.lane; e < 64; e += c.width) Ps[e] = Pc[e];
    }
    if (ric_relax && !relax_P(Pc, N - 1, dc, c.lds + 240, trec(N - 1))) ++bad;
    // stage records (H_w 64 | J 40 | C_{i-1} 6), prefetched one stage ahead
    ld* fb0 = c.lds + 400;
    ld* fb1 = c.lds + 512;
    auto rec = [&](int i, int e) -> double {
      if (e < 64) {
        const int r = e / 8, q = e % 8;
        return (r < D.nw && q < D.nw) ? A(L.Kst)[(int64_t)i * nb * nb + (NS + r) * nb + NS + q] : 0.0;
      }
      if (e < 104) return A(L.LD)[(int64_t)i * nb * nb + JOFF + (e - 64)];  // J_i, unscaled, stride 8
      if (e < 110) {
        const int a = (e - 104) / 3, b = (e - 104) % 3;
        return (i >= 1 && b < nv) ? A(L.Off)[(int64_t)i * nb * nb + (NS + 5 + a) * nb + NS + 5 + b] : 0.0;
      }
      return 0.0;
    };
    constexpr int PF = (112 + Ctx::width - 1) / Ctx::width;
    if (N >= 2)
      for (int e = c.lane; e < 112; e += c.width) fb0[e] = rec(N - 2, e);
    c.sync();
    for (int i = N - 2; i >= 0; --i) {
      HTP_PROF0();
      ld* cur = ((N - 2 - i) & 1) ? fb1 : fb0;
      ld* nxt = ((N - 2 - i) & 1) ? fb0 : fb1;
      double pre[PF];
      for (int u = 0; u < PF; ++u) {
        const int e = c.lane + u * c.width;
        pre[u] = (i > 0 && e < 112) ? rec(i - 1, e) : 0.0;
      }
      for (int e = c.lane; e < 64; e += c.width) Hw[e] = cur[e];
      for (int e = c.lane; e < 40; e += c.width) Jm[e] = cur[64 + e];
      for (int e = c.lane; e < 6; e += c.width) Cb[e] = cur[104 + e];
      if (i > 0)
        for (int u = 0; u < PF; ++u) {
          const int e = c.lane + u * c.width;
          if (e < 112) nxt[e] = pre[u];
        }
      c.sync();
      HTP_PROF(0);
      // PJx = P[:,0:5] Jx ; PB = P[:,0:5] Jv + P[:,5:5+nv]
      for (int e = c.lane; e < nz * (NS + nv); e += c.width) {
        const int r = e / (NS + nv), q = e % (NS + nv);
        double acc = 0.0;
        for (int t = 0; t < NS; ++t) acc += Pc[r * 8 + t] * Jm[t * 8 + q];
        if (q < NS) PJx[r * 5 + q] = acc;
        else PB[r * 3 + (q - NS)] = acc + Pc[r * 8 + NS + (q - NS)];
      }
      c.sync();
      HTP_PROF(1);
      // Rt = R + B'PB ; St = S + B'PA ; AtPA = Jx' P Jx
      for (int e = c.lane; e < nv * nv + nv * nz + 25; e += c.width) {
        if (e < nv * nv) {
          const int a = e / nv, b = e % nv;
          double acc = Hw[(NS + a) * 8 + NS + b] + PB[(NS + a) * 3 + b];
          for (int t = 0; t < NS; ++t) acc += Jm[t * 8 + NS + a] * PB[t * 3 + b];
          Rt[a * 3 + b] = acc;
        } else if (e < nv * nv + nv * nz) {
          const int f = e - nv * nv, a = f / nz, q = f % nz;
          double acc;
          if (q < NS) {
            acc = Hw[(NS + a) * 8 + q];
            for (int t = 0; t < NS; ++t) acc += PB[t * 3 + a] * Jm[t * 8 + q];
          } else {
            acc = (a < 2) ? Cb[a * 3 + (q - NS)] : 0.0;
          }
          St[a * 8 + q] = acc;
        } else {
          const int f = e - nv * nv - nv * nz, r = f / 5, q = f % 5;
          double acc = 0.0;
          for (int t = 0; t < NS; ++t) acc += Jm[t * 8 + r] * PJx[t * 5 + q];
          AtPA[r * 5 + q] = acc;
        }
      }
      c.sync();
      HTP_PROF(2);
      // Cholesky of Rt (redundantly per lane) ; K = -Rt^-1 St (lane per column)
      double Rl[9], Lc[9];
      for (int k = 0; k < 9; ++k) Rl[k] = (k / 3 < nv && k % 3 < nv) ? Rt[k] : 0.0;
      const bool pd = chol3(Rl, nv, Lc);
      if (!pd) ++bad;
      for (int q = c.lane; q < nz; q += c.width) {
        double col[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int a = 0; a < 3; ++a)
          if (a < nv) col[a] = St[a * 8 + q];
        if (pd) chol3_solve(Lc, nv, col);
#pragma unroll
        for (int a = 0; a < 3; ++a)
          if (a < nv) Kl[a * 8 + q] = -col[a];
      }
      c.sync();
      HTP_PROF(3);
      // P_i = Q + A'PA + St'K
      gd* Ps = A(L.LD) + (int64_t)i * nb * nb;
      for (int e = c.lane; e < 64; e += c.width) {
        const int r = e / 8, q = e % 8;
        double acc = 0.0;
        if (r < nz && q < nz) {
          if (r < NS && q < NS) acc = Hw[r * 8 + q] + AtPA[r * 5 + q];
          for (int a = 0; a < nv; ++a) acc += St[a * 8 + r] * Kl[a * 8 + q];
        }
        Pn[e] = acc;
        Ps[e] = acc;
      }
      for (int e = c.lane; e < 24; e += c.width) Ps[64 + e] = Kl[e];
      for (int e = c.lane; e < 9; e += c.width) Ps[88 + e] = Lc[e];
      c.sync();
      for (int e = c.lane; e < 64; e += c.width) Pc[e] = 0.5 * (Pn[e] + Pn[(e % 8) * 8 + e / 8]);  // symmetrise
      c.sync();
      if (ric_relax && !relax_P(Pc, i, dc, c.lds + 240, trec(i))) ++bad;
      HTP_PROF(5);
      if (HTP_RIC_EARLY_EXIT && bad) break;   // wrong inertia is decided (the caller rejects or re-factors)
    }
    return bad;
  }

#if defined(__HIPCC__) || defined(HTP_EMU_WAVE)
  // ------------------------------------------------ Riccati recursion on the matrix core
  // Same recursion as riccati_factor / riccati_solve, written as 16x16 fp64 MFMA tiles over the
  // augmented stage variables u_i = [z_i (rows 0..7, z = [x, u_{i-1}, tau_{i-1}] zero-padded to 8) ;
  // v_i (rows 8..8+nv)], with z_{i+1} = F_i u_i + e_{i+1},  F_i = [[Jx, 0, Jv], [0, 0, I]]:
  //   factor:  M = H_i + F_i' P_{i+1} F_i,  Rt = M_vv, St = M_vz, K = -Rt^-1 St, P_i = M_zz + St' K
  //   backward: w = p_{i+1} - P_{i+1} e_{i+1}, g = [q_i; r_i] + F_i' w, rt_i = g_v, p_i = g_z + K_i' rt_i
  //   forward:  y_i = p_i - P_i z_i, u_i = [z_i; Rt^-1 rt_i + K_i z_i], z_{i+1} = F_i u_i + e_{i+1}
  // Layout (v_mfma_f64_16x16x4f64): lane l holds column l&15 and rows (l>>4) + 4r in register r;
  // vectors live in column 0.  A symmetric P in that layout is the A operand of P F (k-step s =
  // register s); F's rows (FR) are the B operand of P F and the A operand of F' (.); every product's
  // accumulator is the B operand of the next one, so no lane shuffles are needed; Rt / St of the
  // factor go through LDS.  5 MFMAs per stage in the factor and in each solve pass.
  static constexpr int V0 = 8;  // row of v_i in u_i
  // F_i[frow][fcol] (fcol over u_i): stage-independent source of this lane's element
  struct FSrc { int kind, off; };  // 0 zero, 3 J (offset in the LD slot), 4 one
  template <int NV>
  HTP_HD HTP_FI FSrc f_src(int frow, int fcol) const {
    constexpr int nv = NV;
    if (frow < NS) {
      if (fcol < NS) return FSrc{3, JOFF + frow * 8 + fcol};
      if (fcol >= V0 && fcol < V0 + nv) return FSrc{3, JOFF + frow * 8 + NS + (fcol - V0)};
      return FSrc{0, 0};
    }
    if (frow < NS + nv && fcol == V0 + (frow - NS)) return FSrc{4, 0};
    return FSrc{0, 0};
  }
  HTP_HD HTP_FI double f_get(const FSrc& f, const gd* slot) const {
    return f.kind == 3 ? slot[f.off] : (f.kind == 4 ? 1.0 : 0.0);
  }

  // The stage chain's v-block width nv = nw - 5 (2: u; 3: u and tau with time-optimal scaling) as a template
  // argument: every per-lane index test and the 3 x 3 Cholesky unroll at compile time (28 % fewer cycles per
  // factor stage, tools/micro/ric_micro.hip); the arithmetic is unchanged.
  HTP_HD HTP_FI int riccati_factor_mfma(double dc, bool fb = false) {
    if constexpr (PT) return riccati_factor_mfma_t<2, false>(dc);
    else {
#if HTP_BWD_FUSE
      if (fb && !ric_relax) return D.nw == NS + 3 ? riccati_factor_mfma_t<3, true>(dc) : riccati_factor_mfma_t<2, true>(dc);
#endif
      return D.nw == NS + 3 ? riccati_factor_mfma_t<3, false>(dc) : riccati_factor_mfma_t<2, false>(dc);
    }
  }
  // FB: also the backward pass of riccati_solve_mfma_t for the stage right-hand side V already in the workspace
  // (exact dynamics): p_i, rt_i into X exactly as that pass writes them.
  template <int NV, bool FB>
  HTP_HD HTP_FI int riccati_factor_mfma_t(double dc) {
    static_assert(!FB || HTP_FAC_SB > 0, "the fused backward pass reads its records from the factor staging");
    constexpr int nv = NV, nz = NS + nv;
    const int N = D.N, nb = D.nb;
    const int64_t nb2 = (int64_t)nb * nb;
    const int col = c.lane & 15, rg = c.lane >> 4;
    ld* Mv = c.lds;           // 3 x 16: rows v of M
    ld* Pb = c.lds + 48;      // 8 x 8: P_i before symmetrisation
    // stage-independent gather maps of this lane: H in the C layout (4 registers), F rows (2 registers)
    // H sources: 0 zero, 1 Kst w-block (offset), 2 Off jerk cross (offset)
    int hk[4], ho[4];
    FSrc fs[2];
    auto widx = [&](int a) { return a < NS ? a : (a >= V0 && a < V0 + nv ? NS + (a - V0) : -1); };
    for (int r = 0; r < 4; ++r) {
      const int row = rg + 4 * r, wr = widx(row), wc = widx(col);
      hk[r] = 0; ho[r] = 0;
      if (wr >= 0 && wc >= 0) { hk[r] = 1; ho[r] = (NS + wr) * nb + NS + wc; }
      else if (row >= V0 && row - V0 < 2 && col >= NS && col < nz) { hk[r] = 2; ho[r] = (NS + 5 + row - V0) * nb + NS + 5 + (col - NS); }
      else if (col >= V0 && col - V0 < 2 && row >= NS && row < nz) { hk[r] = 2; ho[r] = (NS + 5 + col - V0) * nb + NS + 5 + (row - NS); }
    }
    for (int sgm = 0; sgm < 2; ++sgm) fs[sgm] = f_src<NV>(rg + 4 * sgm, col);
    const gd* Kst = A(L.Kst);
    const gd* Off = A(L.Off);
    const gd* LDa = A(L.LD);
#if HTP_FILL_SEL
    // every record load issued unconditionally from an in-range address, then selected: a load under a per-lane
    // branch let the compiler's wait-count pass put a vmcnt(0) wait between the batch's loads
    auto ld_h = [&](int i, double* h) {
      for (int r = 0; r < 4; ++r) {
        const gd* src = hk[r] == 2 ? Off : Kst;
        const double t = src[(int64_t)i * nb2 + ho[r]];
        h[r] = (hk[r] == 1 || (hk[r] == 2 && i >= 1)) ? t : 0.0;
      }
    };
    auto ld_f = [&](int i, double* f) {
      for (int sgm = 0; sgm < 2; ++sgm) {
        const double t = LDa[(int64_t)i * nb2 + (fs[sgm].kind == 3 ? fs[sgm].off : 0)];
        f[sgm] = fs[sgm].kind == 3 ? t : (fs[sgm].kind == 4 ? 1.0 : 0.0);
      }
    };
#else
    auto ld_h = [&](int i, double* h) {
      for (int r = 0; r < 4; ++r) {
        double v = 0.0;
        if (hk[r] == 1) v = Kst[(int64_t)i * nb2 + ho[r]];
        else if (hk[r] == 2 && i >= 1) v = Off[(int64_t)i * nb2 + ho[r]];
        h[r] = v;
      }
    };
    auto ld_f = [&](int i, double* f) {
      for (int sgm = 0; sgm < 2; ++sgm) f[sgm] = f_get(fs[sgm], LDa + (int64_t)i * nb2);
    };
#endif
    // P_{N-1} = [[H_xx, 0], [0, 0]]
    dbl4 Pc;
    {
      gd* Ps = A(L.LD) + (int64_t)(N - 1) * nb2;
      for (int r = 0; r < 4; ++r) {
        const int row = rg + 4 * r;
        const double v = (row < NS && col < NS) ? Kst[(int64_t)(N - 1) * nb2 + (NS + row) * nb + NS + col] : 0.0;
        Pc[r] = v;
        if (row < 8 && col < 8) Ps[row * 8 + col] = v;
        if (FB && row < 8 && col < 8) Pb[row * 8 + col] = v;   // P_{N-1} as the solve's first stage reads it
      }
    }
    int bad = 0;
    const gd* Vg = A(L.V);
    gd* Xg = A(L.X);
#if HTP_HOIST
    gd* const LDw = uptr(A(L.LD));
    const int ln = c.lane;
    const bool relax_f = c.uniform_i(ric_relax ? 1 : 0) != 0;
#else
    gd* const LDw = nullptr;
    const int ln = 0;
    const bool relax_f = false;
#endif
    const bool c0 = col == 0;
    dbl4 pv = {0.0, 0.0, 0.0, 0.0};                  // the solve's p_{i+1} (riccati_solve_mfma_t, backward)
    if constexpr (FB) {
      for (int r = 0; r < 2; ++r) {
        const int row = rg + 4 * r;
        pv[r] = (c0 && row < NS) ? Vg[(int64_t)(N - 1) * nb + NS + row] : 0.0;
      }
      gd* Xl = Xg + (int64_t)(N - 1) * nb;
      for (int r = 0; r < 2; ++r) {
        const int row = rg + 4 * r;
        if (c0 && row < 8) Xl[row] = pv[r];
      }
      c.sync();
    }
    // relaxed rows: P_i goes through LDS (Pb) into relax_P and back into the C-layout registers
    auto relax_regs = [&](int i) {
      for (int r = 0; r < 2; ++r) {
        const int row = rg + 4 * r;
        if (col < 8) Pb[row * 8 + col] = Pc[r];
      }
      c.sync();
      if (!relax_P(Pb, i, dc, c.lds + 112, trec(i))) ++bad;
      for (int r = 0; r < 2; ++r) {
        const int row = rg + 4 * r;
        Pc[r] = (row < nz && col < nz) ? (double)Pb[row * 8 + col] : 0.0;
      }
      c.sync();
    };
    if (ric_relax) relax_regs(N - 1);
    double hcur[4], fcur[2];
#if HTP_FAC_SB > 0
    // Stage records through this lane's slice of the LDS ring (free during the factor): every HTP_FAC_SB stages
    // one batch of 6 HTP_FAC_SB loads per lane, so the chain waits for memory once per batch instead of once per
    // stage (a stage's work is shorter than a load's latency under load, and every load also waits for the
    // previous stages' P / K / chol stores, which the in-order vmcnt counter places before it).  Same values.
    ld* fring = c.lds + RING_OFF;
    constexpr int FW = FB ? FAC_W_FB : 6;   // per stage: H (4), F (2)[, e_{i+1} (2), [q_i; r_i] (3)]
    // the solve's stage-i record (riccati_solve_mfma_t ld_b): e_{i+1} = V_{i+1} / sc, [q_i; r_i] from V_i
    auto ld_s = [&](int i, double* e) {
      for (int sgm = 0; sgm < 2; ++sgm) {
        const int row = rg + 4 * sgm;
        const bool on = c0 && row < NS;
        const int rr = on ? row : 0;
        const double a = Vg[(int64_t)(i + 1) * nb + rr], b = LDa[(int64_t)(i + 1) * nb2 + SOFF + rr];
        e[sgm] = on ? a * b : 0.0;
      }
      for (int r = 0; r < 3; ++r) {
        const int row = rg + 4 * r;
        const bool on1 = c0 && row < NS, on2 = c0 && row >= V0 && row < V0 + nv;
        const int off = on1 ? NS + row : (on2 ? NS + NS + (row - V0) : 0);
        const double t = Vg[(int64_t)i * nb + off];
        e[2 + r] = (on1 || on2) ? t : 0.0;
      }
    };
    auto fac_fill = [&](int hi) {   // stages hi, hi - 1, ..., hi - HTP_FAC_SB + 1 (those >= 0)
      double v[HTP_FAC_SB][FW];
#pragma unroll
      for (int sb = 0; sb < HTP_FAC_SB; ++sb) {
        const int st = hi - sb >= 0 ? hi - sb : 0;
        ld_h(st, v[sb]);
        ld_f(st, v[sb] + 4);
        if constexpr (FB) ld_s(st, v[sb] + 6);
      }
#pragma unroll
      for (int sb = 0; sb < HTP_FAC_SB; ++sb)
#pragma unroll
        for (int k = 0; k < FW; ++k) fring[(sb * FW + k) * 64 + (HTP_HOIST ? ln : (int)c.lane)] = v[sb][k];
    };
    for (int i = N - 2; i >= 0; --i) {
      HTP_PROF0();
      const int sb = (N - 2 - i) % HTP_FAC_SB;
      if (sb == 0) fac_fill(i);
      const int lnc = HTP_HOIST ? ln : (int)c.lane;
      for (int r = 0; r < 4; ++r) hcur[r] = fring[(sb * FW + r) * 64 + lnc];
      fcur[0] = fring[(sb * FW + 4) * 64 + lnc];
      fcur[1] = fring[(sb * FW + 5) * 64 + lnc];
      // the solve's -P_{i+1} (A operand, from the unsymmetrised P_{i+1} the factor stored: Pb still holds it)
      double smp[2], sre[5];
      if constexpr (FB) {
        for (int sgm = 0; sgm < 2; ++sgm) {
          const int k = rg + 4 * sgm;
          smp[sgm] = -((col < nz && k < nz) ? (double)Pb[col * 8 + k] : 0.0);
        }
        for (int k = 0; k < 5; ++k) sre[k] = fring[(sb * FW + 6 + k) * 64 + lnc];
      }
#else
    double hnxt[4], fnxt[2];
    if (N >= 2) { ld_h(N - 2, hcur); ld_f(N - 2, fcur); }
    for (int i = N - 2; i >= 0; --i) {
      HTP_PROF0();
      if (i > 0) { ld_h(i - 1, hnxt); ld_f(i - 1, fnxt); }  // next stage's record, in flight during this one
      const int lnc = HTP_HOIST ? ln : (int)c.lane;
      double smp[2], sre[5];
#endif
      dbl4 Y = {0.0, 0.0, 0.0, 0.0};
      Y = Ctx::mfma16(Pc[0], fcur[0], Y);
      Y = Ctx::mfma16(Pc[1], fcur[1], Y);
      dbl4 M = {hcur[0], hcur[1], hcur[2], hcur[3]};
      M = Ctx::mfma16(fcur[0], Y[0], M);
      M = Ctx::mfma16(fcur[1], Y[1], M);
      if (rg < nv) Mv[rg * 16 + col] = M[2];  // rows V0 + rg (register 2)
      c.sync();
      HTP_PROF(1);
      dbl4 sg = {0.0, 0.0, 0.0, 0.0};
      if constexpr (FB) {                            // w = p - P e;  g = [q; r] + F' w
        dbl4 w = Ctx::mfma16(smp[0], sre[0], pv);
        w = Ctx::mfma16(smp[1], sre[1], w);
        sg = dbl4{sre[2], sre[3], sre[4], 0.0};
        sg = Ctx::mfma16(fcur[0], w[0], sg);
        sg = Ctx::mfma16(fcur[1], w[1], sg);
      }
      double Rl[9], Lc[9];
      for (int k = 0; k < 9; ++k) Rl[k] = (k / 3 < nv && k % 3 < nv) ? Mv[(k / 3) * 16 + V0 + k % 3] : 0.0;
      const bool pd = chol3(Rl, nv, Lc);
      if (!pd) ++bad;
      double stc[3] = {0.0, 0.0, 0.0};
      for (int a = 0; a < 3; ++a)
        if (a < nv && col < nz) stc[a] = Mv[a * 16 + col];
      const double stA = (rg < nv && col < nz) ? stc[rg] : 0.0;  // St' as the A operand: St[rg][col]
      if (pd) chol3_solve(Lc, nv, stc);
      const double kB = (rg < nv && col < nz) ? -stc[rg] : 0.0;  // K[rg][col] as the B operand
      HTP_PROF(3);
      const dbl4 Pn = Ctx::mfma16(stA, kB, M);
      if constexpr (FB) {                            // p = g_z + K' rt;  X_i = [p_i; rt_i]
        const double kt = (rg < nv && col < nz) ? kB : 0.0;
        pv = Ctx::mfma16(kt, sg[2], sg);
        gd* Xi = Xg + (int64_t)i * nb;
        for (int r = 0; r < 2; ++r) {
          const int row = rg + 4 * r;
          if (c0 && row < nz) Xi[row] = pv[r];
        }
        if (c0 && rg < nv) Xi[nz + rg] = sg[2];
      }
      gd* Ps = (HTP_HOIST ? LDw : A(L.LD)) + (int64_t)i * nb2;
      for (int r = 0; r < 2; ++r) {
        const int row = rg + 4 * r;
        const double v = (row < nz && col < nz) ? Pn[r] : 0.0;
        if (col < 8) { Pb[row * 8 + col] = v; Ps[row * 8 + col] = v; }
      }
      if (rg < 3 && col < 8) Ps[64 + rg * 8 + col] = (rg < nv && col < nz) ? kB : 0.0;
      if (lnc < 9) Ps[88 + lnc] = Lc[lnc];
      c.sync();
      for (int r = 0; r < 4; ++r) {  // P_i = (Pn + Pn') / 2, zero outside nz x nz
        const int row = rg + 4 * r;
        Pc[r] = (r < 2 && row < nz && col < nz) ? 0.5 * (Pb[row * 8 + col] + Pb[col * 8 + row]) : 0.0;
      }
      c.sync();
      if (HTP_HOIST ? relax_f : ric_relax) relax_regs(i);
#if HTP_FAC_SB == 0
      for (int r = 0; r < 4; ++r) hcur[r] = hnxt[r];
      fcur[0] = fnxt[0];
      fcur[1] = fnxt[1];
#endif
      HTP_PROF(5);
      // A non-positive-definite pivot decides the inertia (wrong: factor_ic perturbs and re-factors; the point
      // formulation's block LDL^T re-derives it from the assembled blocks): the remaining stages are not needed.
      // Wave-uniform (every lane holds the same pivot test); successful factorizations are unchanged.
      if (HTP_RIC_EARLY_EXIT && bad) break;
    }
    return bad;
  }

  // Sig = K^-1 [x_{N-1}, x_{N-1}] of the stage chain (point formulation's terminal rows, terminal_schur):
  // the two Riccati passes with the five unit right-hand sides at x_{N-1} carried as columns 0..4 of the
  // 16-wide MFMA tiles (the single-vector passes use column 0 only), so one pass costs the MFMAs of one
  // solve.  The right-hand side is zero outside x_{N-1}: backward p_{N-1} = [I; 0], w = p (e = 0);
  // forward z_0 = 0.  Per-stage p_i (8 x 5) and rt_i (3 x 5) go to the fac slot after relax_P's T / Q.
  // Records are read straight from HBM one stage ahead.  Result: sig[5 x 5] (global).
  HTP_HD HTP_FI void riccati_sigma_mfma(gd* sig) {
    if (D.nw == NS + 3) riccati_sigma_mfma_t<3>(sig);
    else riccati_sigma_mfma_t<2>(sig);
  }
  template <int NV>
  HTP_HD HTP_FI void riccati_sigma_mfma_t(gd* sig) {
    constexpr int nv = NV, nz = NS + nv;
    const int N = D.N, nb = D.nb;
    const int64_t nb2 = (int64_t)nb * nb;
    const int col = c.lane & 15, rg = c.lane >> 4;
    const bool cw = col < NS;                 // a right-hand-side column
    const gd* LDa = A(L.LD);
    gd* Fa = A(L.fac);
    constexpr int PO = 50, RO = 90;           // p_i [8][5] and rt_i [3][5] in fac slot i
    FSrc fT[2], fA[3];
    for (int sgm = 0; sgm < 2; ++sgm) fT[sgm] = f_src<NV>(rg + 4 * sgm, col);
    for (int sgm = 0; sgm < 3; ++sgm) fA[sgm] = f_src<NV>(col, rg + 4 * sgm);
    auto p_at = [&](const gd* slot, int sgm) {
      const int k = rg + 4 * sgm;
      return (col < nz && k < nz) ? (double)slot[col * 8 + k] : 0.0;
    };
    auto t_at = [&](const gd* tr, int sgm, int which) {
      const int k = rg + 4 * sgm;
      return (col < NS && k < NS) ? (double)tr[which * NS * NS + col * NS + k] : 0.0;
    };
    const bool rlx = ric_relax;
    const dbl4 z4 = {0.0, 0.0, 0.0, 0.0};
    // ---------------- backward: p_{N-1} = [I_5; 0] (columns 0..4)
    dbl4 pv = z4;
    for (int r = 0; r < 2; ++r) {
      const int row = rg + 4 * r;
      pv[r] = (cw && row == col) ? 1.0 : 0.0;
    }
    auto st_p = [&](int i, const dbl4& v) {
      gd* d = Fa + (int64_t)i * nb2 + PO;
      for (int r = 0; r < 2; ++r) {
        const int row = rg + 4 * r;
        if (cw && row < 8) d[row * NS + col] = v[r];
      }
    };
    st_p(N - 1, pv);
    struct BR { double mp[2], ft[2], kt, ta[2], qa[2]; };
    auto ld_b = [&](int i, BR& R) {
      const gd* slot = LDa + (int64_t)i * nb2;
      const gd* nslot = slot + nb2;
      const gd* tr = Fa + (int64_t)(i + 1) * nb2;
      for (int sgm = 0; sgm < 2; ++sgm) {
        R.mp[sgm] = -p_at(nslot, sgm);
        R.ft[sgm] = f_get(fT[sgm], slot);
        R.ta[sgm] = rlx ? t_at(tr, sgm, 0) : 0.0;
        R.qa[sgm] = rlx ? t_at(tr, sgm, 1) : 0.0;
      }
      R.kt = (rg < nv && col < nz) ? (double)slot[64 + rg * 8 + col] : 0.0;
    };
    BR bc, bn;
    if (N >= 2) ld_b(N - 2, bc);
    for (int i = N - 2; i >= 0; --i) {
      if (i > 0) ld_b(i - 1, bn);
      dbl4 w = pv;                                   // w = p - P e, e = 0
      if (rlx) {
        dbl4 t = Ctx::mfma16(bc.ta[0], w[0], z4);
        t = Ctx::mfma16(bc.ta[1], w[1], t);
        dbl4 q = Ctx::mfma16(bc.qa[0], w[0], z4);
        q = Ctx::mfma16(bc.qa[1], w[1], q);
        w = Ctx::mfma16(bc.mp[0], t[0], w);
        w = Ctx::mfma16(bc.mp[1], t[1], w);
        w[0] = q[0];
        if (rg == 0) w[1] = q[1];
      }
      dbl4 g = z4;                                   // g = F' w ([q; r] = 0)
      g = Ctx::mfma16(bc.ft[0], w[0], g);
      g = Ctx::mfma16(bc.ft[1], w[1], g);
      pv = Ctx::mfma16(bc.kt, g[2], g);              // p = g_z + K' rt
      st_p(i, pv);
      gd* rt = Fa + (int64_t)i * nb2 + RO;
      if (cw && rg < nv) rt[rg * NS + col] = g[2];
      bc = bn;
    }
    c.sync();
    // ---------------- forward: z_0 = 0
    dbl4 zu = z4;
    struct FR { double mp[2], p[2], ka[2], fa[3], rt[3], lc[9], ta[2], qa[2]; };
    auto ld_f = [&](int i, FR& R) {
      const gd* slot = LDa + (int64_t)i * nb2;
      const gd* fs = Fa + (int64_t)i * nb2;
      const bool last = i >= N - 1;
      for (int sgm = 0; sgm < 2; ++sgm) {
        const int row = rg + 4 * sgm, k = rg + 4 * sgm;
        R.mp[sgm] = rlx ? -p_at(slot, sgm) : 0.0;
        R.p[sgm] = (rlx && cw && row < nz) ? (double)fs[PO + row * NS + col] : 0.0;
        R.ka[sgm] = (!last && col >= V0 && col < V0 + nv && k < nz) ? (double)slot[64 + (col - V0) * 8 + k] : 0.0;
        R.ta[sgm] = rlx ? t_at(fs, sgm, 0) : 0.0;
        R.qa[sgm] = rlx ? t_at(fs, sgm, 1) : 0.0;
      }
      for (int sgm = 0; sgm < 3; ++sgm) R.fa[sgm] = last ? 0.0 : f_get(fA[sgm], slot);
      for (int a = 0; a < 3; ++a) R.rt[a] = (!last && cw && a < nv) ? (double)fs[RO + a * NS + col] : 0.0;
      for (int k = 0; k < 9; ++k) R.lc[k] = last ? 0.0 : (double)slot[88 + k];
    };
    FR fc, fn;
    ld_f(0, fc);
    for (int i = 0; i < N; ++i) {
      if (i < N - 1) ld_f(i + 1, fn);
      if (rlx) {                                     // z = zh + T r_x,  r = p - P zh
        dbl4 y = {fc.p[0], fc.p[1], 0.0, 0.0};
        y = Ctx::mfma16(fc.mp[0], zu[0], y);
        y = Ctx::mfma16(fc.mp[1], zu[1], y);
        dbl4 t = Ctx::mfma16(fc.ta[0], y[0], z4);
        t = Ctx::mfma16(fc.ta[1], y[1], t);
        zu[0] += t[0];
        zu[1] += t[1];
      }
      if (i < N - 1) {
        double kv[3] = {fc.rt[0], fc.rt[1], fc.rt[2]};
        chol3_solve(fc.lc, nv, kv);
        dbl4 u = {zu[0], zu[1], (cw && rg < nv) ? kv[rg] : 0.0, 0.0};
        u = Ctx::mfma16(fc.ka[0], zu[0], u);
        u = Ctx::mfma16(fc.ka[1], zu[1], u);
        dbl4 zn = z4;                                // z_{i+1} = F u (e = 0)
        zn = Ctx::mfma16(fc.fa[0], u[0], zn);
        zn = Ctx::mfma16(fc.fa[1], u[1], zn);
        zn = Ctx::mfma16(fc.fa[2], u[2], zn);
        zu = zn;
      }
      fc = fn;
    }
    for (int r = 0; r < 2; ++r) {                    // x_{N-1}: rows 0..4 of z, columns 0..4
      const int row = rg + 4 * r;
      if (cw && row < NS) sig[row * NS + col] = zu[r];
    }
    c.sync();
  }

  // V (block order [y|x|u|tau]) -> X (same order), the two passes on the matrix core.
  // Stage data reach the passes through an LDS ring of RING_SB + 1 stage records (the LD slot's
  // P | K | chol(Rt) | J | 1/sc prefix, V_i, X_i): one cooperative, coalesced global -> LDS copy
  // per block of RING_SB stages, so a block pays one memory latency instead of one per stage;
  // the MFMA operands of stage i are then gathered from LDS one stage ahead (values unchanged:
  // bit-identical to gathering them from HBM).
  // stages [lo, lo + cnt) of LD / V / X into the ring (cnt <= RING_SB + 1); stages >= N skipped
  HTP_HD HTP_FI void ring_fill(ld* ring, int lo, int cnt, const gd* V, const gd* X, const RingSrc* hs = nullptr) {
    const int N = hs ? hs->N : D.N, nb = hs ? hs->nb : D.nb;
    const int64_t nb2 = (int64_t)nb * nb;
    const int lane_ = hs ? hs->lane : (int)c.lane;
    const bool relax_ = hs ? hs->relax : ric_relax;
    const gd* LDs = hs ? hs->LD : A(L.LD);
    const gd* FAs = hs ? hs->fac : A(L.fac);
#if HTP_RING_FILL_LANE
    // Lane l copies elements k = l + 64 j (j < 4) of every stage record; where element k comes from (LD slot,
    // V_i, X_i or the T / Q records in fac) does not depend on the stage, so the four sources are resolved once
    // and each load is base + stage * stride.  Same values as the element-major copy below.
    constexpr int J = (RS_L + 63) / 64;
    const gd* src[J];
    int64_t strd[J];
    bool ok[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int k = lane_ + 64 * j;
      if (k < RS_SLOT) { src[j] = LDs + k; strd[j] = nb2; ok[j] = true; }
      else if (k < RS_X) { src[j] = V + (k - RS_V); strd[j] = nb; ok[j] = k - RS_V < nb; }
      else if (k < RS_T) { src[j] = X + (k - RS_X); strd[j] = nb; ok[j] = k - RS_X < nb; }
      else { src[j] = FAs + (k < RS_L ? k - RS_T : 0); strd[j] = nb2; ok[j] = k < RS_L && relax_; }
    }
    double v[RING_SB + 1][J];
#pragma unroll
    for (int sb = 0; sb <= RING_SB; ++sb) {               // every load of the block issues first
      const int st = lo + sb;
      const bool in = sb < cnt && st < N;
      const int64_t stc = in ? st : 0;
#pragma unroll
      for (int j = 0; j < J; ++j) v[sb][j] = (in && ok[j]) ? (double)src[j][stc * strd[j]] : 0.0;
    }
#pragma unroll
    for (int sb = 0; sb <= RING_SB; ++sb)
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int k = lane_ + 64 * j;
        if (sb < cnt && k < RS_L) ring[sb * RS_L + k] = v[sb][j];
      }
#else
    const gd* LDa = A(L.LD);
    const gd* Fa = A(L.fac);
    const int tot = cnt * RS_L;
    constexpr int U = ((RING_SB + 1) * RS_L + 63) / 64;
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {                       // every load of the block issues first
      const int e = c.lane + u * c.width, sidx = e / RS_L, k = e - sidx * RS_L, st = lo + sidx;
      const bool ok = e < tot && st < N;
      const int stc = ok ? st : 0;
      const gd* src = k < RS_SLOT ? LDa + (int64_t)stc * nb2 + k
                    : (k < RS_X ? V + (int64_t)stc * nb + (k - RS_V)
                                : (k < RS_T ? X + (int64_t)stc * nb + (k - RS_X) : Fa + (int64_t)stc * nb2 + (k - RS_T)));
      const bool in_blk = k < RS_SLOT || (k < RS_X ? k - RS_V < nb : (k < RS_T ? k - RS_X < nb : ric_relax));
      v[u] = (ok && in_blk) ? *src : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = c.lane + u * c.width;
      if (e < tot) ring[e] = v[u];
    }
#endif
  }

  HTP_HD HTP_FI void riccati_solve_mfma(const gd* V, gd* X, bool skip_bwd = false) {
    if constexpr (PT) riccati_solve_mfma_t<2>(V, X);
    else if (D.nw == NS + 3) riccati_solve_mfma_t<3>(V, X, skip_bwd);
    else riccati_solve_mfma_t<2>(V, X, skip_bwd);
  }
  // skip_bwd: the backward pass already ran inside the factorization (HTP_BWD_FUSE); X holds p_i, rt_i
  template <int NV>
  HTP_HD HTP_FI void riccati_solve_mfma_t(const gd* V, gd* X, bool skip_bwd = false) {
#if defined(HTP_KKT_PROF) && HTP_KKT_PROF == 2
    long long kt_ric = c.clock();
#endif
    constexpr int nv = NV, nz = NS + nv;
    const int N = D.N, nb = D.nb;
    const int col = c.lane & 15, rg = c.lane >> 4;
    const bool c0 = col == 0;
    ld* ring = c.lds + RING_OFF;
    // per-lane record maps: F rows as B / F' as A (2), F as A (3), P as A (2), K' as A (1), K at rows V0.. as A (2)
    FSrc fT[2], fA[3];
    for (int sgm = 0; sgm < 2; ++sgm) fT[sgm] = f_src<NV>(rg + 4 * sgm, col);
    for (int sgm = 0; sgm < 3; ++sgm) fA[sgm] = f_src<NV>(col, rg + 4 * sgm);
    auto p_at = [&](const ld* slot, int sgm) {  // P[col][4 sgm + rg] (P symmetric, 8 x 8 stride 8)
      const int k = rg + 4 * sgm;
      return (col < nz && k < nz) ? (double)slot[col * 8 + k] : 0.0;
    };
    auto f_at = [&](const FSrc& f, const ld* slot) {
      return f.kind == 3 ? (double)slot[f.off] : (f.kind == 4 ? 1.0 : 0.0);
    };
    int lo = 0;                                       // first stage held by the ring
    auto rs = [&](int i) -> const ld* { return ring + (i - lo) * RS_L; };
    // ---------------- backward
    // p_{N-1} = [q_{N-1}; 0]
    dbl4 pv = {0.0, 0.0, 0.0, 0.0};
    for (int r = 0; r < 2; ++r) {
      const int row = rg + 4 * r;
      pv[r] = (c0 && row < NS) ? V[(int64_t)(N - 1) * nb + NS + row] : 0.0;
    }
    if (!skip_bwd) {
      gd* Xl = X + (int64_t)(N - 1) * nb;
      for (int r = 0; r < 2; ++r) {
        const int row = rg + 4 * r;
        if (c0 && row < 8) Xl[row] = pv[r];
      }
    }
    // stage-i record of the backward pass: -P_{i+1} (A, 2), F_i' (A, 2), K_i' (A, 1), [q_i; r_i] (C, 3),
    // e_{i+1} (B, 2, unscaled)
    // T_i as the A operand of T r_x: lane supplies T[col][4 sgm + rg] (zero outside 5 x 5)
    auto t_at = [&](const ld* slot, int sgm, int which) {   // which 0: T, 1: Q
      const int k = rg + 4 * sgm;
      return (col < NS && k < NS) ? (double)slot[RS_T + which * NS * NS + col * NS + k] : 0.0;
    };
    const bool rlx = ric_relax;
    const dbl4 z4 = {0.0, 0.0, 0.0, 0.0};
    const RingSrc hsrc = ring_src();
    (void)hsrc;
    struct BRec { double mp[2], ft[2], kt, qr[3], e[2], ta[2], qa[2]; };
    auto ld_b = [&](int i, BRec& R) {
      const ld* slot = rs(i);
      const ld* nslot = slot + RS_L;
      for (int sgm = 0; sgm < 2; ++sgm) {
        R.mp[sgm] = -p_at(nslot, sgm);
        R.ft[sgm] = f_at(fT[sgm], slot);
        const int row = rg + 4 * sgm;
        R.e[sgm] = (c0 && row < NS) ? nslot[RS_V + row] * nslot[SOFF + row] : 0.0;
        R.ta[sgm] = rlx ? t_at(nslot, sgm, 0) : 0.0;
        R.qa[sgm] = rlx ? t_at(nslot, sgm, 1) : 0.0;
      }
      R.kt = (rg < nv && col < nz) ? (double)slot[64 + rg * 8 + col] : 0.0;
      for (int r = 0; r < 3; ++r) {
        const int row = rg + 4 * r;
        double v = 0.0;
        if (c0 && row < NS) v = slot[RS_V + NS + row];
        else if (c0 && row >= V0 && row < V0 + nv) v = slot[RS_V + NS + NS + (row - V0)];
        R.qr[r] = v;
      }
    };
    BRec bc, bn;
    for (int hi = skip_bwd ? -1 : N - 2; hi >= 0; hi -= RING_SB) {
      lo = hi - RING_SB + 1 > 0 ? hi - RING_SB + 1 : 0;
      c.sync();                                       // the previous block's LDS reads are done
      HTP_SPROF0();
      ring_fill(ring, lo, hi - lo + 2, V, X, HTP_HOIST ? &hsrc : nullptr);         // stages lo .. hi + 1
      c.sync();
      ld_b(hi, bc);
      HTP_SPROF(0);
      for (int i = hi; i >= lo; --i) {
        if (i > lo) ld_b(i - 1, bn);
        dbl4 w = Ctx::mfma16(bc.mp[0], bc.e[0], pv);          // w = p - P e
        w = Ctx::mfma16(bc.mp[1], bc.e[1], w);
        if (rlx) {                              // w_x = Q w_x, w_c -= P[c,x] T w_x (relax_P)
          dbl4 t = Ctx::mfma16(bc.ta[0], w[0], z4);
          t = Ctx::mfma16(bc.ta[1], w[1], t);
          dbl4 q = Ctx::mfma16(bc.qa[0], w[0], z4);
          q = Ctx::mfma16(bc.qa[1], w[1], q);
          w = Ctx::mfma16(bc.mp[0], t[0], w);
          w = Ctx::mfma16(bc.mp[1], t[1], w);
          w[0] = q[0];                          // rows 0..3
          if (rg == 0) w[1] = q[1];             // row 4
        }
        dbl4 g = {bc.qr[0], bc.qr[1], bc.qr[2], 0.0};         // g = [q; r] + F' w
        g = Ctx::mfma16(bc.ft[0], w[0], g);
        g = Ctx::mfma16(bc.ft[1], w[1], g);
        pv = Ctx::mfma16(bc.kt, g[2], g);                      // p = g_z + K' rt   (rt = g rows V0..)
        gd* Xi = X + (int64_t)i * nb;
        for (int r = 0; r < 2; ++r) {
          const int row = rg + 4 * r;
          if (c0 && row < nz) Xi[row] = pv[r];
        }
        if (c0 && rg < nv) Xi[nz + rg] = g[2];
        bc = bn;
        HTP_SPROF(1);
      }
    }
    c.sync();
    HTP_PROF(6);
#if defined(HTP_KKT_PROF) && HTP_KKT_PROF == 2
    { const long long t_ = c.clock(); kprof[2] += t_ - kt_ric; kt_ric = t_; }
#endif
    // ---------------- forward: z_0 = [V_0[0:5] / sc; 0]
    const gd* scE = A(L.scE);
    dbl4 zu = {0.0, 0.0, 0.0, 0.0};  // [z_i; v_i] in column 0
    for (int r = 0; r < 2; ++r) {
      const int row = rg + 4 * r;
      zu[r] = (c0 && row < NS) ? V[row] / scE[row] : 0.0;
    }
    // stage-i record of the forward pass: -P_i (A, 2), p_i (C, 2), K_i at rows V0.. (A, 2), F_i (A, 3),
    // e_{i+1} (C, 2), rt_i (3) + chol(Rt_i) (9), 1/sc of y_i (2)
    struct FRec { double mp[2], p[2], ka[2], fa[3], e[2], rt[3], lc[9], isc[2], ta[2], qa[2]; };
    auto ld_f = [&](int i, FRec& R) {
      const ld* slot = rs(i);
      const ld* nslot = slot + RS_L;
      const bool last = i >= N - 1;
      for (int sgm = 0; sgm < 2; ++sgm) {
        const int row = rg + 4 * sgm, k = rg + 4 * sgm;
        R.mp[sgm] = -p_at(slot, sgm);
        R.p[sgm] = (c0 && row < nz) ? (double)slot[RS_X + row] : 0.0;
        R.ka[sgm] = (!last && col >= V0 && col < V0 + nv && k < nz) ? (double)slot[64 + (col - V0) * 8 + k] : 0.0;
        R.e[sgm] = (!last && c0 && row < NS) ? nslot[RS_V + row] * nslot[SOFF + row] : 0.0;
        R.isc[sgm] = (row < NS) ? (double)slot[SOFF + row] : 0.0;
        R.ta[sgm] = rlx ? t_at(slot, sgm, 0) : 0.0;
        R.qa[sgm] = rlx ? t_at(slot, sgm, 1) : 0.0;
      }
      for (int sgm = 0; sgm < 3; ++sgm) R.fa[sgm] = last ? 0.0 : f_at(fA[sgm], slot);
      for (int a = 0; a < 3; ++a) R.rt[a] = (!last && a < nv) ? (double)slot[RS_X + nz + a] : 0.0;
#if !HTP_KV_HOIST
      for (int k = 0; k < 9; ++k) R.lc[k] = last ? 0.0 : (double)slot[88 + k];
#endif
    };
    FRec fc, fn;
    for (lo = 0; lo < N; lo += RING_SB) {
      const int hi = lo + RING_SB - 1 < N - 1 ? lo + RING_SB - 1 : N - 1;
      c.sync();
      HTP_SPROF0();
      ring_fill(ring, lo, hi - lo + 2, V, X, HTP_HOIST ? &hsrc : nullptr);   // stages lo .. hi + 1 (X_i: p_i, rt_i)
      c.sync();
#if HTP_KV_HOIST
      // Rt_i^-1 rt_i does not depend on the forward recursion: one lane per stage of the block solves it and
      // leaves it in the stage's rt slot (the same chol3_solve on the same values), off the chain
      if (hsrc.lane <= hi - lo && lo + hsrc.lane < N - 1) {
        ld* sl = ring + hsrc.lane * RS_L;
        double kv[3], lc[9];
        for (int a = 0; a < 3; ++a) kv[a] = a < nv ? (double)sl[RS_X + nz + a] : 0.0;
        for (int k = 0; k < 9; ++k) lc[k] = sl[88 + k];
        chol3_solve(lc, nv, kv);
        for (int a = 0; a < 3; ++a)
          if (a < nv) sl[RS_X + nz + a] = kv[a];
      }
      c.sync();
#endif
      ld_f(lo, fc);
      HTP_SPROF(2);
      for (int i = lo; i <= hi; ++i) {
        if (i < hi) ld_f(i + 1, fn);
        dbl4 y = {fc.p[0], fc.p[1], 0.0, 0.0};                 // y = p - P z
        y = Ctx::mfma16(fc.mp[0], zu[0], y);
        y = Ctx::mfma16(fc.mp[1], zu[1], y);
        if (rlx) {                 // z = zh + T r_x, y = Q r_x (relax_P); zh was the nominal state
          dbl4 t = Ctx::mfma16(fc.ta[0], y[0], z4);
          t = Ctx::mfma16(fc.ta[1], y[1], t);
          dbl4 q = Ctx::mfma16(fc.qa[0], y[0], z4);
          q = Ctx::mfma16(fc.qa[1], y[1], q);
          zu[0] += t[0];
          zu[1] += t[1];
          y[0] = q[0];
          y[1] = q[1];
        }
        gd* Xi = X + (int64_t)i * nb;
        const double zr0 = zu[0], zr1 = zu[1];
        for (int r = 0; r < 2; ++r) {
          const int row = rg + 4 * r;
          if (c0 && row < NS) Xi[row] = y[r] * fc.isc[r];
        }
        if (i < N - 1) {
          double kv[3] = {fc.rt[0], fc.rt[1], fc.rt[2]};
#if !HTP_KV_HOIST
          chol3_solve(fc.lc, nv, kv);
#endif
          dbl4 u = {zu[0], zu[1], (c0 && rg < nv) ? kv[rg] : 0.0, 0.0};  // u = [z; Rt^-1 rt + K z]
          u = Ctx::mfma16(fc.ka[0], zu[0], u);
          u = Ctx::mfma16(fc.ka[1], zu[1], u);
          if (c0 && rg < nv) Xi[NS + NS + rg] = u[2];
          dbl4 zn = {fc.e[0], fc.e[1], 0.0, 0.0};              // z_{i+1} = F u + e
          zn = Ctx::mfma16(fc.fa[0], u[0], zn);
          zn = Ctx::mfma16(fc.fa[1], u[1], zn);
          zn = Ctx::mfma16(fc.fa[2], u[2], zn);
          zu = zn;
        }
        for (int r = 0; r < 2; ++r) {
          const int row = rg + 4 * r;
          if (c0 && row < NS) Xi[NS + row] = r == 0 ? zr0 : zr1;
        }
        fc = fn;
        HTP_SPROF(3);
      }
    }
    c.sync();
    HTP_PROF(7);
#if defined(HTP_KKT_PROF) && HTP_KKT_PROF == 2
    kprof[3] += c.clock() - kt_ric;
#endif
  }
#endif


  // V (block order [y|x|u|tau]) -> X (same order) with the Riccati factor.
  // Each stage's inputs are packed into a fixed 128/192-entry record that the
  // wave loads with one coalesced round trip, one stage ahead of use
  // (double-buffered in LDS), so the sequential passes are LDS-latency bound.
  static constexpr int RB = 128;  // backward record
  // per-stage slot of L.LD (nb*nb >= 144 doubles) on the Riccati path: P [0,64), K [64,88),
  // chol(Rt) [88,97), unscaled dynamics Jacobian J_i [97,137), 1/scaling of the y_i rows [137,142)
  static constexpr int JOFF = 97;
  static constexpr int SOFF = 137;
  static constexpr int RF = 192;  // forward record

  // Record element e of stage i as (source, offset): the source pointer advances
  // affinely with i, so the per-stage gather is one load (two for a scaled V
  // entry) per element with no element-dependent branching.
  enum { RK_ZERO = 0, RK_LDN, RK_LDC, RK_VNS, RK_VC, RK_XC };
  struct RecDesc {
    int kind, off, off2;
    bool next;  // needs stage i + 1 (zero on the last stage)
  };
  HTP_HD HTP_FI RecDesc rec_back_desc(int e) const {
    const int nv = D.nw - NS, nz = NS + nv;
    const RecDesc z{RK_ZERO, 0, 0, false};
    if (e < 40) { const int r = e / 5, t = e % 5; return (r < nz) ? RecDesc{RK_LDN, r * 8 + t, 0, false} : z; }  // P_{i+1}
    if (e < 80) return (((e - 40) % 8) < D.nw) ? RecDesc{RK_LDC, JOFF + (e - 40), 0, false} : z;              // J_i
    if (e < 85) return RecDesc{RK_VNS, e - 80, SOFF + (e - 80), false};                                        // e_{i+1}
    if (e < 90) return RecDesc{RK_VC, NS + (e - 85), 0, false};                                                // q_i
    if (e < 93) return (e - 90 < nv) ? RecDesc{RK_VC, NS + NS + (e - 90), 0, false} : z;                       // r_i
    if (e >= 96 && e < 120) return RecDesc{RK_LDC, 64 + (e - 96), 0, false};                                   // K_i
    return z;
  }
  HTP_HD HTP_FI RecDesc rec_fwd_desc(int e) const {
    const int nv = D.nw - NS, nz = NS + nv;
    const RecDesc z{RK_ZERO, 0, 0, false};
    if (e < 40) return RecDesc{RK_LDC, e, 0, false};                                                  // P_i rows 0..4
    if (e < 48) return (e - 40 < nz) ? RecDesc{RK_XC, e - 40, 0, false} : z;                          // p_i
    if (e < 51) return (e - 48 < nv) ? RecDesc{RK_XC, nz + (e - 48), 0, true} : z;                    // rt_i
    if (e < 60) return RecDesc{RK_LDC, 88 + (e - 51), 0, true};                                      // chol(Rt_i)
    if (e < 84) return RecDesc{RK_LDC, 64 + (e - 60), 0, true};                                      // K_i
    if (e < 124) return (((e - 84) % 8) < D.nw) ? RecDesc{RK_LDC, JOFF + (e - 84), 0, true} : z;     // J_i
    if (e < 129) return RecDesc{RK_VNS, e - 124, SOFF + (e - 124), true};                            // e_{i+1}
    if (e < 134) return RecDesc{RK_LDC, SOFF + (e - 129), 0, false};                                 // 1/sc of y_i
    return z;
  }
  HTP_HD HTP_FI double rec_get(const RecDesc& d, int i, const gd* V, const gd* X) const {
    const int nb = D.nb;
    const int64_t nb2 = (int64_t)nb * nb;
    if (d.kind == RK_ZERO || (d.next && i >= D.N - 1)) return 0.0;
    const gd* LDc = A(L.LD) + (int64_t)i * nb2;
    const gd* src = (d.kind == RK_LDN) ? LDc + nb2
                  : (d.kind == RK_LDC) ? LDc
                  : (d.kind == RK_VNS) ? V + (int64_t)(i + 1) * nb
                  : (d.kind == RK_VC) ? V + (int64_t)i * nb
                                      : X + (int64_t)i * nb;
    double v = src[d.off];
    if (d.kind == RK_VNS) v *= LDc[nb2 + d.off2];
    return v;
  }

  HTP_HD HTP_FI void riccati_solve(const gd* V, gd* X) {
    const int N = D.N, nb = D.nb, nv = D.nw - NS, nz = NS + nv;
    ld* buf0 = c.lds;             // two records (RF each)
    ld* buf1 = c.lds + RF;
    ld* pv = c.lds + 2 * RF;      // p (8)
    ld* wv = pv + 8;              // w (8)
    ld* rt = pv + 16;             // rt (3)
    ld* zv = pv + 24;             // z (8)
    ld* vv = pv + 32;             // v (3)
    ld* yv = pv + 40;             // y (5)
    constexpr int PB = (RF + Ctx::width - 1) / Ctx::width;
    RecDesc db[PB], dfw[PB];
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      db[u] = rec_back_desc(c.lane + u * c.width);
      dfw[u] = rec_fwd_desc(c.lane + u * c.width);
    }
    // ---------------- backward: p_{N-1} = [q_{N-1}; 0]
    for (int k = c.lane; k < 8; k += c.width) {
      const double val = (k < NS) ? V[(int64_t)(N - 1) * nb + NS + k] : 0.0;
      pv[k] = val;
      X[(int64_t)(N - 1) * nb + k] = val;
    }
    if (N >= 2)
      for (int u = 0; u < PB; ++u)
        if (c.lane + u * c.width < RB) buf0[c.lane + u * c.width] = rec_get(db[u], N - 2, V, X);
    // records are gathered two stages ahead of use: the one of stage i-1 (preA) was issued
    // during stage i+1, so a full stage of latency is hidden behind this one's work
    // (backward records read only LD and V, which the pass does not write)
    double preA[PB];
    for (int u = 0; u < PB; ++u) {
      const int e = c.lane + u * c.width;
      preA[u] = (N >= 3 && e < RB) ? rec_get(db[u], N - 3, V, X) : 0.0;
    }
    c.sync();
    HTP_PROF0();
    for (int i = N - 2; i >= 0; --i) {
      ld* cur = ((N - 2 - i) & 1) ? buf1 : buf0;
      ld* nxt = ((N - 2 - i) & 1) ? buf0 : buf1;
      double pre[PB];
      for (int u = 0; u < PB; ++u) {
        const int e = c.lane + u * c.width;
        pre[u] = (i > 1 && e < RB) ? rec_get(db[u], i - 2, V, X) : 0.0;
      }
      for (int r = c.lane; r < nz; r += c.width) {  // w = p - P e
        double acc = pv[r];
        for (int t = 0; t < NS; ++t) acc -= cur[r * 5 + t] * cur[80 + t];
        wv[r] = acc;
      }
      c.sync();
      if (ric_relax) {  // w_x = Q_{i+1} w_x, w_c -= P[c,x] T_{i+1} w_x  (relax_P)
        const gd* T = trec(i + 1);
        constexpr int PN1 = (8 + Ctx::width - 1) / Ctx::width;
        double wn[PN1];
        int u = 0;
        for (int r = c.lane; r < nz; r += c.width, ++u) {
          double acc = r < NS ? 0.0 : wv[r];
          for (int b = 0; b < NS; ++b) {
            if (r < NS) acc += T[NS * NS + r * NS + b] * wv[b];
            else {
              double tb = 0.0;
              for (int k = 0; k < NS; ++k) tb += T[b * NS + k] * wv[k];
              acc -= cur[r * 5 + b] * tb;
            }
          }
          wn[u] = acc;
        }
        c.sync();
        u = 0;
        for (int r = c.lane; r < nz; r += c.width, ++u) wv[r] = wn[u];
        c.sync();
      }
      for (int a2 = c.lane; a2 < nv; a2 += c.width) {  // rt = r + Jv' w + w_v
        double acc = cur[90 + a2] + wv[NS + a2];
        for (int t = 0; t < NS; ++t) acc += cur[40 + t * 8 + NS + a2] * wv[t];
        rt[a2] = acc;
      }
      c.sync();
      gd* Xi = X + (int64_t)i * nb;
      constexpr int PN = (8 + Ctx::width - 1) / Ctx::width;
      double pnew[PN];
      {
        int u = 0;
        for (int r = c.lane; r < nz; r += c.width, ++u) {  // p = q + Jx' w + K' rt
          double acc = (r < NS) ? cur[85 + r] : 0.0;
          if (r < NS)
            for (int t = 0; t < NS; ++t) acc += cur[40 + t * 8 + r] * wv[t];
          for (int a2 = 0; a2 < nv; ++a2) acc += cur[96 + a2 * 8 + r] * rt[a2];
          pnew[u] = acc;
          Xi[r] = acc;
        }
      }
      for (int a2 = c.lane; a2 < nv; a2 += c.width) Xi[nz + a2] = rt[a2];
      c.sync();
      {
        int u = 0;
        for (int r = c.lane; r < nz; r += c.width, ++u) pv[r] = pnew[u];
      }
      if (i > 0)
        for (int u = 0; u < PB; ++u) {
          const int e = c.lane + u * c.width;
          if (e < RB) nxt[e] = preA[u];
        }
      for (int u = 0; u < PB; ++u) preA[u] = pre[u];
      c.sync();
    }
    HTP_PROF(6);
    // ---------------- forward: z_0 = [x_0; 0]; v = Rt^-1 rt + K z; y = (p - P z)[0:5]
    {
      const gd* scE = A(L.scE);
      for (int k = c.lane; k < 8; k += c.width) zv[k] = (k < NS) ? V[k] / scE[k] : 0.0;
    }
    for (int u = 0; u < PB; ++u)
      if (c.lane + u * c.width < RF) buf0[c.lane + u * c.width] = rec_get(dfw[u], 0, V, X);
    // two stages ahead, as in the backward pass: the record of stage i+2 reads X_{i+2}
    // (p, rt of the backward pass), which this pass overwrites only at stage i+2
    double preF[PB];
    for (int u = 0; u < PB; ++u) {
      const int e = c.lane + u * c.width;
      preF[u] = (1 < N && e < RF) ? rec_get(dfw[u], 1, V, X) : 0.0;
    }
    c.sync();
    for (int i = 0; i < N; ++i) {
      ld* cur = (i & 1) ? buf1 : buf0;
      ld* nxt = (i & 1) ? buf0 : buf1;
      double pre[PB];
      for (int u = 0; u < PB; ++u) {
        const int e = c.lane + u * c.width;
        pre[u] = (i + 2 < N && e < RF) ? rec_get(dfw[u], i + 2, V, X) : 0.0;
      }
      if (ric_relax) {  // x_i = xh_i + T_i r_x, yh_i = Q_i r_x  with r = p - P zh (relax_P)
        const gd* T = trec(i);
        double rr[NS], tx[NS], qx[NS];
        for (int k = 0; k < NS; ++k) {
          double acc = cur[40 + k];
          for (int t = 0; t < nz; ++t) acc -= cur[k * 8 + t] * zv[t];
          rr[k] = acc;
        }
        for (int a = 0; a < NS; ++a) {
          double at = 0.0, aq = 0.0;
          for (int b = 0; b < NS; ++b) {
            at += T[a * NS + b] * rr[b];
            aq += T[NS * NS + a * NS + b] * rr[b];
          }
          tx[a] = at;
          qx[a] = aq;
        }
        c.sync();
        for (int k = c.lane; k < NS; k += c.width) {
          yv[k] = qx[k] * cur[129 + k];
          zv[k] += tx[k];
        }
        c.sync();
      } else {
        for (int k = c.lane; k < NS; k += c.width) {
          double acc = cur[40 + k];
          for (int t = 0; t < nz; ++t) acc -= cur[k * 8 + t] * zv[t];
          yv[k] = acc * cur[129 + k];
        }
      }
      if (i < N - 1) {
        double kv[3] = {cur[48], cur[49], cur[50]};
        double Lc[9];
        for (int e = 0; e < 9; ++e) Lc[e] = cur[51 + e];
        chol3_solve(Lc, nv, kv);
        for (int a2 = c.lane; a2 < nv; a2 += c.width) {
          double acc = kv[a2];
          for (int t = 0; t < nz; ++t) acc += cur[60 + a2 * 8 + t] * zv[t];
          vv[a2] = acc;
        }
      }
      c.sync();
      gd* Xi = X + (int64_t)i * nb;
      constexpr int PN = (8 + Ctx::width - 1) / Ctx::width;
      double zn[PN];
      int un = 0;
      if (i < N - 1)
        for (int k = c.lane; k < nz; k += c.width, ++un) {
          double acc;
          if (k < NS) {
            acc = cur[124 + k];
            for (int t = 0; t < NS; ++t) acc += cur[84 + k * 8 + t] * zv[t];
            for (int a2 = 0; a2 < nv; ++a2) acc += cur[84 + k * 8 + NS + a2] * vv[a2];
          } else {
            acc = vv[k - NS];
          }
          zn[un] = acc;
        }
      for (int k = c.lane; k < NS; k += c.width) {
        Xi[k] = yv[k];
        Xi[NS + k] = zv[k];
      }
      if (i < N - 1)
        for (int a2 = c.lane; a2 < nv; a2 += c.width) Xi[NS + NS + a2] = vv[a2];
      c.sync();
      if (i < N - 1) {
        un = 0;
        for (int k = c.lane; k < nz; k += c.width, ++un) zv[k] = zn[un];
        for (int u = 0; u < PB; ++u) {
          const int e = c.lane + u * c.width;
          if (e < RF) nxt[e] = preF[u];
        }
      }
      for (int u = 0; u < PB; ++u) preF[u] = pre[u];
      c.sync();
    }
    HTP_PROF(7);
  }

  // ---------------------------------------------- point formulation: hard terminal rows
  // optimizer_points.py:273-278 adds X_{N-1} = end as equality rows (stage-chain block N):
  //   K Z + C' y_T = r_Z,  C Z - E_T y_T = r_T,   C Z = s_T o x_{N-1},  E_T = dc (+ e_R in restoration).
  // With K the stage chain (Riccati), the terminal multipliers solve the 5 x 5 system
  //   (S_T Sig S_T + E_T) y_T = s_T o (K^-1 r_Z)_x - r_T,   Sig = K^-1 [x_{N-1}, x_{N-1}],
  // then Z = K^-1 (r_Z - C' y_T).  Inertia (Sylvester, Schur on y_T): the 5 terminal negatives iff
  // S_T Sig S_T + E_T is positive definite.  Sig = five solves with unit right-hand sides at x_{N-1}.
  HTP_HD HTP_FI void ric_solve(const gd* V, gd* X, bool skip_bwd = false) {
#if defined(__HIPCC__) || defined(HTP_EMU_WAVE)
    if constexpr (Ctx::kMfma) { riccati_solve_mfma(V, X, skip_bwd); return; }
#endif
    riccati_solve(V, X);
  }
  // chol(S_T Sig S_T + E_T) (15, reciprocal pivots) and s_T (5) into fac slot N; false if not pos. def.
  HTP_HD HTP_FI bool terminal_schur(double dc) {
    const int N = D.N, nb = D.nb;
    gd* V = A(L.V);
    gd* X = A(L.X);
    gd* rec = A(L.fac) + (int64_t)N * nb * nb;
    const gd* scE = A(L.scE);
    const gd* eR = A(L.eR);
#if defined(__HIPCC__) || defined(HTP_EMU_WAVE)
    if constexpr (Ctx::kMfma) {
      riccati_sigma_mfma(rec + 20);       // all five columns in one pair of passes
    } else
#endif
    {
      for (int k = 0; k < NS; ++k) {
        for (int e = c.lane; e < N * nb; e += c.width) V[e] = (e == (N - 1) * nb + NS + k) ? 1.0 : 0.0;
        c.sync();
        ric_solve(V, X);
        c.sync();
        for (int j = c.lane; j < NS; j += c.width) rec[20 + k * NS + j] = X[(int64_t)(N - 1) * nb + NS + j];
        c.sync();
      }
    }
    double Sm[NS * NS], Lc[15], sT[NS];
    for (int k = 0; k < NS; ++k) sT[k] = scE[D.eTerm + k];
    for (int a = 0; a < NS; ++a)
      for (int b = 0; b < NS; ++b) {
        const double sig = 0.5 * (rec[20 + a * NS + b] + rec[20 + b * NS + a]);
        Sm[a * NS + b] = sT[a] * sig * sT[b] + (a == b ? dc + (rs ? eR[D.eTerm + a] : 0.0) : 0.0);
      }
    const bool ok = chol5(Sm, Lc);
    c.sync();
    for (int e = c.lane; e < 20; e += c.width) rec[e] = e < 15 ? Lc[e] : sT[e - 15];
    c.sync();
    return ok;
  }
  // the stage-chain solve with the terminal rows: V (blocks 0..N-1, block N = r_T) -> X (block N = y_T)
  HTP_HD HTP_FI void ric_solve_terminal(gd* V, gd* X) {
    const int N = D.N, nb = D.nb;
    const gd* rec = A(L.fac) + (int64_t)N * nb * nb;
    ric_solve(V, X);
    c.sync();
    double Lc[15], sT[NS], y[NS];
    for (int e = 0; e < 15; ++e) Lc[e] = rec[e];
    for (int k = 0; k < NS; ++k) {
      sT[k] = rec[15 + k];
      y[k] = sT[k] * X[(int64_t)(N - 1) * nb + NS + k] - V[(int64_t)N * nb + k];
    }
    chol5_fwd(Lc, y);
    chol5_bwd(Lc, y);
    c.sync();
    for (int k = c.lane; k < NS; k += c.width) {
      V[(int64_t)(N - 1) * nb + NS + k] -= sT[k] * y[k];
      X[(int64_t)N * nb + k] = y[k];
    }
    c.sync();
    ric_solve(V, X);
    c.sync();
  }

  // ---------------------------------------------------------- factorization
  // returns true if the inertia is the one IPOPT requires
  HTP_HD HTP_PHASE void factorize(bool ls, double dw, double dc, int& neg_out, int& zero_out) {
    const int N = D.N, nb = D.nb;
    int neg = 0, zero = 0;
    long long t0 = c.clock();
    bwd_ready = false;
    if (rs) compute_eR(ls, dw);
    local_factor_sweep<EN_, EM_>(ls, dw, dc, neg, zero);
    neg = c.isum(neg);
    zero = c.isum(zero);
    c.sync();
    long long t1 = c.clock();
    cyc[0] += t1 - t0;
    // Inertia bookkeeping.  Each eliminated block is a saddle-point matrix
    // [H, C'; C, -dc I] whose constraint rows C have full row rank, so it has
    // at least as many negative eigenvalues as rows (Sylvester on the Schur
    // complement).  Every local block therefore contributes >= 2 negatives
    // and the stage system >= 5N: the total equals IPOPT's required count iff
    // the local blocks hold exactly 2P and the stage system exactly 5N.
    // Extra local negatives => wrong inertia, decided without the stage
    // factorization.  With exact dynamics (dc == 0) the stage count is 5N iff
    // every Riccati pivot Rt is positive definite; dc > 0 takes the block
    // Bunch-Kaufman path below.
    // (A zero local pivot only needs reporting: IPOPT's reaction -- dc, then
    // dw -- does not depend on the stage system.)
    if (zero > 0 || neg != (PT ? 0 : 2 * D.P)) {
      use_ric = false;
      neg_out = -1;
      zero_out = zero;
      return;
    }
    for (int i = c.lane; i < N; i += c.width) assemble_stage(i, ls, dw, dc);
    if constexpr (PT) assemble_term_pt(dc);
    c.sync();
    long long t2 = c.clock();
    cyc[1] += t2 - t1;
    // delta_c > 0 and the restoration phase relax the dynamics rows: the same recursion through
    // relax_P.  The point formulation's hard terminal rows (block N) enter through their 5 x 5 Schur
    // complement (terminal_schur).
    if ((!PT || HTP_PT_RICCATI) && (HTP_RELAX_RICCATI || (dc == 0.0 && !rs))) {
      int bad;
      ric_relax = dc != 0.0 || rs;
#if defined(__HIPCC__) || defined(HTP_EMU_WAVE)
      if constexpr (Ctx::kMfma) {
#if HTP_BWD_FUSE
        // the Newton step's rhs is known here (fused local sweep: pairR is this trial's): build V and run the
        // solve's backward pass with the factor
        const bool fb = fuse_rhs && !PT && !ric_relax && !ls;
        if (fb) { build_stage_rhs(ls, dw, dc, A(L.xt), A(L.rc)); c.sync(); }
        bad = riccati_factor_mfma(dc, fb);
        bwd_ready = fb && !bad;
#else
        bad = riccati_factor_mfma(dc);
#endif
      }
      else
#endif
        bad = riccati_factor(dc);
      use_ric = true;
      bool done = true;
      if constexpr (PT) {
        // Riccati pivots and the terminal Schur complement all positive definite => exact inertia.
        // Otherwise the chain without its terminal rows may still be indefinite on directions the
        // terminal rows remove: the block LDL^T below decides (the reference's exact inertia).
        if (!bad && !terminal_schur(dc)) bad = 1;
        done = bad == 0;
      }
      if (done) {
        cyc[2] += c.clock() - t2;
        neg_out = bad ? -1 : neg + NS * N + NS + D.md;
        zero_out = zero;
        return;
      }
    }
    use_ric = false;
    // sequential block LDL^T over stages, in LDS:
    //   D_i = K_ii - Off_i Dinv_{i-1} Off_i',  LD_i = Off_i Dinv_{i-1},
    //   Dinv_i = D_i^{-1} from a Bunch-Kaufman factor (inertia of D_i).
    ld* Acur = c.lds;                   // nb x nb
    ld* Dinv = c.lds + NBMAX * NBMAX;   // nb x nb (previous stage inverse)
    ld* Obuf = c.lds + 2 * NBMAX * NBMAX;
    ld* Tmp = c.lds + 3 * NBMAX * NBMAX;
    li* ipc = c.ildsp;
    int sneg = 0, szero = 0;
    const int nb2 = nb * nb;
    for (int i = 0; i < D.nblk; ++i) {
      const gd* K = A(L.Kst) + (int64_t)i * nb2;
      for (int e = c.lane; e < nb2; e += c.width) Acur[e] = K[e];
      if (i > 0) {
        const gd* O = A(L.Off) + (int64_t)i * nb2;
        for (int e = c.lane; e < nb2; e += c.width) Obuf[e] = O[e];
      }
      c.sync();
      if (i > 0) {
        gd* LD = A(L.LD) + (int64_t)i * nb2;
        for (int e = c.lane; e < nb2; e += c.width) {  // Tmp = LD = Off Dinv
          const int r = e / nb, q = e % nb;
          double acc = 0.0;
          for (int t = 0; t < nb; ++t) acc += Obuf[r * nb + t] * Dinv[t * nb + q];
          Tmp[e] = acc;
          LD[e] = acc;
        }
        c.sync();
        for (int e = c.lane; e < nb2; e += c.width) {  // Acur -= LD Off'
          const int r = e / nb, q = e % nb;
          double acc = 0.0;
          for (int t = 0; t < nb; ++t) acc += Tmp[r * nb + t] * Obuf[q * nb + t];
          Acur[e] -= acc;
        }
        c.sync();
      }
      bk_factor(Acur, ipc, nb, sneg, szero);
      bk_inverse(Acur, ipc, nb, Dinv);
      gd* F = A(L.fac) + (int64_t)i * nb2;
      for (int e = c.lane; e < nb2; e += c.width) F[e] = Dinv[e];
      c.sync();
    }
    cyc[2] += c.clock() - t2;
    // terminal block contributes 5 negatives; inequality multipliers md negatives
#ifdef HTP_HOST_DEBUG
    printf("[dbg]   pairs neg=%d (exp %d) zero=%d stages neg=%d (exp %d) zero=%d\n", neg, 2 * D.P, zero, sneg, NS * N, szero);
#endif
    neg_out = neg + sneg + (PT ? 0 : NS) + D.md;
    zero_out = zero + szero;
  }

  // solve K [ox; os; oc; od] = [bx; bs; bc; bd] with the current factorization
  // Restoration phase: the n/p rows (S_n + dw) dn + dy = b_n, (S_p + dw) dp - dy = b_p are eliminated onto the
  // constraint rows (eR = 1/(S_n+dw) + 1/(S_p+dw) on the diagonal), b_c -> b_c - b_n/(S_n+dw) + b_p/(S_p+dw).
  HTP_HD HTP_FI void np_diag(int j, bool ls, double dw, double& sn, double& sp) const {
    const gd* R = A(L.R); const gd* zR = A(L.zR);
    const int jp = j < D.mc ? j + D.mc : j + D.md;   // n index j -> its p index
    sn = ls ? 1.0 : zR[j] / R[j] + dw;
    sp = ls ? 1.0 : zR[jp] / R[jp] + dw;
  }
  HTP_HD HTP_FI void compute_eR(bool ls, double dw) {
    gd* eR = A(L.eR);
    double sn_[SW_U], sp_[SW_U];
    sweep(D.mc + D.md, [&](int r, int k) { np_diag(r < D.mc ? r : r + D.mc, ls, dw, sn_[k], sp_[k]); },  // n index of row r
          [&](int r, int k) { eR[r] = 1.0 / sn_[k] + 1.0 / sp_[k]; });
    c.sync();
  }

  // stage right-hand side V (block order [y|x|u|tau]) of the KKT system from bx, bc and the local blocks' stage
  // contributions (pairR); each stage's rhs is built in registers and stored once
  HTP_HD HTP_FI void build_stage_rhs(bool ls, double dw, double dc, const gd* bx, const gd* bc) {
    const int N = D.N, nb = D.nb;
    const gd* PR = A(L.pairR);
    const gd* scE = A(L.scE);
    gd* V = A(L.V);
    const int MK = blocks_per_stage();
    for (int i = c.lane; i < N; i += c.width) {
      gd* r = V + (int64_t)i * nb;
      const int rowbase = (i == 0) ? 0 : D.eDyn + NS * (i - 1);
      double rv[NBMAX];
      for (int k = 0; k < NS; ++k) rv[k] = bc[rowbase + k];
      for (int k = 0; k < NS; ++k) rv[NS + k] = bx[NS * i + k];
      for (int a = NS; a < NBMAX - NS; ++a) rv[NS + a] = 0.0;
      if (i < N - 1) {
        rv[NS + 5] = bx[D.oU + NC * i];
        rv[NS + 6] = bx[D.oU + NC * i + 1];
        if (D.topt) rv[NS + 7] = bx[D.oTAU + i];
      } else {
        if constexpr (!PT)
          for (int k = 0; k < NS; ++k) {
            const double st = scE[D.eTerm + k];
            const double Hs = term_H(k, ls, dw), Et = term_E(k, ls, dw, dc);
            rv[NS + k] -= st / Et * (st * bx[D.oS + k] / Hs - bc[D.eTerm + k]);
          }
      }
      for (int q = 0; q < MK; ++q) {
        const int p = blk(i, q);
        rv[NS + 0] += PR[3 * p];
        rv[NS + 1] += PR[3 * p + 1];
        rv[NS + 3] += PR[3 * p + 2];
      }
      for (int a = 0; a < NBMAX; ++a)
        if (a < nb) r[a] = rv[a];
    }
  }

  HTP_HD HTP_PHASE void kkt_solve(bool ls, double dw, double dc, const gd* bx, const gd* bs, const gd* bc,
                        const gd* bd, gd* ox, gd* os, gd* oc, gd* od, const gd* bR = nullptr, gd* oR = nullptr,
                        bool rhs_done = false) {
    const int N = D.N, nb = D.nb;
    const long long t0 = c.clock();
    if (rs) {  // fold the n/p right-hand sides into the constraint rows
      gd* fc = A(L.rcf); gd* fd = A(L.rdf);
      double sn_[SW_U], sp_[SW_U], b_[SW_U], bn_[SW_U], bp_[SW_U];
      sweep(D.mc + D.md, [&](int r, int k) {
              const int j = r < D.mc ? r : r + D.mc, jp = r < D.mc ? r + D.mc : r + D.mc + D.md;
              np_diag(j, ls, dw, sn_[k], sp_[k]);
              b_[k] = r < D.mc ? bc[r] : bd[r - D.mc];
              bn_[k] = bR[j];
              bp_[k] = bR[jp];
            },
            [&](int r, int k) {
              const double v = b_[k] - bn_[k] / sn_[k] + bp_[k] / sp_[k];
              if (r < D.mc) fc[r] = v;
              else fd[r - D.mc] = v;
            });
      c.sync();
      bc = fc;
      bd = fd;
    }
#ifdef HTP_KKT_PROF
    long long tk = c.clock();
#endif
    if (!rhs_done) local_rhs_sweep<EN_, EM_>(ls, dw, dc, bx, bs, bc, bd);   // else: pairR from the factor sweep
    c.sync();
    HTP_KPROF(0, tk);
#if defined(HTP_KKT_PROF) && HTP_KKT_PROF == 2
    kprof[6] += 1;
#endif
    const gd* scE = A(L.scE);
    gd* V = A(L.V);
#if HTP_BWD_FUSE
    const bool bwd = rhs_done && bwd_ready;   // V and the backward pass came with the factorization
#else
    const bool bwd = false;
#endif
    bwd_ready = false;
    if (!bwd) build_stage_rhs(ls, dw, dc, bx, bc);
    if constexpr (PT)
      for (int e = c.lane; e < nb; e += c.width) V[(int64_t)N * nb + e] = (e < NS) ? bc[D.eTerm + e] : 0.0;
    c.sync();
#if defined(HTP_KKT_PROF) && HTP_KKT_PROF == 2
    HTP_KPROF(1, tk);
#endif
    gd* X = A(L.X);
    if (use_ric) {
      if constexpr (PT) ric_solve_terminal(V, X);
      else ric_solve(V, X, bwd);
    } else {
    // forward: V_i -= LD_i V_{i-1}
    for (int i = 1; i < D.nblk; ++i) {
      const gd* LD = A(L.LD) + (int64_t)i * nb * nb;
      gd* vi = V + (int64_t)i * nb;
      const gd* vp = V + (int64_t)(i - 1) * nb;
      for (int r = c.lane; r < nb; r += c.width) {
        double acc = 0.0;
        for (int t = 0; t < nb; ++t) acc += LD[r * nb + t] * vp[t];
        vi[r] -= acc;
      }
      c.sync();
    }
    // backward: X_i = Dinv_i (V_i - Off_{i+1}' X_{i+1})
    ld* tv = c.lds + 3 * NBMAX * NBMAX;
    for (int i = D.nblk - 1; i >= 0; --i) {
      gd* xi = X + (int64_t)i * nb;
      const gd* vi = V + (int64_t)i * nb;
      for (int r = c.lane; r < nb; r += c.width) {
        double acc = vi[r];
        if (i < D.nblk - 1) {
          const gd* O = A(L.Off) + (int64_t)(i + 1) * nb * nb;
          const gd* xn = X + (int64_t)(i + 1) * nb;
          for (int t = 0; t < nb; ++t) acc -= O[t * nb + r] * xn[t];
        }
        tv[r] = acc;
      }
      c.sync();
      const gd* F = A(L.fac) + (int64_t)i * nb * nb;
      for (int r = c.lane; r < nb; r += c.width) {
        double acc = 0.0;
        for (int t = 0; t < nb; ++t) acc += F[r * nb + t] * tv[t];
        xi[r] = acc;
      }
      c.sync();
    }
    }
    // scatter stage solution
#if HTP_HOIST
    // every load of the stage before its first store (a load issued after a store waits for it)
    for (int i = c.lane; i < N; i += c.width) {
      const gd* xg = X + (int64_t)i * nb;
      double xi[NBMAX];
      for (int a = 0; a < NBMAX; ++a) xi[a] = xg[a < nb ? a : 0];
      const int rowbase = (i == 0) ? 0 : D.eDyn + NS * (i - 1);
      if (i == N - 1) {
        if constexpr (PT) {
          double xt_[NS];
          for (int k = 0; k < NS; ++k) xt_[k] = X[(int64_t)N * nb + k];
          for (int k = 0; k < NS; ++k) oc[rowbase + k] = xi[k];
          for (int k = 0; k < NS; ++k) ox[NS * i + k] = xi[NS + k];
          for (int k = 0; k < NS; ++k) oc[D.eTerm + k] = xt_[k];
        } else {
          double yt[NS], xs[NS];
          for (int k = 0; k < NS; ++k) {
            const double st = scE[D.eTerm + k];
            const double Hs = term_H(k, ls, dw), Et = term_E(k, ls, dw, dc);
            const double bxs = bx[D.oS + k];
            yt[k] = (st * xi[NS + k] + st * bxs / Hs - bc[D.eTerm + k]) / Et;
            xs[k] = (bxs - st * yt[k]) / Hs;
          }
          for (int k = 0; k < NS; ++k) oc[rowbase + k] = xi[k];
          for (int k = 0; k < NS; ++k) ox[NS * i + k] = xi[NS + k];
          for (int k = 0; k < NS; ++k) {
            oc[D.eTerm + k] = yt[k];
            ox[D.oS + k] = xs[k];
          }
        }
      } else {
        for (int k = 0; k < NS; ++k) oc[rowbase + k] = xi[k];
        for (int k = 0; k < NS; ++k) ox[NS * i + k] = xi[NS + k];
        ox[D.oU + NC * i] = xi[NS + 5];
        ox[D.oU + NC * i + 1] = xi[NS + 6];
        if (D.topt) ox[D.oTAU + i] = xi[NS + 7];
      }
    }
    if (false)
#endif
    for (int i = c.lane; i < N; i += c.width) {
      const gd* xi = X + (int64_t)i * nb;
      const int rowbase = (i == 0) ? 0 : D.eDyn + NS * (i - 1);
      for (int k = 0; k < NS; ++k) oc[rowbase + k] = xi[k];
      for (int k = 0; k < NS; ++k) ox[NS * i + k] = xi[NS + k];
      if (i < N - 1) {
        ox[D.oU + NC * i] = xi[NS + 5];
        ox[D.oU + NC * i + 1] = xi[NS + 6];
        if (D.topt) ox[D.oTAU + i] = xi[NS + 7];
      } else if constexpr (PT) {
        for (int k = 0; k < NS; ++k) oc[D.eTerm + k] = X[(int64_t)N * nb + k];
      } else {
        for (int k = 0; k < NS; ++k) {
          const double st = scE[D.eTerm + k];
          const double Hs = term_H(k, ls, dw), Et = term_E(k, ls, dw, dc);
          const double yt = (st * xi[NS + k] + st * bx[D.oS + k] / Hs - bc[D.eTerm + k]) / Et;
          oc[D.eTerm + k] = yt;
          ox[D.oS + k] = (bx[D.oS + k] - st * yt) / Hs;
        }
      }
    }
    c.sync();
#if defined(HTP_KKT_PROF) && HTP_KKT_PROF == 2
    HTP_KPROF(4, tk);
#else
    HTP_KPROF(1, tk);
#endif
    local_back_sweep<EN_, EM_>(ls, dw, dc, bx, bs, bc, bd, ox, os, oc, od);
    c.sync();
#if defined(HTP_KKT_PROF) && HTP_KKT_PROF == 2
    HTP_KPROF(5, tk);
#else
    HTP_KPROF(2, tk);
#endif
    if (rs) {  // dn = (b_n - dy) / (S_n + dw), dp = (b_p + dy) / (S_p + dw)
      double sn_[SW_U], sp_[SW_U], dy_[SW_U], bn_[SW_U], bp_[SW_U];
      sweep(D.mc + D.md, [&](int r, int k) {
              const int j = r < D.mc ? r : r + D.mc, jp = r < D.mc ? r + D.mc : r + D.mc + D.md;
              np_diag(j, ls, dw, sn_[k], sp_[k]);
              dy_[k] = r < D.mc ? oc[r] : od[r - D.mc];
              bn_[k] = bR[j];
              bp_[k] = bR[jp];
            },
            [&](int r, int k) {
              const int j = r < D.mc ? r : r + D.mc, jp = r < D.mc ? r + D.mc : r + D.mc + D.md;
              oR[j] = (bn_[k] - dy_[k]) / sn_[k];
              oR[jp] = (bp_[k] + dy_[k]) / sp_[k];
            });
      c.sync();
    }
    cyc[3] += c.clock() - t0;
  }
  // ======================================================== IPM driver
  // Mirrors oracle/ipm.py (_Ipm.run, find_trial, backtrack, second_order_correction,
  // try_soft_resto_step, restoration, resto_check, resto_resto) decision by decision.
  int nbL, nbU, nsL, nsU;  // counts of finite bounds

  HTP_HD HTP_FI void count_bounds() {
    const gd* xL = A(L.xL);
    const gd* xU = A(L.xU);
    const gd* dU = A(L.dU);
    int a = 0, b = 0, e = 0;
    HTP_UNROLL
    for (int q = c.lane; q < D.n; q += c.width) {
      a += finite_(xL[q]);
      b += finite_(xU[q]);
    }
    HTP_UNROLL
    for (int r = c.lane; r < D.md; r += c.width) e += finite_(dU[r]);
    nbL = c.isum(a);
    nbU = c.isum(b);
    nsL = D.md;
    nsU = c.isum(e);
  }

  struct Err { double dual, comp, s_d, s_c, prim_b, prim_nlp; };

  // J_R' y entry of restoration variable j (n: +y, p: -y)
  HTP_HD HTP_FI double np_jty(int j, const gd* yc, const gd* yd) const {
    const int mc = D.mc, md = D.md;
    if (j < mc) return yc[j];
    if (j < 2 * mc) return -yc[j - mc];
    if (j < 2 * mc + md) return yd[j - 2 * mc];
    return -yd[j - 2 * mc - md];
  }

  // grad Lagrangian (x part, w/o bound multipliers) at (x, yc, yd) -> out; gf must hold grad f at x
  HTP_HD HTP_FI void grad_lag_at(const gd* x, const gd* yc, const gd* yd, const gd* gf, gd* out) {
    eval_jt(x, yc, yd, out);
    double a_[SW_U], b_[SW_U];
    sweep(D.n, [&](int q, int k) { a_[k] = out[q]; b_[k] = gf[q]; }, [&](int q, int k) { out[q] = a_[k] + b_[k]; });
    c.sync();
  }
  HTP_HD HTP_FI void grad_lag_into(gd* out) { grad_lag_at(A(L.x), A(L.yc), A(L.yd), A(L.gf), out); }

  // e2 (optional): the same errors at a second barrier parameter mu2, from the same sweeps -- iterate() needs the
  // mu = 0 optimality errors and the barrier errors at the current mu of one point; only comp depends on mu
  HTP_HD HTP_PHASE Err errors(const gd* gl, double mu_, double mu2 = 0.0, Err* e2 = nullptr) const {
    const gd* x = A(L.x); const gd* xL = A(L.xL); const gd* xU = A(L.xU);
    const gd* zL = A(L.zL); const gd* zU = A(L.zU);
    const gd* s = A(L.s); const gd* dL = A(L.dL); const gd* dU = A(L.dU);
    const gd* vL = A(L.vL); const gd* vU = A(L.vU);
    const gd* yc = A(L.yc); const gd* yd = A(L.yd);
    const gd* cc = A(L.c); const gd* dd = A(L.d);
    double dual = 0, comp = 0, comp2 = 0, zsum = 0, ysum = 0, pb = 0, pn = 0;
    const bool two = e2 != nullptr;
    {
      double g_[SW_U], zl_[SW_U], zu_[SW_U], x_[SW_U], xl_[SW_U], xu_[SW_U];
      sweep(D.n, [&](int q, int k) { g_[k] = gl[q]; zl_[k] = zL[q]; zu_[k] = ubx(q) ? (double)zU[q] : 0.0; x_[k] = x[q]; xl_[k] = xL[q]; xu_[k] = ubx(q) ? (double)xU[q] : HTP_INF; },
            [&](int, int k) {
              dual = dmax(dual, dabs(g_[k] - zl_[k] + zu_[k]));
              if (finite_(xl_[k])) {
                comp = dmax(comp, dabs((x_[k] - xl_[k]) * zl_[k] - mu_));
                if (two) comp2 = dmax(comp2, dabs((x_[k] - xl_[k]) * zl_[k] - mu2));
                zsum += dabs(zl_[k]);
              }
              if (finite_(xu_[k])) {
                comp = dmax(comp, dabs((xu_[k] - x_[k]) * zu_[k] - mu_));
                if (two) comp2 = dmax(comp2, dabs((xu_[k] - x_[k]) * zu_[k] - mu2));
                zsum += dabs(zu_[k]);
              }
            });
    }
    {
      double yd_[SW_U], vl_[SW_U], vu_[SW_U], s_[SW_U], dl_[SW_U], du_[SW_U], d_[SW_U];
      sweep(D.md, [&](int r, int k) { yd_[k] = yd[r]; vl_[k] = vL[r]; vu_[k] = ubs(r) ? (double)vU[r] : 0.0; s_[k] = s[r]; dl_[k] = dL[r]; du_[k] = ubs(r) ? (double)dU[r] : HTP_INF; d_[k] = dd[r]; },
            [&](int, int k) {
              dual = dmax(dual, dabs(-yd_[k] - vl_[k] + vu_[k]));
              comp = dmax(comp, dabs((s_[k] - dl_[k]) * vl_[k] - mu_));
              if (two) comp2 = dmax(comp2, dabs((s_[k] - dl_[k]) * vl_[k] - mu2));
              zsum += dabs(vl_[k]);
              if (finite_(du_[k])) {
                comp = dmax(comp, dabs((du_[k] - s_[k]) * vu_[k] - mu_));
                if (two) comp2 = dmax(comp2, dabs((du_[k] - s_[k]) * vu_[k] - mu2));
                zsum += dabs(vu_[k]);
              }
              ysum += dabs(yd_[k]);
              pb = dmax(pb, dabs(d_[k] - s_[k]));
              double v = dmax(0.0, dl_[k] - d_[k]);
              if (finite_(du_[k])) v = dmax(v, d_[k] - du_[k]);
              pn = dmax(pn, v);
            });
    }
    {
      double yc_[SW_U], c_[SW_U];
      sweep(D.mc, [&](int r, int k) { yc_[k] = yc[r]; c_[k] = cc[r]; },
            [&](int, int k) {
              ysum += dabs(yc_[k]);
              pb = dmax(pb, dabs(c_[k]));
              pn = dmax(pn, dabs(c_[k]));
            });
    }
    if (rs) {  // n/p: rho + J_R'y - z_R, complementarity R z_R
      const gd* R = A(L.R); const gd* zR = A(L.zR);
      const double rho = o.resto_penalty_parameter;
      double jt_[SW_U], r_[SW_U], z_[SW_U];
      sweep(nR, [&](int j, int k) { jt_[k] = np_jty(j, yc, yd); r_[k] = R[j]; z_[k] = zR[j]; },
            [&](int, int k) {
              dual = dmax(dual, dabs(rho + jt_[k] - z_[k]));
              comp = dmax(comp, dabs(r_[k] * z_[k] - mu_));
              if (two) comp2 = dmax(comp2, dabs(r_[k] * z_[k] - mu2));
              zsum += dabs(z_[k]);
            });
    }
    Err e;
    e.dual = c.maxv(dual);
    e.comp = c.maxv(comp);
    zsum = c.sum(zsum);
    ysum = c.sum(ysum);
    e.prim_b = c.maxv(pb);
    e.prim_nlp = c.maxv(pn);
    const int nz = nbL + nbU + nsL + nsU + (rs ? nR : 0), ny = D.mc + D.md;
    e.s_d = dmax(o.s_max, (ysum + zsum) / (double)(ny + nz > 0 ? ny + nz : 1)) / o.s_max;
    e.s_c = dmax(o.s_max, zsum / (double)(nz > 0 ? nz : 1)) / o.s_max;
    if (two) {
      *e2 = e;
      e2->comp = c.maxv(comp2);
    }
    return e;
  }

  // IPOPT curr_primal_dual_system_error(mu): averaged 1-norms of dual infeasibility, primal
  // infeasibility and relaxed complementarity at the point given by the arrays
  HTP_HD HTP_FI double pd_error(const gd* gl, const gd* x, const gd* s, const gd* yc, const gd* yd, const gd* zL,
                                const gd* zU, const gd* vL, const gd* vU, const gd* R, const gd* zR, const gd* cc,
                                const gd* dd, double mu_, bool safe = false) const {
    const gd* xL = A(L.xL); const gd* xU = A(L.xU); const gd* dL = A(L.dL); const gd* dU = A(L.dU);
    const gd* czL = A(L.zL); const gd* czU = A(L.zU); const gd* cvL = A(L.vL); const gd* cvU = A(L.vU);
    auto sl = [&](double v, double z, double b) { return safe ? safe_slack(v, z, b, mu_) : v; };
    double du = 0, pr = 0, cs = 0;
    int ncs = 0;
    for (int q = c.lane; q < D.n; q += c.width) {
      du += dabs(gl[q] - zL[q] + zU[q]);
      if (finite_(xL[q])) { cs += dabs(sl(x[q] - xL[q], czL[q], xL[q]) * zL[q] - mu_); ++ncs; }
      if (finite_(xU[q])) { cs += dabs(sl(xU[q] - x[q], czU[q], xU[q]) * zU[q] - mu_); ++ncs; }
    }
    for (int r = c.lane; r < D.md; r += c.width) {
      du += dabs(-yd[r] - vL[r] + vU[r]);
      pr += dabs(dd[r] - s[r]);
      cs += dabs(sl(s[r] - dL[r], cvL[r], dL[r]) * vL[r] - mu_);
      ++ncs;
      if (finite_(dU[r])) { cs += dabs(sl(dU[r] - s[r], cvU[r], dU[r]) * vU[r] - mu_); ++ncs; }
    }
    for (int r = c.lane; r < D.mc; r += c.width) pr += dabs(cc[r]);
    if (rs) {
      const double rho = o.resto_penalty_parameter;
      for (int j = c.lane; j < nR; j += c.width) {
        du += dabs(rho + np_jty(j, yc, yd) - zR[j]);
        cs += dabs(R[j] * zR[j] - mu_);
        ++ncs;
      }
    }
    du = c.sum(du);
    pr = c.sum(pr);
    cs = c.sum(cs);
    ncs = c.isum(ncs);
    const int ndual = D.n + D.md + (rs ? nR : 0), nprim = D.mc + D.md;
    return du / (double)(ndual > 0 ? ndual : 1) + (nprim ? pr / (double)nprim : 0.0) + (ncs ? cs / (double)ncs : 0.0);
  }

  // unscaled constraint violation (original NLP at x: c, d arrays are scaled); the restoration
  // problem is unscaled and its inequality bounds are the relaxed scaled ones
  HTP_HD HTP_FI double unscaled_viol() const {
    const gd* cc = A(L.c); const gd* dd = A(L.d);
    const gd* scE = A(L.scE); const gd* scI = A(L.scI);
    const double dmn = par(P_DMIN);
    double v = 0;
    if (rs) {
      const gd* dL = A(L.dL); const gd* dU = A(L.dU);
      {
        double c_[SW_U];
        sweep(D.mc, [&](int r, int k) { c_[k] = cc[r]; }, [&](int, int k) { v = dmax(v, dabs(c_[k])); });
      }
      {
        double l_[SW_U], d_[SW_U], u_[SW_U];
        sweep(D.md, [&](int r, int k) { l_[k] = dL[r]; d_[k] = dd[r]; u_[k] = dU[r]; },
              [&](int, int k) {
                v = dmax(v, l_[k] - d_[k]);
                if (finite_(u_[k])) v = dmax(v, d_[k] - u_[k]);
              });
      }
      return c.maxv(v);
    }
    {
      double c_[SW_U], e_[SW_U];
      sweep(D.mc, [&](int r, int k) { c_[k] = cc[r]; e_[k] = scE[r]; },
            [&](int, int k) { v = dmax(v, dabs(c_[k]) / e_[k]); });
    }
    {
      double d_[SW_U], i_[SW_U];
      sweep(D.md, [&](int r, int k) { d_[k] = dd[r]; i_[k] = scI[r]; },
            [&](int r, int k) {
              const double g = d_[k] / i_[k];
              if ((r & 1) == 0) v = dmax(v, dmax(0.0 - g, g - 1.0));
              else if (PT) v = dmax(v, dmax(dmn - g, g - 100000.0));
              else v = dmax(v, dmn - g);
            });
    }
    return c.maxv(v);
  }

  HTP_HD HTP_FI double theta_of(const gd* cc, const gd* dd, const gd* s) const {
    double t = 0;
    {
      double c_[SW_U];
      sweep(D.mc, [&](int r, int k) { c_[k] = cc[r]; }, [&](int, int k) { t += dabs(c_[k]); });
    }
    {
      double d_[SW_U], s_[SW_U];
      sweep(D.md, [&](int r, int k) { d_[k] = dd[r]; s_[k] = s[r]; }, [&](int, int k) { t += dabs(d_[k] - s_[k]); });
    }
    return c.sum(t);
  }

  // original-problem theta at (x, s) during the restoration phase: c = c_R - n + p, d = d_R - n_d + p_d
  HTP_HD HTP_FI double orig_inf_max_rs(const gd* cc, const gd* dd, const gd* s, const gd* R) const {
    const int mc = D.mc, md = D.md;
    double t = 0;
    {
      double c_[SW_U], n_[SW_U], p_[SW_U];
      sweep(mc, [&](int r, int k) { c_[k] = cc[r]; n_[k] = R[r]; p_[k] = R[mc + r]; },
            [&](int, int k) { t = dmax(t, dabs(c_[k] - n_[k] + p_[k])); });
    }
    {
      double d_[SW_U], n_[SW_U], p_[SW_U], s_[SW_U];
      sweep(md, [&](int r, int k) { d_[k] = dd[r]; n_[k] = R[2 * mc + r]; p_[k] = R[2 * mc + md + r]; s_[k] = s[r]; },
            [&](int, int k) { t = dmax(t, dabs(d_[k] - n_[k] + p_[k] - s_[k])); });
    }
    return c.maxv(t);
  }
  HTP_HD HTP_FI double orig_theta_rs(const gd* cc, const gd* dd, const gd* s, const gd* R) const {
    const int mc = D.mc, md = D.md;
    double t = 0;
    {
      double c_[SW_U], n_[SW_U], p_[SW_U];
      sweep(mc, [&](int r, int k) { c_[k] = cc[r]; n_[k] = R[r]; p_[k] = R[mc + r]; },
            [&](int, int k) { t += dabs(c_[k] - n_[k] + p_[k]); });
    }
    {
      double d_[SW_U], n_[SW_U], p_[SW_U], s_[SW_U];
      sweep(md, [&](int r, int k) { d_[k] = dd[r]; n_[k] = R[2 * mc + r]; p_[k] = R[2 * mc + md + r]; s_[k] = s[r]; },
            [&](int, int k) { t += dabs(d_[k] - n_[k] + p_[k] - s_[k]); });
    }
    return c.sum(t);
  }

  // barrier function at (x, s[, R]); +inf if a slack is not positive.  resto_obj: the restoration
  // problem's objective and n/p barrier terms, else the original sf * f
  HTP_BARRIER_ATTR HTP_HD double barrier(const gd* x, const gd* s, const gd* Rv, double mu_, bool resto_obj) const {
    const gd* xL = A(L.xL); const gd* xU = A(L.xU);
    const gd* dL = A(L.dL); const gd* dU = A(L.dU);
    const double kd = o.kappa_d * mu_;
    double lg = 0.0, lin = 0.0;
    int bad = 0;
    const gd* zL = A(L.zL); const gd* zU = A(L.zU); const gd* vL = A(L.vL); const gd* vU = A(L.vU);
    {
      double x_[SW_U], xl_[SW_U], xu_[SW_U];
      sweep(D.n, [&](int q, int k) { x_[k] = x[q]; xl_[k] = xL[q]; xu_[k] = ubx(q) ? (double)xU[q] : HTP_INF; },
            [&](int q, int k) {
              const bool hl = finite_(xl_[k]), hu = finite_(xu_[k]);
              if (hl) { const double v = safe_slack(x_[k] - xl_[k], zL[q], xl_[k], mu_); if (v <= 0) bad = 1; else lg += sm::log(v); if (!hu) lin += v; }
              if (hu) { const double v = safe_slack(xu_[k] - x_[k], zU[q], xu_[k], mu_); if (v <= 0) bad = 1; else lg += sm::log(v); if (!hl) lin += v; }
            });
    }
    double fobj = 0.0;
    if (resto_obj) {  // rho sum R + eta/2 |D_R (x - x_R)|^2 ; n/p barrier terms (lower bounds 0)
      const gd* xR = A(L.xR); const gd* dr = A(L.dr);
      const double et = o.resto_proximity_weight * sqrt(mu_);
      double px = 0.0, sr = 0.0;
      {
        double d_[SW_U], x_[SW_U], r_[SW_U];
        sweep(D.n, [&](int q, int k) { d_[k] = dr[q]; x_[k] = x[q]; r_[k] = xR[q]; },
              [&](int, int k) { const double t = d_[k] * (x_[k] - r_[k]); px += t * t; });
      }
      {
        double v_[SW_U];
        sweep(nR, [&](int j, int k) { v_[k] = Rv[j]; },
              [&](int, int k) {
                const double v = v_[k];
                if (v <= 0) bad = 1; else lg += sm::log(v);
                lin += v;
                sr += v;
              });
      }
      fobj = o.resto_penalty_parameter * c.sum(sr) + 0.5 * et * c.sum(px);
    }
    {
      double s_[SW_U], dl_[SW_U], du_[SW_U];
      sweep(D.md, [&](int r, int k) { s_[k] = s[r]; dl_[k] = dL[r]; du_[k] = ubs(r) ? (double)dU[r] : HTP_INF; },
            [&](int r, int k) {
              const bool hu = finite_(du_[k]);
              const double v = safe_slack(s_[k] - dl_[k], vL[r], dl_[k], mu_);
              if (v <= 0) bad = 1; else lg += sm::log(v);
              if (!hu) lin += v;
              if (hu) { const double w = safe_slack(du_[k] - s_[k], vU[r], du_[k], mu_); if (w <= 0) bad = 1; else lg += sm::log(w); }
            });
    }
    bad = c.isum(bad);
    lg = c.sum(lg);
    lin = c.sum(lin);
    if (bad) return HTP_INF;
    if (!resto_obj) fobj = sf * eval_f(x);
    return fobj - mu_ * lg + kd * lin;
  }

  // restoration objective gradient (x part): eta D_R^2 (x - x_R)
  HTP_HD HTP_FI void eval_grad_f_rs(const gd* x, gd* g) const {
    const gd* xR = A(L.xR); const gd* dr = A(L.dr);
    double d_[SW_U], x_[SW_U], r_[SW_U];
    sweep(D.n, [&](int q, int k) { d_[k] = dr[q]; x_[k] = x[q]; r_[k] = xR[q]; },
          [&](int q, int k) { g[q] = eta * d_[k] * d_[k] * (x_[k] - r_[k]); });
    c.sync();
  }
  HTP_HD HTP_FI void eval_grad_mode(const gd* x) {
    if (rs) eval_grad_f_rs(x, A(L.gf));
    else eval_grad_f(x, A(L.gf), sf);
  }
  // constraint values of the current mode at (x[, R]) into (cc, dd)
  HTP_HD HTP_FI void eval_cons_mode(const gd* x, const gd* Rv, gd* cc, gd* dd) const {
    eval_cons(x, cc, dd);
    if (rs) {
      const int mc = D.mc, md = D.md;
      double v_[SW_U], n_[SW_U], p_[SW_U];
      sweep(mc, [&](int r, int k) { v_[k] = cc[r]; n_[k] = Rv[r]; p_[k] = Rv[mc + r]; },
            [&](int r, int k) { cc[r] = v_[k] + (n_[k] - p_[k]); });
      sweep(md, [&](int r, int k) { v_[k] = dd[r]; n_[k] = Rv[2 * mc + r]; p_[k] = Rv[2 * mc + md + r]; },
            [&](int r, int k) { dd[r] = v_[k] + (n_[k] - p_[k]); });
      c.sync();
    }
  }

  // barrier gradient -> gx (n), gs (md); needs gf current (n/p part: rho - mu/R + kd, computed inline)
  HTP_HD HTP_FI void grad_barrier(double mu_, gd* gx, gd* gs) const {
    const gd* x = A(L.x); const gd* xL = A(L.xL); const gd* xU = A(L.xU);
    const gd* s = A(L.s); const gd* dL = A(L.dL); const gd* dU = A(L.dU);
    const gd* gf = A(L.gf);
    const double kd = o.kappa_d * mu_;
    {
      double x_[SW_U], xl_[SW_U], xu_[SW_U], g_[SW_U];
      sweep(D.n, [&](int q, int k) { x_[k] = x[q]; xl_[k] = xL[q]; xu_[k] = ubx(q) ? (double)xU[q] : HTP_INF; g_[k] = gf[q]; },
            [&](int q, int k) {
              const bool hl = finite_(xl_[k]), hu = finite_(xu_[k]);
              double g = g_[k];
              if (hl) g -= mu_ / (x_[k] - xl_[k]);
              if (hu) g += mu_ / (xu_[k] - x_[k]);
              if (hl && !hu) g += kd;
              if (hu && !hl) g -= kd;
              gx[q] = g;
            });
    }
    {
      double s_[SW_U], dl_[SW_U], du_[SW_U];
      sweep(D.md, [&](int r, int k) { s_[k] = s[r]; dl_[k] = dL[r]; du_[k] = ubs(r) ? (double)dU[r] : HTP_INF; },
            [&](int r, int k) {
              const bool hu = finite_(du_[k]);
              double g = -mu_ / (s_[k] - dl_[k]);
              if (hu) g += mu_ / (du_[k] - s_[k]);
              else g += kd;
              gs[r] = g;
            });
    }
    c.sync();
  }
  HTP_HD HTP_FI double np_grad_barrier(int j, const gd* R, double mu_) const {
    return o.resto_penalty_parameter - mu_ / R[j] + o.kappa_d * mu_;
  }

  HTP_HD HTP_FI double frac_primal(const gd* dx, const gd* ds, const gd* dR) const {
    const gd* x = A(L.x); const gd* xL = A(L.xL); const gd* xU = A(L.xU);
    const gd* s = A(L.s); const gd* dL = A(L.dL); const gd* dU = A(L.dU);
    double a = 1.0;
    {
      double x_[SW_U], xl_[SW_U], xu_[SW_U], d_[SW_U];
      sweep(D.n, [&](int q, int k) { x_[k] = x[q]; xl_[k] = xL[q]; xu_[k] = ubx(q) ? (double)xU[q] : HTP_INF; d_[k] = dx[q]; },
            [&](int, int k) {
              if (finite_(xl_[k]) && d_[k] < 0) a = dmin(a, -tau * (x_[k] - xl_[k]) / d_[k]);
              if (finite_(xu_[k]) && -d_[k] < 0) a = dmin(a, -tau * (xu_[k] - x_[k]) / (-d_[k]));
            });
    }
    {
      double s_[SW_U], dl_[SW_U], du_[SW_U], d_[SW_U];
      sweep(D.md, [&](int r, int k) { s_[k] = s[r]; dl_[k] = dL[r]; du_[k] = ubs(r) ? (double)dU[r] : HTP_INF; d_[k] = ds[r]; },
            [&](int, int k) {
              if (d_[k] < 0) a = dmin(a, -tau * (s_[k] - dl_[k]) / d_[k]);
              if (finite_(du_[k]) && -d_[k] < 0) a = dmin(a, -tau * (du_[k] - s_[k]) / (-d_[k]));
            });
    }
    if (rs) {
      const gd* R = A(L.R);
      double r_[SW_U], d_[SW_U];
      sweep(nR, [&](int j, int k) { r_[k] = R[j]; d_[k] = dR[j]; },
            [&](int, int k) { if (d_[k] < 0) a = dmin(a, -tau * r_[k] / d_[k]); });
    }
    return c.minv(a);
  }

  // bound-multiplier steps for (dx, ds[, dR]) -> dzL, dzU, dvL, dvU[, dzR] ; returns alpha_dual
  HTP_HD HTP_FI double dual_steps(const gd* dx, const gd* ds, const gd* dR) {
    const gd* x = A(L.x); const gd* xL = A(L.xL); const gd* xU = A(L.xU);
    const gd* s = A(L.s); const gd* dL = A(L.dL); const gd* dU = A(L.dU);
    const gd* zL = A(L.zL); const gd* zU = A(L.zU);
    const gd* vL = A(L.vL); const gd* vU = A(L.vU);
    gd* dzL = A(L.dzL); gd* dzU = A(L.dzU); gd* dvL = A(L.dvL); gd* dvU = A(L.dvU);
    double a = 1.0;
    {
      double x_[SW_U], xl_[SW_U], xu_[SW_U], zl_[SW_U], zu_[SW_U], d_[SW_U];
      sweep(D.n, [&](int q, int k) { x_[k] = x[q]; xl_[k] = xL[q]; xu_[k] = ubx(q) ? (double)xU[q] : HTP_INF; zl_[k] = zL[q]; zu_[k] = ubx(q) ? (double)zU[q] : 0.0; d_[k] = dx[q]; },
            [&](int q, int k) {
              double t = 0.0, u = 0.0;
              if (finite_(xl_[k])) { const double sl = x_[k] - xl_[k]; t = (mu - zl_[k] * sl - zl_[k] * d_[k]) / sl; if (t < 0) a = dmin(a, -tau * zl_[k] / t); }
              if (finite_(xu_[k])) { const double su = xu_[k] - x_[k]; u = (mu - zu_[k] * su + zu_[k] * d_[k]) / su; if (u < 0) a = dmin(a, -tau * zu_[k] / u); }
              dzL[q] = t;
              dzU[q] = u;
            });
    }
    {
      double s_[SW_U], dl_[SW_U], du_[SW_U], vl_[SW_U], vu_[SW_U], d_[SW_U];
      sweep(D.md, [&](int r, int k) { s_[k] = s[r]; dl_[k] = dL[r]; du_[k] = ubs(r) ? (double)dU[r] : HTP_INF; vl_[k] = vL[r]; vu_[k] = ubs(r) ? (double)vU[r] : 0.0; d_[k] = ds[r]; },
            [&](int r, int k) {
              const double sl = s_[k] - dl_[k];
              const double t = (mu - vl_[k] * sl - vl_[k] * d_[k]) / sl;
              if (t < 0) a = dmin(a, -tau * vl_[k] / t);
              double u = 0.0;
              if (finite_(du_[k])) { const double su = du_[k] - s_[k]; u = (mu - vu_[k] * su + vu_[k] * d_[k]) / su; if (u < 0) a = dmin(a, -tau * vu_[k] / u); }
              dvL[r] = t;
              dvU[r] = u;
            });
    }
    if (rs) {
      const gd* R = A(L.R); const gd* zR = A(L.zR);
      gd* dzR = A(L.dzR);
      double z_[SW_U], r_[SW_U], d_[SW_U];
      sweep(nR, [&](int j, int k) { z_[k] = zR[j]; r_[k] = R[j]; d_[k] = dR[j]; },
            [&](int j, int k) {
              const double t = (mu - z_[k] * r_[k] - z_[k] * d_[k]) / r_[k];
              if (t < 0) a = dmin(a, -tau * z_[k] / t);
              dzR[j] = t;
            });
    }
    c.sync();
    return c.minv(a);
  }

  // IpoptCalculatedQuantities::CalculateSafeSlack: a slack below eps * min(1, mu) becomes
  // min(max(mu / z, s_min), max(slack, 0) + slack_move * max(1, |bound|)) (z: current multiplier)
  static constexpr double SLACK_MOVE = 1.8189894035458565e-12;  // eps^(3/4)
  HTP_HD HTP_FI static double safe_slack(double v, double z, double bound, double mu_) {
    const double smin = 2.220446049250313e-16 * dmin(1.0, mu_);
    if (!(v < smin)) return v;
    return dmin(dmax(mu_ / z, smin), dmax(v, 0.0) + SLACK_MOVE * dmax(1.0, dabs(bound)));
  }

  HTP_HD HTP_FI static bool cmp_le(double lhs, double rhs, double basval) {
    return lhs - rhs <= 10.0 * 2.220446049250313e-16 * dabs(basval);
  }

  // factorization with inertia correction (IPOPT PDPerturbationHandler, simplified)
  HTP_HD HTP_FI bool factor_ic(double& dw, double& dc) {
    dw = 0.0;
    dc = 0.0;
    const int need = D.mc + D.md;
    for (;;) {
      int neg, zero;
      ic_scan = HTP_IC_SCAN && !PT && !rs;
      ic_skip = 0;
      factorize(false, dw, dc, neg, zero);
      ic_scan = false;
      ++n_factor;
#ifdef HTP_HOST_DEBUG
      printf("[dbg] factor dw=%g dc=%g neg=%d need=%d zero=%d skip=%d\n", dw, dc, neg, need, zero, ic_skip);
#endif
      if (neg == need && zero == 0) return true;
      if (zero > 0 && dc == 0.0) { dc = o.dc_bar * sm::pow(mu, o.kappa_c); continue; }
      for (int k = 0; k <= ic_skip; ++k) {
        dw = next_dw(dw);
        if (dw > o.dw_max) return false;
      }
    }
  }
  // IPOPT's next trial delta_w after a factorization with the wrong inertia
  HTP_HD HTP_FI double next_dw(double dw) const {
    if (dw == 0.0) return (dw_last == 0.0) ? o.dw0 : dmax(o.dw_min, o.kw_minus * dw_last);
    return ((dw_last == 0.0 || 1e5 * dw_last < dw) ? o.kw_plus_bar : o.kw_plus) * dw;
  }

  // ---------------------------------------------------------- filter / acceptor state
  static constexpr int NLS = 24;  // doubles of LsState when saved
  struct LsState {
    double last_mu, wd_th, wd_ph, wd_gbd, wd_alpha, wd_dw, wd_dc, th_max, th_min, dwl, mu_, tau_;
    int in_wd, wd_short, wd_trial, tiny_last, tiny_flag, in_soft, soft_cnt, last_rej_filter, cnt_filter_rej,
        n_filter_resets, fallback, acc_count;
  };
  LsState ls_;
  int nfilt_resto_base = 0;
  int n_resto = 0;
  bool have_acc = false;

  HTP_HD HTP_FI void ls_reset() {
    ls_.last_mu = -1.0;
    ls_.wd_th = ls_.wd_ph = ls_.wd_gbd = ls_.wd_alpha = ls_.wd_dw = ls_.wd_dc = 0.0;
    ls_.in_wd = ls_.wd_short = ls_.wd_trial = ls_.tiny_last = ls_.tiny_flag = 0;
    ls_.in_soft = ls_.soft_cnt = ls_.last_rej_filter = ls_.cnt_filter_rej = ls_.n_filter_resets = 0;
    ls_.fallback = ls_.acc_count = 0;
  }
  HTP_HD HTP_FI void ls_save(gd* v) const {
    if (c.lane == 0) {
      const double dv[12] = {ls_.last_mu, ls_.wd_th, ls_.wd_ph, ls_.wd_gbd, ls_.wd_alpha, ls_.wd_dw, ls_.wd_dc,
                             theta_max, theta_min, dw_last, mu, tau};
      const int iv[12] = {ls_.in_wd, ls_.wd_short, ls_.wd_trial, ls_.tiny_last, ls_.tiny_flag, ls_.in_soft,
                          ls_.soft_cnt, ls_.last_rej_filter, ls_.cnt_filter_rej, ls_.n_filter_resets, ls_.fallback,
                          ls_.acc_count};
      for (int k = 0; k < 12; ++k) { v[k] = dv[k]; v[12 + k] = (double)iv[k]; }
    }
    c.sync();
  }
  HTP_HD HTP_FI void ls_load(const gd* v) {
    ls_.last_mu = c.uniform(v[0]); ls_.wd_th = c.uniform(v[1]); ls_.wd_ph = c.uniform(v[2]);
    ls_.wd_gbd = c.uniform(v[3]); ls_.wd_alpha = c.uniform(v[4]); ls_.wd_dw = c.uniform(v[5]);
    ls_.wd_dc = c.uniform(v[6]); theta_max = c.uniform(v[7]); theta_min = c.uniform(v[8]);
    dw_last = c.uniform(v[9]); mu = c.uniform(v[10]); tau = c.uniform(v[11]);
    int* iv[12] = {&ls_.in_wd, &ls_.wd_short, &ls_.wd_trial, &ls_.tiny_last, &ls_.tiny_flag, &ls_.in_soft,
                   &ls_.soft_cnt, &ls_.last_rej_filter, &ls_.cnt_filter_rej, &ls_.n_filter_resets, &ls_.fallback,
                   &ls_.acc_count};
    for (int k = 0; k < 12; ++k) *iv[k] = (int)c.uniform(v[12 + k]);
  }

  HTP_HD HTP_FI void filter_add(double theta, double phi) {
    c.sync();
    if (c.lane == 0) {
      if (nfilt < FMAX) { f_th[nfilt] = (1 - o.gamma_theta) * theta; f_ph[nfilt] = phi - o.gamma_phi * theta; }
      else { for (int k = 1; k < FMAX; ++k) { f_th[k - 1] = f_th[k]; f_ph[k - 1] = f_ph[k]; }
             f_th[FMAX - 1] = (1 - o.gamma_theta) * theta; f_ph[FMAX - 1] = phi - o.gamma_phi * theta; }
    }
    if (nfilt < FMAX) ++nfilt;
    c.sync();
  }
  HTP_HD HTP_FI bool filter_ok(double th_t, double ph_t) const {
    for (int k = 0; k < nfilt; ++k)
      if (!(th_t < f_th[k] || ph_t < f_ph[k])) return false;
    return true;
  }
  HTP_HD HTP_FI bool is_ftype(double th, double gbd, double a) const {
    return gbd < 0 && a * sm::pow(-gbd, o.s_phi) > o.delta * sm::pow(th, o.s_theta);
  }
  HTP_HD HTP_FI bool armijo(double ph, double gbd, double a, double ph_t) const {
    return cmp_le(ph_t - ph, o.eta_phi * a * gbd, ph);
  }
  HTP_HD HTP_FI bool acc_to_iterate(double th, double ph, double ph_t, double th_t, bool from_resto) const {
    if (!from_resto && ph_t > ph) {
      const double basval = dabs(ph) > 10.0 ? sm::log10(dabs(ph)) : 1.0;
      if (sm::log10(ph_t - ph) > o.obj_max_inc + basval) return false;
    }
    return cmp_le(th_t, (1 - o.gamma_theta) * th, th) || cmp_le(ph_t - ph, -o.gamma_phi * th, ph);
  }
  // FilterLSAcceptor::CheckAcceptabilityOfTrialPoint against reference (th, ph, gbd)
  HTP_HD HTP_FI bool check_trial(double th, double ph, double gbd, double a_test, double th_t, double ph_t) {
    if ((HTP_NAN_GUARD ? !(th_t <= theta_max) : th_t > theta_max) || !(ph_t < 1e300)) return false;   // NaN: evaluation error
    bool ok;
    if (a_test > 0 && is_ftype(th, gbd, a_test) && th <= theta_min) ok = armijo(ph, gbd, a_test, ph_t);
    else ok = acc_to_iterate(th, ph, ph_t, th_t, false);
    if (!ok) { ls_.last_rej_filter = 0; return false; }
    if (!filter_ok(th_t, ph_t)) { ls_.last_rej_filter = 1; return false; }
    return true;
  }
  HTP_HD HTP_FI void update_for_next_iteration(double th, double ph, double gbd, double a_test, double ph_t) {
    if (!(is_ftype(th, gbd, a_test) && armijo(ph, gbd, a_test, ph_t))) filter_add(th, ph);
    if (o.max_filter_resets > 0) {
      if (ls_.n_filter_resets < o.max_filter_resets) {
        if (ls_.last_rej_filter) {
          if (++ls_.cnt_filter_rej >= o.filter_reset_trigger) {
            nfilt = 0;
            ls_.cnt_filter_rej = 0;
            ++ls_.n_filter_resets;
          }
        } else {
          ls_.cnt_filter_rej = 0;
        }
      }
      ls_.last_rej_filter = 0;
    }
  }

  // trial point (xt, st[, Rt]) values: ct, dt, theta, barrier
  HTP_HD HTP_PHASE void trial_values(const gd* xt, const gd* st, const gd* Rt, double& th_t, double& ph_t) {
    gd* ct = A(L.ct);
    gd* dtv = A(L.dt);
    eval_cons_mode(xt, Rt, ct, dtv);
    th_t = theta_of(ct, dtv, st);
    ph_t = barrier(xt, st, Rt, mu, rs);
  }
  HTP_HD HTP_FI void set_trial(double alpha, const gd* dx, const gd* ds, const gd* dR) {
    const gd* x = A(L.x); const gd* s = A(L.s);
    gd* xt = A(L.xt); gd* st = A(L.st);
    {
      double a_[SW_U], b_[SW_U];
      sweep(D.n, [&](int q, int k) { a_[k] = x[q]; b_[k] = dx[q]; }, [&](int q, int k) { xt[q] = a_[k] + alpha * b_[k]; });
      sweep(D.md, [&](int r, int k) { a_[k] = s[r]; b_[k] = ds[r]; }, [&](int r, int k) { st[r] = a_[k] + alpha * b_[k]; });
    }
    if (rs) {
      const gd* R = A(L.R);
      gd* Rt = A(L.Rt);
      double r_[SW_U], d_[SW_U];
      sweep(nR, [&](int j, int k) { r_[k] = R[j]; d_[k] = dR[j]; }, [&](int j, int k) { Rt[j] = r_[k] + alpha * d_[k]; });
    }
    c.sync();
  }

  HTP_HD HTP_FI void copy_arr(gd* dst, const gd* src, int n) {
    double a_[SW_U];
    sweep(n, [&](int q, int k) { a_[k] = src[q]; }, [&](int q, int k) { dst[q] = a_[k]; });
    c.sync();
  }

  HTP_HD HTP_FI void run(Result& res) {
    for (int k = 0; k < 8; ++k) cyc[k] = 0;
    const long long t0 = c.clock();
    initialize();
    iterate(res);
    if (c.lane == 0) {
      for (int k = 0; k < 8; ++k) res.cyc[k] = cyc[k];
#ifdef HTP_PROF_ON
#if HTP_PROF_ON == 2   // the Riccati solve passes split: backward fill / stages, forward fill / stages; factor sub-steps
      { const long long v[7] = {spcyc[0], spcyc[1], spcyc[2], spcyc[3], pcyc[1], pcyc[3], pcyc[5]};
        const int slot[7] = {0, 1, 2, 3, 5, 6, 7};
        for (int k = 0; k < 7; ++k) res.cyc[slot[k]] = v[k]; }
#else
      for (int k = 0; k < 8; ++k)
        if (k != 4) res.cyc[k] = pcyc[k];
#endif
#endif
#ifdef HTP_LPROF
      { const int slot[7] = {0, 1, 2, 3, 5, 6, 7};
        for (int k = 0; k < 7; ++k) res.cyc[slot[k]] = lprof[k]; }
#endif
#ifdef HTP_KKT_PROF
#if HTP_KKT_PROF == 2
      const int slot[7] = {0, 1, 2, 3, 5, 6, 7};
      for (int k = 0; k < 7; ++k) res.cyc[slot[k]] = kprof[k];
#else
      for (int k = 0; k < 3; ++k) res.cyc[5 + k] = kprof[k];
#endif
#endif
      res.cyc[4] = c.clock() - t0;
    }
  }

  HTP_HD HTP_FI void initialize() {
    n_factor = 0;
    for (int k = 0; k < 8; ++k) cyc[k] = 0;
    dw_last = 0.0;
    nfilt = 0;
    rs = false;
    nR = 2 * D.mc + 2 * D.md;
    n_resto = 0;
    have_acc = false;
    ls_reset();
    set_bounds_and_x0();
    HTP_TRACE("[trace] bounds\n");
    compute_scaling();
    HTP_TRACE("[trace] scaling sf=%g\n", sf);
    relax_and_push();
    HTP_TRACE("[trace] push\n");
    gd* x = A(L.x); gd* s = A(L.s);
    gd* cc = A(L.c); gd* dd = A(L.d);
    eval_cons(x, cc, dd);
    HTP_TRACE("[trace] cons\n");
    set_slack_bounds_and_push();
    count_bounds();
    HTP_TRACE("[trace] counted %d %d %d\n", nbL, nbU, nsU);
    {
      const gd* xL = A(L.xL); const gd* xU = A(L.xU); const gd* dU = A(L.dU);
      gd* zL = A(L.zL); gd* zU = A(L.zU); gd* vL = A(L.vL); gd* vU = A(L.vU);
      HTP_UNROLL
      for (int q = c.lane; q < D.n; q += c.width) {
        zL[q] = finite_(xL[q]) ? o.bound_mult_init_val : 0.0;
        zU[q] = finite_(xU[q]) ? o.bound_mult_init_val : 0.0;
      }
      HTP_UNROLL
      for (int r = c.lane; r < D.md; r += c.width) {
        vL[r] = o.bound_mult_init_val;
        vU[r] = finite_(dU[r]) ? o.bound_mult_init_val : 0.0;
      }
      c.sync();
    }
    eval_grad_f(x, A(L.gf), sf);
    ls_multipliers();
    mu = o.mu_init;
    tau = dmax(o.tau_min, 1.0 - mu);
    {
      const double th0 = theta_of(cc, dd, s);
      theta_max = 1e4 * dmax(1.0, th0);
      theta_min = 1e-4 * dmax(1.0, th0);
    }
  }

  // least-squares constraint multipliers [I 0 Jc' Jd'; 0 I 0 -I; Jc 0 0 0; Jd -I 0 0] (current mode);
  // y = 0 unless the inertia is right and |y|_inf <= constr_mult_init_max
  HTP_HD HTP_FI void ls_multipliers() {
    gd* yc = A(L.yc); gd* yd = A(L.yd);
    HTP_UNROLL
    for (int r = c.lane; r < D.mc; r += c.width) yc[r] = 0.0;
    HTP_UNROLL
    for (int r = c.lane; r < D.md; r += c.width) yd[r] = 0.0;
    c.sync();
    int neg, zero;
    factorize(true, 0.0, 0.0, neg, zero);
    ++n_factor;
    HTP_TRACE("[trace] LS factor neg=%d zero=%d\n", neg, zero);
    if (!(neg == D.mc + D.md && zero == 0)) return;
    gd* bx = A(L.rx); gd* bs = A(L.rs); gd* bc = A(L.rc); gd* bd = A(L.rd);
    const gd* gf = A(L.gf);
    const gd* zL = A(L.zL); const gd* zU = A(L.zU); const gd* vL = A(L.vL); const gd* vU = A(L.vU);
    HTP_UNROLL
    for (int q = c.lane; q < D.n; q += c.width) bx[q] = -(gf[q] - zL[q] + zU[q]);
    HTP_UNROLL
    for (int r = c.lane; r < D.md; r += c.width) { bs[r] = -(-vL[r] + vU[r]); bd[r] = 0.0; }
    HTP_UNROLL
    for (int r = c.lane; r < D.mc; r += c.width) bc[r] = 0.0;
    gd* bR = A(L.rRx);
    if (rs) {
      const gd* zR = A(L.zR);
      for (int j = c.lane; j < nR; j += c.width) bR[j] = -(o.resto_penalty_parameter - zR[j]);
    }
    c.sync();
    kkt_solve(true, 0.0, 0.0, bx, bs, bc, bd, A(L.dx), A(L.ds), A(L.dyc), A(L.dyd), bR, A(L.dR));
    HTP_TRACE("[trace] LS solve\n");
    const gd* a1 = A(L.dyc); const gd* a2 = A(L.dyd);
    double mx = 0.0;
    HTP_UNROLL
    for (int r = c.lane; r < D.mc; r += c.width) mx = dmax(mx, dabs(a1[r]));
    HTP_UNROLL
    for (int r = c.lane; r < D.md; r += c.width) mx = dmax(mx, dabs(a2[r]));
    mx = c.maxv(mx);
    if (mx <= o.constr_mult_init_max) {
      HTP_UNROLL
      for (int r = c.lane; r < D.mc; r += c.width) yc[r] = a1[r];
      HTP_UNROLL
      for (int r = c.lane; r < D.md; r += c.width) yd[r] = a2[r];
    }
    c.sync();
  }

  // Newton right-hand side at the current point: rx (into xt), rs, rc, rd[, rRx] ; gbx (sx), gbs (ss)
  // returns the directional-derivative factors via gBD once the step exists (newton_gbd)
  HTP_HD HTP_FI void build_newton_rhs(const gd* gl) {
    gd* gbx = A(L.sx); gd* gbs = A(L.ss);
    grad_barrier(mu, gbx, gbs);
    gd* rx = A(L.xt);
    gd* rs_ = A(L.rs); gd* rc = A(L.rc); gd* rd = A(L.rd);
    const gd* gf = A(L.gf); const gd* yd = A(L.yd); const gd* cc = A(L.c); const gd* dd = A(L.d);
    const gd* s = A(L.s);
    {
      double a_[SW_U], b_[SW_U], g_[SW_U];
      sweep(D.n, [&](int q, int k) { a_[k] = gl[q]; b_[k] = gf[q]; g_[k] = gbx[q]; },
            [&](int q, int k) { rx[q] = -(a_[k] - b_[k] + g_[k]); });
    }
    {
      double a_[SW_U], b_[SW_U], d_[SW_U], s_[SW_U];
      sweep(D.md, [&](int r, int k) { a_[k] = gbs[r]; b_[k] = yd[r]; d_[k] = dd[r]; s_[k] = s[r]; },
            [&](int r, int k) { rs_[r] = -(a_[k] - b_[k]); rd[r] = -(d_[k] - s_[k]); });
    }
    {
      double a_[SW_U];
      sweep(D.mc, [&](int r, int k) { a_[k] = cc[r]; }, [&](int r, int k) { rc[r] = -a_[k]; });
    }
    if (rs) {
      const gd* R = A(L.R); const gd* yc = A(L.yc);
      gd* rR = A(L.rRx);
      const gd* yd_ = A(L.yd);
      double b_[SW_U], t_[SW_U];
      sweep(nR, [&](int j, int k) { b_[k] = np_grad_barrier(j, R, mu); t_[k] = np_jty(j, yc, yd_); },
            [&](int j, int k) { rR[j] = -(b_[k] + t_[k]); });
    }
    c.sync();
  }
  // gradient of the barrier function along (dx, ds[, dR]); gbx, gbs must be current (sx, ss)
  HTP_HD HTP_FI double newton_gbd(const gd* dx, const gd* ds, const gd* dR) {
    const gd* gbx = A(L.sx); const gd* gbs = A(L.ss);
    double g = 0.0;
    {
      double a_[SW_U], b_[SW_U];
      sweep(D.n, [&](int q, int k) { a_[k] = gbx[q]; b_[k] = dx[q]; }, [&](int, int k) { g += a_[k] * b_[k]; });
      sweep(D.md, [&](int r, int k) { a_[k] = gbs[r]; b_[k] = ds[r]; }, [&](int, int k) { g += a_[k] * b_[k]; });
    }
    if (rs) {
      const gd* R = A(L.R);
      double b_[SW_U], d_[SW_U];
      sweep(nR, [&](int j, int k) { b_[k] = np_grad_barrier(j, R, mu); d_[k] = dR[j]; },
            [&](int, int k) { g += b_[k] * d_[k]; });
    }
    return c.sum(g);
  }

  // accept the trial step alpha along (dx, ds, dyc, dyd[, dR]): primal from x + a dx (bitwise the trial
  // point), dual step with a_dual, kappa_Sigma safeguard; constraint values from the trial (ct, dt)
  HTP_HD HTP_FI void accept_step(double a_primal, double a_dual, const gd* dx, const gd* ds, const gd* dyc,
                                 const gd* dyd, const gd* dR) {
    gd* x = A(L.x); gd* s = A(L.s);
    gd* zL = A(L.zL); gd* zU = A(L.zU); gd* vL = A(L.vL); gd* vU = A(L.vU);
    gd* yc = A(L.yc); gd* yd = A(L.yd);
    const gd* dzL = A(L.dzL); const gd* dzU = A(L.dzU);
    const gd* dvL = A(L.dvL); const gd* dvU = A(L.dvU);
    gd* xL = A(L.xL); gd* xU = A(L.xU);
    gd* dL = A(L.dL); gd* dU = A(L.dU);
    const double ks = o.kappa_sigma;
    {
      double x_[SW_U], d_[SW_U], xl_[SW_U], xu_[SW_U], zl_[SW_U], zu_[SW_U], dzl_[SW_U], dzu_[SW_U];
      sweep(D.n, [&](int q, int k) { x_[k] = x[q]; d_[k] = dx[q]; xl_[k] = xL[q]; xu_[k] = ubx(q) ? (double)xU[q] : HTP_INF; zl_[k] = zL[q];
                                      zu_[k] = ubx(q) ? (double)zU[q] : 0.0; dzl_[k] = dzL[q]; dzu_[k] = ubx(q) ? (double)dzU[q] : 0.0; },
            [&](int q, int k) {
              const double xn = x_[k] + a_primal * d_[k];
              x[q] = xn;
              if (finite_(xl_[k])) {
                const double v0 = xn - xl_[k], v = safe_slack(v0, zl_[k], xl_[k], mu);
                if (v != v0) xL[q] = xn - v;
                const double z = zl_[k] + a_dual * dzl_[k];
                zL[q] = dmax(dmin(z, ks * mu / v), mu / (ks * v));
              }
              if (finite_(xu_[k])) {
                const double v0 = xu_[k] - xn, v = safe_slack(v0, zu_[k], xu_[k], mu);
                if (v != v0) xU[q] = xn + v;
                const double z = zu_[k] + a_dual * dzu_[k];
                zU[q] = dmax(dmin(z, ks * mu / v), mu / (ks * v));
              }
            });
    }
    {
      double s_[SW_U], d_[SW_U], y_[SW_U], dy_[SW_U], vl_[SW_U], dvl_[SW_U], dl_[SW_U], vu_[SW_U], dvu_[SW_U], du_[SW_U];
      sweep(D.md, [&](int r, int k) { s_[k] = s[r]; d_[k] = ds[r]; y_[k] = yd[r]; dy_[k] = dyd[r]; vl_[k] = vL[r];
                                       dvl_[k] = dvL[r]; dl_[k] = dL[r]; vu_[k] = ubs(r) ? (double)vU[r] : 0.0; dvu_[k] = ubs(r) ? (double)dvU[r] : 0.0; du_[k] = ubs(r) ? (double)dU[r] : HTP_INF; },
            [&](int r, int k) {
              const double sn = s_[k] + a_primal * d_[k];
              s[r] = sn;
              yd[r] = y_[k] + a_primal * dy_[k];
              {
                const double v0 = sn - dl_[k], v = safe_slack(v0, vl_[k], dl_[k], mu);
                if (v != v0) dL[r] = sn - v;
                const double z = vl_[k] + a_dual * dvl_[k];
                vL[r] = dmax(dmin(z, ks * mu / v), mu / (ks * v));
              }
              if (finite_(du_[k])) {
                const double v0 = du_[k] - sn, v = safe_slack(v0, vu_[k], du_[k], mu);
                if (v != v0) dU[r] = sn + v;
                const double z = vu_[k] + a_dual * dvu_[k];
                vU[r] = dmax(dmin(z, ks * mu / v), mu / (ks * v));
              }
            });
    }
    {
      double y_[SW_U], dy_[SW_U];
      sweep(D.mc, [&](int r, int k) { y_[k] = yc[r]; dy_[k] = dyc[r]; },
            [&](int r, int k) { yc[r] = y_[k] + a_primal * dy_[k]; });
    }
    if (rs) {
      gd* R = A(L.R); gd* zR = A(L.zR);
      const gd* dzR = A(L.dzR);
      double r_[SW_U], d_[SW_U], z_[SW_U], dz_[SW_U];
      sweep(nR, [&](int j, int k) { r_[k] = R[j]; d_[k] = dR[j]; z_[k] = zR[j]; dz_[k] = dzR[j]; },
            [&](int j, int k) {
              const double rn = r_[k] + a_primal * d_[k];
              R[j] = rn;
              const double z = z_[k] + a_dual * dz_[k];
              zR[j] = dmax(dmin(z, ks * mu / rn), mu / (ks * rn));
            });
    }
    c.sync();
    copy_arr(A(L.c), A(L.ct), D.mc);
    copy_arr(A(L.d), A(L.dt), D.md);
  }

  // IpBacktrackingLineSearch::DetectTinyStep (x includes R in the restoration phase)
  HTP_HD HTP_FI bool detect_tiny_step(const gd* dx, const gd* ds, const gd* dyc, const gd* dyd, const gd* dR) {
    if (o.tiny_step_tol == 0.0) return false;
    const gd* x = A(L.x); const gd* s = A(L.s); const gd* cc = A(L.c); const gd* dd = A(L.d);
    double mx = 0.0, ms = 0.0, my = 0.0, pv = 0.0;
    {
      double d_[SW_U], x_[SW_U];
      sweep(D.n, [&](int q, int k) { d_[k] = dx[q]; x_[k] = x[q]; },
            [&](int, int k) { mx = nmax(mx, dabs(d_[k]) / (1.0 + dabs(x_[k]))); });
      if (rs) {
        const gd* R = A(L.R);
        sweep(nR, [&](int j, int k) { d_[k] = dR[j]; x_[k] = R[j]; },
              [&](int, int k) { mx = nmax(mx, dabs(d_[k]) / (1.0 + dabs(x_[k]))); });
      }
    }
    {
      double d_[SW_U], s_[SW_U], y_[SW_U], v_[SW_U];
      sweep(D.md, [&](int r, int k) { d_[k] = ds[r]; s_[k] = s[r]; y_[k] = dyd[r]; v_[k] = dd[r]; },
            [&](int, int k) {
              ms = nmax(ms, dabs(d_[k]) / (1.0 + dabs(s_[k])));
              my = nmax(my, dabs(y_[k]));
              pv = nmax(pv, dabs(v_[k] - s_[k]));
            });
    }
    {
      double y_[SW_U], c_[SW_U];
      sweep(D.mc, [&](int r, int k) { y_[k] = dyc[r]; c_[k] = cc[r]; },
            [&](int, int k) {
              my = nmax(my, dabs(y_[k]));
              pv = nmax(pv, dabs(c_[k]));
            });
    }
    // a NaN anywhere in the step is not a tiny step (the wave maxima below drop NaN operands)
    if (HTP_NAN_GUARD && c.isum((mx == mx && ms == ms && my == my && pv == pv) ? 0 : 1) > 0) return false;
    mx = c.maxv(mx); ms = c.maxv(ms); my = c.maxv(my); pv = c.maxv(pv);
    if (mx > o.tiny_step_tol || ms > o.tiny_step_tol) return false;
    if (my >= o.tiny_step_y_tol) return false;
    if (pv > 1e-4) return false;
    return true;
  }

  // ---------------------------------------------------------- watchdog
  // stores the current point, its constraint values, the step and the reference values
  HTP_COLD HTP_HD void start_watchdog(double th, double ph, double gbd, double dw, double dc) {
    ls_.in_wd = 1;
    ls_.wd_th = th; ls_.wd_ph = ph; ls_.wd_gbd = gbd; ls_.wd_dw = dw; ls_.wd_dc = dc;
    ls_.wd_trial = 0;
    ls_.wd_alpha = frac_primal(A(L.dx), A(L.ds), A(L.dR));
    copy_arr(A(L.wx), A(L.x), D.n); copy_arr(A(L.ws), A(L.s), D.md);
    copy_arr(A(L.wyc), A(L.yc), D.mc); copy_arr(A(L.wyd), A(L.yd), D.md);
    copy_arr(A(L.wzL), A(L.zL), D.n); copy_arr(A(L.wzU), A(L.zU), D.n);
    copy_arr(A(L.wvL), A(L.vL), D.md); copy_arr(A(L.wvU), A(L.vU), D.md);
    copy_arr(A(L.wc), A(L.c), D.mc); copy_arr(A(L.wd), A(L.d), D.md);
    copy_arr(A(L.wdx), A(L.dx), D.n); copy_arr(A(L.wds), A(L.ds), D.md);
    copy_arr(A(L.wdyc), A(L.dyc), D.mc); copy_arr(A(L.wdyd), A(L.dyd), D.md);
    if (rs) { copy_arr(A(L.wR), A(L.R), nR); copy_arr(A(L.wzR), A(L.zR), nR); copy_arr(A(L.wdR), A(L.dR), nR); }
  }
  // back to the stored point and step; its gradients, Newton rhs and the stored matrix (for SOC)
  HTP_COLD HTP_HD void stop_watchdog() {
    ls_.in_wd = 0;
    copy_arr(A(L.x), A(L.wx), D.n); copy_arr(A(L.s), A(L.ws), D.md);
    copy_arr(A(L.yc), A(L.wyc), D.mc); copy_arr(A(L.yd), A(L.wyd), D.md);
    copy_arr(A(L.zL), A(L.wzL), D.n); copy_arr(A(L.zU), A(L.wzU), D.n);
    copy_arr(A(L.vL), A(L.wvL), D.md); copy_arr(A(L.vU), A(L.wvU), D.md);
    copy_arr(A(L.c), A(L.wc), D.mc); copy_arr(A(L.d), A(L.wd), D.md);
    copy_arr(A(L.dx), A(L.wdx), D.n); copy_arr(A(L.ds), A(L.wds), D.md);
    copy_arr(A(L.dyc), A(L.wdyc), D.mc); copy_arr(A(L.dyd), A(L.wdyd), D.md);
    if (rs) { copy_arr(A(L.R), A(L.wR), nR); copy_arr(A(L.zR), A(L.wzR), nR); copy_arr(A(L.dR), A(L.wdR), nR); }
    eval_grad_mode(A(L.x));
    gd* gl = A(L.rx);
    grad_lag_into(gl);
    build_newton_rhs(gl);
    int neg, zero;
    factorize(false, ls_.wd_dw, ls_.wd_dc, neg, zero);
    ++n_factor;
    ls_.wd_short = 0;
  }

  // ---------------------------------------------------------- line search
  // DoBacktrackingLineSearch with second-order corrections.  On return the trial point (xt, st[, Rt],
  // ct, dt) holds the last tested point; the step arrays hold the direction actually taken.
  HTP_HD HTP_PHASE bool backtrack(double th, double ph, double gbd, bool skip_first, int& n_steps,
                                  double& a_primal, double& a_test, double& ph_acc, double& th_acc,
                                  double dw, double dc) {
    gd* x = A(L.x); gd* s = A(L.s);
    gd* dx = A(L.dx); gd* ds = A(L.ds); gd* dyc = A(L.dyc); gd* dyd = A(L.dyd); gd* dR = A(L.dR);
    const gd* cc = A(L.c); const gd* dd = A(L.d);
    const double alpha_max = frac_primal(dx, ds, dR);
    double alpha_min;
    if (ls_.in_wd) {
      alpha_min = alpha_max;
    } else {
      alpha_min = o.gamma_theta;
      if (gbd < 0) {
        alpha_min = dmin(o.gamma_theta, o.gamma_phi * th / (-gbd));
        if (th <= theta_min) alpha_min = dmin(alpha_min, o.delta * sm::pow(th, o.s_theta) / sm::pow(-gbd, o.s_phi));
      }
      alpha_min *= o.alpha_min_frac;
    }
    double alpha = alpha_max;
    if (skip_first) alpha *= 0.5;
    bool accept = false;
    const double theta_curr = th;  // the reference point is the current point here
    double th_t = 0.0, ph_t = 0.0;
    gd* xt = A(L.xt); gd* st = A(L.st); gd* Rt = A(L.Rt);
    while (alpha > alpha_min || n_steps == 0) {
      set_trial(alpha, dx, ds, dR);
      trial_values(xt, st, Rt, th_t, ph_t);
      a_test = ls_.in_wd ? ls_.wd_alpha : alpha;
      if (check_trial(th, ph, gbd, a_test, th_t, ph_t)) { accept = true; break; }
      HTP_TRACE("[trace]   ls alpha=%.17g th_t=%.17g ph_t=%.17g (theta=%.17g phi=%.17g gBD=%.17g amax=%.17g)\n", alpha, th_t, ph_t, th, ph, gbd, alpha_max);
      if (ls_.in_wd) break;
      if (alpha == alpha_max && theta_curr <= th_t && o.max_soc > 0) {
        // second-order corrections (IPOPT TrySecondOrderCorrection); rhs x part is rxk (sx)
        gd* csoc = A(L.csoc); gd* dsoc = A(L.dsoc);
        const gd* ct = A(L.ct); const gd* dtv = A(L.dt);
        HTP_UNROLL
        for (int r = c.lane; r < D.mc; r += c.width) csoc[r] = alpha * cc[r] + ct[r];
        HTP_UNROLL
        for (int r = c.lane; r < D.md; r += c.width) dsoc[r] = alpha * (dd[r] - s[r]) + (dtv[r] - st[r]);
        c.sync();
        double th_old = th;
        gd* sx = A(L.dzL);  // temporaries (dz arrays are recomputed after acceptance)
        gd* ss_ = A(L.dvL); gd* syc = A(L.syc); gd* syd = A(L.syd); gd* sR = A(L.dzR);
        gd* nrc = A(L.ct); gd* nrd = A(L.dt);
        const gd* rxk = A(L.sx);
        bool soc_ok = false;
        for (int k = 0; k < o.max_soc; ++k) {
          HTP_UNROLL
          for (int r = c.lane; r < D.mc; r += c.width) nrc[r] = -csoc[r];
          HTP_UNROLL
          for (int r = c.lane; r < D.md; r += c.width) nrd[r] = -dsoc[r];
          c.sync();
          kkt_solve(false, dw, dc, rxk, A(L.rs), nrc, nrd, sx, ss_, syc, syd, A(L.rRx), sR);
          const double a_soc = frac_primal(sx, ss_, sR);
          set_trial(a_soc, sx, ss_, sR);
          double th_soc, ph_soc;
          trial_values(xt, st, Rt, th_soc, ph_soc);
          if (check_trial(th, ph, gbd, a_test, th_soc, ph_soc)) {
            soc_ok = true; alpha = a_soc; th_t = th_soc; ph_t = ph_soc;
            copy_arr(dx, sx, D.n); copy_arr(ds, ss_, D.md); copy_arr(dyc, syc, D.mc); copy_arr(dyd, syd, D.md);
            if (rs) copy_arr(dR, sR, nR);
            break;
          }
          if (th_soc > o.kappa_soc * th_old) break;
          th_old = th_soc;
          const gd* ct2 = A(L.ct); const gd* dt2 = A(L.dt);
          HTP_UNROLL
          for (int r = c.lane; r < D.mc; r += c.width) csoc[r] = a_soc * csoc[r] + ct2[r];
          HTP_UNROLL
          for (int r = c.lane; r < D.md; r += c.width) dsoc[r] = a_soc * dsoc[r] + (dt2[r] - st[r]);
          c.sync();
        }
        if (soc_ok) { accept = true; break; }
      }
      alpha *= 0.5;
      ++n_steps;
    }
    a_primal = alpha;
    ph_acc = ph_t;
    th_acc = th_t;
    if (accept) update_for_next_iteration(th, ph, gbd, a_test, ph_t);
    (void)x;
    return accept;
  }

  // TrySoftRestoStep: the primal-dual step with alpha = min(primal, dual fraction to the boundary).
  // Returns 0 (rejected: nothing changed), 1 (accepted: primal-dual error reduced), 2 (accepted and
  // acceptable to the original filter criteria).  On acceptance the new iterate is in place.
  HTP_COLD HTP_HD int try_soft_resto_step(double th, double ph, double gbd, const gd* gl) {
    const gd* dx = A(L.dx); const gd* ds = A(L.ds); const gd* dyc = A(L.dyc); const gd* dyd = A(L.dyd);
    const gd* dR = A(L.dR);
    const double ap = frac_primal(dx, ds, dR);
    const double ad = dual_steps(dx, ds, dR);
    const double a = dmin(ap, ad);
    set_trial(a, dx, ds, dR);
    gd* xt = A(L.xt); gd* st = A(L.st); gd* Rt = A(L.Rt);
    double th_t, ph_t;
    trial_values(xt, st, Rt, th_t, ph_t);
    // trial multipliers (the watchdog arrays are free whenever this runs)
    gd* tyc = A(L.wyc); gd* tyd = A(L.wyd); gd* tzL = A(L.wzL); gd* tzU = A(L.wzU);
    gd* tvL = A(L.wvL); gd* tvU = A(L.wvU); gd* tzR = A(L.wzR);
    {
      const gd* xL = A(L.xL); const gd* xU = A(L.xU); const gd* dL = A(L.dL); const gd* dU = A(L.dU);
      const gd* yc = A(L.yc); const gd* yd = A(L.yd); const gd* zL = A(L.zL); const gd* zU = A(L.zU);
      const gd* vL = A(L.vL); const gd* vU = A(L.vU);
      const gd* dzL = A(L.dzL); const gd* dzU = A(L.dzU); const gd* dvL = A(L.dvL); const gd* dvU = A(L.dvU);
      const double ks = o.kappa_sigma;
      for (int q = c.lane; q < D.n; q += c.width) {
        tzL[q] = zL[q]; tzU[q] = zU[q];
        if (finite_(xL[q])) { const double z = zL[q] + a * dzL[q], v = safe_slack(xt[q] - xL[q], zL[q], xL[q], mu); tzL[q] = dmax(dmin(z, ks * mu / v), mu / (ks * v)); }
        if (finite_(xU[q])) { const double z = zU[q] + a * dzU[q], v = safe_slack(xU[q] - xt[q], zU[q], xU[q], mu); tzU[q] = dmax(dmin(z, ks * mu / v), mu / (ks * v)); }
      }
      for (int r = c.lane; r < D.md; r += c.width) {
        tyd[r] = yd[r] + a * dyd[r];
        { const double z = vL[r] + a * dvL[r], v = safe_slack(st[r] - dL[r], vL[r], dL[r], mu); tvL[r] = dmax(dmin(z, ks * mu / v), mu / (ks * v)); }
        tvU[r] = vU[r];
        if (finite_(dU[r])) { const double z = vU[r] + a * dvU[r], v = safe_slack(dU[r] - st[r], vU[r], dU[r], mu); tvU[r] = dmax(dmin(z, ks * mu / v), mu / (ks * v)); }
      }
      for (int r = c.lane; r < D.mc; r += c.width) tyc[r] = yc[r] + a * dyc[r];
      if (rs) {
        const gd* zR = A(L.zR); const gd* dzR = A(L.dzR);
        for (int j = c.lane; j < nR; j += c.width) {
          const double z = zR[j] + a * dzR[j], v = Rt[j];
          tzR[j] = dmax(dmin(z, ks * mu / v), mu / (ks * v));
        }
      }
      c.sync();
    }
    const int sat = check_trial(th, ph, gbd, 0.0, th_t, ph_t) ? 1 : 0;
    if (!sat) {
      const double e_cur = pd_error(gl, A(L.x), A(L.s), A(L.yc), A(L.yd), A(L.zL), A(L.zU), A(L.vL), A(L.vU),
                                    A(L.R), A(L.zR), A(L.c), A(L.d), mu);
      gd* gft = A(L.dzL); gd* glt = A(L.dzU);
      if (rs) eval_grad_f_rs(xt, gft);
      else eval_grad_f(xt, gft, sf);
      grad_lag_at(xt, tyc, tyd, gft, glt);
      const double e_tr = pd_error(glt, xt, st, tyc, tyd, tzL, tzU, tvL, tvU, Rt, tzR, A(L.ct), A(L.dt), mu, true);
      if (!(e_tr <= o.soft_resto_pderror_reduction_factor * e_cur)) return 0;
    }
    {  // AdjustVariableBounds for slacks the safe-slack rule corrected (current multipliers)
      gd* xL = A(L.xL); gd* xU = A(L.xU); gd* dL = A(L.dL); gd* dU = A(L.dU);
      const gd* zL = A(L.zL); const gd* zU = A(L.zU); const gd* vL = A(L.vL); const gd* vU = A(L.vU);
      for (int q = c.lane; q < D.n; q += c.width) {
        if (finite_(xL[q])) { const double v0 = xt[q] - xL[q], v = safe_slack(v0, zL[q], xL[q], mu); if (v != v0) xL[q] = xt[q] - v; }
        if (finite_(xU[q])) { const double v0 = xU[q] - xt[q], v = safe_slack(v0, zU[q], xU[q], mu); if (v != v0) xU[q] = xt[q] + v; }
      }
      for (int r = c.lane; r < D.md; r += c.width) {
        { const double v0 = st[r] - dL[r], v = safe_slack(v0, vL[r], dL[r], mu); if (v != v0) dL[r] = st[r] - v; }
        if (finite_(dU[r])) { const double v0 = dU[r] - st[r], v = safe_slack(v0, vU[r], dU[r], mu); if (v != v0) dU[r] = st[r] + v; }
      }
      c.sync();
    }
    copy_arr(A(L.x), xt, D.n); copy_arr(A(L.s), st, D.md);
    copy_arr(A(L.yc), tyc, D.mc); copy_arr(A(L.yd), tyd, D.md);
    copy_arr(A(L.zL), tzL, D.n); copy_arr(A(L.zU), tzU, D.n); copy_arr(A(L.vL), tvL, D.md); copy_arr(A(L.vU), tvU, D.md);
    if (rs) { copy_arr(A(L.R), Rt, nR); copy_arr(A(L.zR), tzR, nR); }
    copy_arr(A(L.c), A(L.ct), D.mc); copy_arr(A(L.d), A(L.dt), D.md);
    eval_grad_mode(A(L.x));
    return sat ? 2 : 1;
  }

  // n/p in closed form for the constraint residuals (cv) of row j (IpRestoIterateInitializer::solve_quadratic)
  HTP_HD HTP_FI static void np_closed_form(double cv, double mu_, double rho, double& nv, double& pv) {
    const double a = mu_ / (2.0 * rho) - 0.5 * cv;
    nv = a + sqrt(a * a + cv * mu_ / (2.0 * rho));
    pv = cv + nv;
  }
  // R (and zR = mu / R) from original residuals c (cres, mc) and d - s (dres, md)
  HTP_HD HTP_FI void np_init(const gd* cres, const gd* dv, const gd* s, double mu_) {
    gd* R = A(L.R); gd* zR = A(L.zR);
    const int mc = D.mc, md = D.md;
    const double rho = o.resto_penalty_parameter;
    for (int r = c.lane; r < mc; r += c.width) {
      double nv, pv;
      np_closed_form(cres[r], mu_, rho, nv, pv);
      R[r] = nv; R[mc + r] = pv; zR[r] = mu_ / nv; zR[mc + r] = mu_ / pv;
    }
    for (int r = c.lane; r < md; r += c.width) {
      double nv, pv;
      np_closed_form(dv[r] - s[r], mu_, rho, nv, pv);
      R[2 * mc + r] = nv; R[2 * mc + md + r] = pv; zR[2 * mc + r] = mu_ / nv; zR[2 * mc + md + r] = mu_ / pv;
    }
    c.sync();
  }

  // MinC_1NrmRestorationPhase: save the original iterate and state, set up the restoration problem
  // (RestoIterateInitializer) at the current point
  HTP_COLD HTP_HD void enter_resto(double th, double ph, double gbd) {
    gd* osv = A(L.osv);
    ls_save(osv);
    if (c.lane == 0) { osv[24] = th; osv[25] = ph; osv[26] = gbd; osv[27] = (double)nfilt; }
    {
      gd* of = A(L.ofilt);
      if (c.lane == 0)
        for (int k = 0; k < nfilt; ++k) { of[k] = f_th[k]; of[FMAX + k] = f_ph[k]; }
      c.sync();
    }
    gd* x = A(L.x); gd* s = A(L.s); gd* cc = A(L.c); gd* dd = A(L.d);
    copy_arr(A(L.ox), x, D.n); copy_arr(A(L.os), s, D.md);
    copy_arr(A(L.oyc), A(L.yc), D.mc); copy_arr(A(L.oyd), A(L.yd), D.md);
    copy_arr(A(L.ozL), A(L.zL), D.n); copy_arr(A(L.ozU), A(L.zU), D.n);
    copy_arr(A(L.ovL), A(L.vL), D.md); copy_arr(A(L.ovU), A(L.vU), D.md);
    double m = mu;
    for (int r = c.lane; r < D.mc; r += c.width) m = dmax(m, dabs(cc[r]));
    for (int r = c.lane; r < D.md; r += c.width) m = dmax(m, dabs(dd[r] - s[r]));
    const double mu_r = c.maxv(m);
    const double rho = o.resto_penalty_parameter;
    {
      gd* xR = A(L.xR); gd* dr = A(L.dr);
      for (int q = c.lane; q < D.n; q += c.width) { xR[q] = x[q]; dr[q] = 1.0 / dmax(1.0, dabs(x[q])); }
    }
    np_init(cc, dd, s, mu_r);
    {
      gd* zL = A(L.zL); gd* zU = A(L.zU); gd* vL = A(L.vL); gd* vU = A(L.vU);
      for (int q = c.lane; q < D.n; q += c.width) { zL[q] = dmin(rho, zL[q]); zU[q] = dmin(rho, zU[q]); }
      for (int r = c.lane; r < D.md; r += c.width) { vL[r] = dmin(rho, vL[r]); vU[r] = dmin(rho, vU[r]); }
      c.sync();
    }
    rs = true;
    mu = mu_r;
    tau = dmax(o.tau_min, 1.0 - mu);
    eta = o.resto_proximity_weight * sqrt(mu);
    {  // restoration constraint values c + n - p, d + n_d - p_d
      const gd* R = A(L.R);
      const int mc = D.mc, md = D.md;
      for (int r = c.lane; r < mc; r += c.width) cc[r] += R[r] - R[mc + r];
      for (int r = c.lane; r < md; r += c.width) dd[r] += R[2 * mc + r] - R[2 * mc + md + r];
      c.sync();
    }
    eval_grad_f_rs(x, A(L.gf));
    ls_multipliers();
    nfilt = 0;
    dw_last = 0.0;
    ls_reset();
    const double th0 = theta_of(cc, dd, s);
    theta_max = 1e4 * dmax(1.0, th0);
    theta_min = 1e-4 * dmax(1.0, th0);
    ++n_resto;
  }

  // RestoConvergenceCheck: original theta reduced by required_infeasibility_reduction and the point
  // acceptable to the original filter and to the original iterate
  HTP_HD HTP_FI bool resto_converged() {
    const gd* osv = A(L.osv);
    const gd* s = A(L.s);
    const double th_R = c.uniform(osv[24]), ph_R = c.uniform(osv[25]), mu_o = c.uniform(osv[10]);
    const int nf = (int)c.uniform(osv[27]);
    const double th_o = orig_theta_rs(A(L.c), A(L.d), s, A(L.R));
    if (th_o > o.required_infeasibility_reduction * th_R) return false;
    const double ph_o = barrier(A(L.x), s, A(L.R), mu_o, false);
    const gd* of = A(L.ofilt);
    for (int k = 0; k < nf; ++k)
      if (!(th_o < of[k] || ph_o < of[FMAX + k])) return false;
    return acc_to_iterate(th_R, ph_R, ph_o, th_o, true);
  }

  // back to the original problem with x, s of the restoration phase: bound multipliers take one
  // complementarity Newton step for the whole primal change (all reset to 1 if > threshold), y = 0
  HTP_COLD HTP_HD void leave_resto() {
    rs = false;
    const gd* osv = A(L.osv);
    ls_load(osv);
    nfilt = (int)c.uniform(osv[27]);
    {
      const gd* of = A(L.ofilt);
      if (c.lane == 0)
        for (int k = 0; k < nfilt; ++k) { f_th[k] = of[k]; f_ph[k] = of[FMAX + k]; }
      c.sync();
    }
    gd* x = A(L.x); gd* s = A(L.s);
    eval_cons(x, A(L.c), A(L.d));
    const gd* xL = A(L.xL); const gd* xU = A(L.xU); const gd* dL = A(L.dL); const gd* dU = A(L.dU);
    const gd* ox = A(L.ox); const gd* os = A(L.os);
    const gd* ozL = A(L.ozL); const gd* ozU = A(L.ozU); const gd* ovL = A(L.ovL); const gd* ovU = A(L.ovU);
    gd* dzL = A(L.dzL); gd* dzU = A(L.dzU); gd* dvL = A(L.dvL); gd* dvU = A(L.dvU);
    double a = 1.0;
    auto step = [&](double z, double cs, double ts) { return (mu + z * (cs - ts)) / ts - z; };
    for (int q = c.lane; q < D.n; q += c.width) {
      double t = 0.0, u = 0.0;
      if (finite_(xL[q])) { t = step(ozL[q], ox[q] - xL[q], x[q] - xL[q]); if (t < 0) a = dmin(a, -tau * ozL[q] / t); }
      if (finite_(xU[q])) { u = step(ozU[q], xU[q] - ox[q], xU[q] - x[q]); if (u < 0) a = dmin(a, -tau * ozU[q] / u); }
      dzL[q] = t; dzU[q] = u;
    }
    for (int r = c.lane; r < D.md; r += c.width) {
      double t = step(ovL[r], os[r] - dL[r], s[r] - dL[r]), u = 0.0;
      if (t < 0) a = dmin(a, -tau * ovL[r] / t);
      if (finite_(dU[r])) { u = step(ovU[r], dU[r] - os[r], dU[r] - s[r]); if (u < 0) a = dmin(a, -tau * ovU[r] / u); }
      dvL[r] = t; dvU[r] = u;
    }
    c.sync();
    a = c.minv(a);
    gd* zL = A(L.zL); gd* zU = A(L.zU); gd* vL = A(L.vL); gd* vU = A(L.vU);
    double bmax = 0.0;
    for (int q = c.lane; q < D.n; q += c.width) {
      zL[q] = ozL[q] + a * dzL[q]; zU[q] = ozU[q] + a * dzU[q];
      bmax = dmax(bmax, dmax(dabs(zL[q]), dabs(zU[q])));
    }
    for (int r = c.lane; r < D.md; r += c.width) {
      vL[r] = ovL[r] + a * dvL[r]; vU[r] = ovU[r] + a * dvU[r];
      bmax = dmax(bmax, dmax(dabs(vL[r]), dabs(vU[r])));
    }
    c.sync();
    if (c.maxv(bmax) > o.bound_mult_reset_threshold) {
      for (int q = c.lane; q < D.n; q += c.width) { zL[q] = finite_(xL[q]) ? 1.0 : 0.0; zU[q] = finite_(xU[q]) ? 1.0 : 0.0; }
      for (int r = c.lane; r < D.md; r += c.width) { vL[r] = 1.0; vU[r] = finite_(dU[r]) ? 1.0 : 0.0; }
    }
    gd* yc = A(L.yc); gd* yd = A(L.yd);
    for (int r = c.lane; r < D.mc; r += c.width) yc[r] = 0.0;
    for (int r = c.lane; r < D.md; r += c.width) yd[r] = 0.0;
    c.sync();
    eval_grad_f(x, A(L.gf), sf);
  }

  // RestoRestorationPhase: n, p reset in closed form at the current x (restoration mu), zR = mu / R
  HTP_COLD HTP_HD void resto_resto() {
    gd* ct = A(L.ct); gd* dtv = A(L.dt);
    eval_cons(A(L.x), ct, dtv);
    np_init(ct, dtv, A(L.s), mu);
    const gd* R = A(L.R);
    gd* cc = A(L.c); gd* dd = A(L.d);
    const int mc = D.mc, md = D.md;
    for (int r = c.lane; r < mc; r += c.width) cc[r] = ct[r] + R[r] - R[mc + r];
    for (int r = c.lane; r < md; r += c.width) dd[r] = dtv[r] + R[2 * mc + r] - R[2 * mc + md + r];
    c.sync();
  }

  HTP_HD HTP_FI void iterate(Result& res) {
    gd* x = A(L.x); gd* s = A(L.s);
    gd* cc = A(L.c); gd* dd = A(L.d);
    // phi / theta of the current point are carried over from the accepted trial point
    // (bitwise identical: x_new is computed by the same expression as x_trial)
    double phi_cache = 0.0, mu_cache = -1.0, theta_cache = -1.0;
    int status = ST_MAXITER, it = 0;
    bool rs_first = false;
    double nlp_err = 0.0;
    gd* gl = A(L.rx);
    gd* dx = A(L.dx); gd* ds = A(L.ds); gd* dyc = A(L.dyc); gd* dyd = A(L.dyd); gd* dR = A(L.dR);
    const long long t_start = c.wall();
    const double wall_limit = o.max_cpu_time > 0.0 ? o.max_cpu_time * o.wall_rate : -1.0;
    for (;;) {
      long long tq0 = c.clock();
      grad_lag_into(gl);
      Err emu;  // errors at the current mu, from the same sweeps (the first barrier test below)
      Err e0 = errors(gl, 0.0, mu, &emu);
      HTP_TRACE("[trace] it %d%s err dual=%.17g comp=%.17g prim=%.17g mu=%.17g\n", it, rs ? " R" : "", e0.dual, e0.comp, e0.prim_nlp, mu);
      nlp_err = dmax(dmax(e0.dual / e0.s_d, e0.prim_nlp), e0.comp / e0.s_c);
      const double uv = unscaled_viol();
      const double sfm = rs ? 1.0 : sf;
      const bool optimal = nlp_err <= o.tol && e0.dual / sfm <= o.dual_inf_tol && uv <= o.constr_viol_tol &&
                           e0.comp / sfm <= o.compl_inf_tol;
      const bool acc_lvl = nlp_err <= o.acceptable_tol && e0.dual / sfm <= o.acceptable_dual_inf_tol &&
                           uv <= o.acceptable_constr_viol_tol && e0.comp / sfm <= o.acceptable_compl_inf_tol;
      if (rs) {
        if (!rs_first && resto_converged()) {
          leave_resto();
          mu_cache = -1.0;
          theta_cache = -1.0;
          continue;  // the original problem resumes with this iteration number
        }
        if (!rs_first && (optimal || (acc_lvl && ls_.acc_count + 1 >= o.acceptable_iter))) {
          // RestoConvergenceCheck: max-norm primal infeasibility of the original problem <= 1e2 tol ->
          // "Restoration_Failed" (converged to a feasible point the filter rejects), else locally infeasible
          const double ot = orig_inf_max_rs(cc, dd, s, A(L.R));
          status = ot <= 1e2 * o.tol ? ST_RESTORATION : ST_INFEASIBLE;
          if (have_acc) { copy_arr(x, A(L.ax), D.n); status = ST_ACCEPTABLE; }
          break;
        }
        ls_.acc_count = acc_lvl ? ls_.acc_count + 1 : 0;
      } else {
        if (optimal) { status = ST_SUCCESS; break; }
        if (acc_lvl) {
          if (++ls_.acc_count >= o.acceptable_iter) { status = ST_ACCEPTABLE; break; }
        } else {
          ls_.acc_count = 0;
        }
      }
      if (it >= o.max_iter) { status = ST_MAXITER; break; }
      // max_cpu_time after the convergence / acceptable / iteration-limit tests, in IPOPT's
      // OptimalityErrorConvergenceCheck order (and after RestoConvergenceCheck in the restoration phase)
      if (wall_limit > 0.0 && (double)(c.wall() - t_start) > wall_limit) { status = ST_CPUTIME; break; }
      rs_first = false;
      // monotone barrier update (a tiny step forces a decrease)
      bool stop_tiny = false;
      for (bool first = true;; first = false) {
        Err eb = first ? emu : errors(gl, mu);
        const double berr = dmax(dmax(eb.dual / eb.s_d, eb.prim_b), eb.comp / eb.s_c);
        if (berr > o.kappa_eps * mu && !ls_.tiny_flag) break;
        const double nm = dmax(o.tol / 10.0, dmin(o.kappa_mu * mu, sm::pow(mu, o.theta_mu)));
        if (nm == mu) { if (ls_.tiny_flag) stop_tiny = true; break; }
        mu = nm;
        tau = dmax(o.tau_min, 1.0 - mu);
        nfilt = 0;
        ls_.tiny_flag = 0;
        if (rs) {  // the restoration objective depends on mu (eta = sqrt(mu))
          eta = o.resto_proximity_weight * sqrt(mu);
          eval_grad_f_rs(x, A(L.gf));
          grad_lag_into(gl);
        }
      }
      if (stop_tiny) { status = ST_TINYSTEP; break; }
      ls_.tiny_flag = 0;
      cyc[5] += c.clock() - tq0;
      // Newton step: rx (in xt), rs, rc, rd[, rRx]; barrier gradient in sx, ss
      build_newton_rhs(gl);
      double dw = 0.0, dc = 0.0;
      fuse_rhs = HTP_FUSE_RHS && !PT && !rs;   // restoration folds its n/p rows into the rhs per trial: unfused
      const bool have_step = factor_ic(dw, dc);
      const bool rhs_done = fuse_rhs;
      fuse_rhs = false;
      if (!have_step) {
        ls_.fallback = 1;
      } else {
        if (dw > 0.0) dw_last = dw;
        HTP_TRACE("[trace] factored dw=%g\n", dw);
        kkt_solve(false, dw, dc, A(L.xt), A(L.rs), A(L.rc), A(L.rd), dx, ds, dyc, dyd, A(L.rRx), dR, rhs_done);
      }
      // ---- line search (IpBacktrackingLineSearch::FindAcceptableTrialPoint)
      long long tls = c.clock();
      if (!rs && acc_lvl) { copy_arr(A(L.ax), x, D.n); have_acc = true; }
      if (ls_.last_mu != mu) { ls_.in_wd = 0; ls_.wd_short = 0; ls_.last_mu = mu; }
      double phi = (mu_cache == mu) ? phi_cache : barrier(x, s, A(L.R), mu, rs);
      double theta = (theta_cache >= 0.0) ? theta_cache : theta_of(cc, dd, s);
      bool goto_resto = ls_.fallback != 0;
      ls_.fallback = 0;
      double gbd = goto_resto ? 0.0 : newton_gbd(dx, ds, dR);
      // A step with a NaN / infinite entry (a KKT system solved beyond floating-point range): IPOPT cuts back on
      // every trial-point evaluation error and so never takes such a step -- its line search fails and the
      // restoration phase is called, which is where this goes directly.
      if (HTP_NAN_GUARD && !goto_resto && !(dabs(gbd) < HTP_INF)) { goto_resto = true; gbd = 0.0; }
      copy_arr(A(L.sx), A(L.xt), D.n);  // keep the Newton rhs (x part) for second-order corrections
      double rth = theta, rph = phi, rgbd = gbd;
      if (ls_.in_wd) { rth = ls_.wd_th; rph = ls_.wd_ph; rgbd = ls_.wd_gbd; }
      bool accept = false;
      int n_steps = 0;
      double a_primal = 0.0, a_test = 0.0, ph_t = 0.0, th_t = 0.0;
      double cdw = dw, cdc = dc;
      bool tiny = !goto_resto && detect_tiny_step(dx, ds, dyc, dyd, dR);
      if (ls_.in_wd && (goto_resto || tiny)) {
        stop_watchdog();
        copy_arr(A(L.sx), A(L.xt), D.n);
        theta = rth; phi = rph; cdw = ls_.wd_dw; cdc = ls_.wd_dc;
        goto_resto = tiny = false;
      }
      if (o.watchdog_shortened_iter_trigger > 0 && !ls_.in_wd && !goto_resto && !tiny && !ls_.in_soft &&
          ls_.wd_short >= o.watchdog_shortened_iter_trigger)
        start_watchdog(theta, phi, gbd, dw, dc);
      if (tiny) {
        a_primal = frac_primal(dx, ds, dR);
        set_trial(a_primal, dx, ds, dR);
        trial_values(A(L.xt), A(L.st), A(L.Rt), th_t, ph_t);
        if (ls_.tiny_last) ls_.tiny_flag = 1;
        ls_.tiny_last = 1;
        accept = true;
      } else {
        ls_.tiny_last = 0;
      }
      int soft = 0;
      if (!goto_resto && !tiny) {
        if (ls_.in_soft) {
          if (++ls_.soft_cnt > o.max_soft_resto_iters) {
            accept = false;
          } else {
            soft = try_soft_resto_step(rth, rph, rgbd, gl);
            if (soft == 2) { ls_.in_soft = 0; ls_.soft_cnt = 0; }
          }
        } else {
          bool skip = false;
          for (;;) {
            accept = backtrack(rth, rph, rgbd, skip, n_steps, a_primal, a_test, ph_t, th_t, cdw, cdc);
            if (ls_.in_wd) {
              if (accept) { ls_.in_wd = 0; break; }
              if (++ls_.wd_trial > o.watchdog_trial_iter_max) {
                stop_watchdog();
                copy_arr(A(L.sx), A(L.xt), D.n);
                rth = ls_.wd_th; rph = ls_.wd_ph; rgbd = ls_.wd_gbd;
                theta = rth; phi = rph; cdw = ls_.wd_dw; cdc = ls_.wd_dc;
                skip = true;
                continue;
              }
              accept = true;  // the watchdog takes the full step unchecked
              break;
            }
            break;
          }
        }
      }
      if (!soft && !accept) {
        if (!ls_.in_soft && o.soft_resto_pderror_reduction_factor > 0.0 && !goto_resto) {
          filter_add(rth, rph);  // PrepareRestoPhaseStart
          soft = try_soft_resto_step(rth, rph, rgbd, gl);
          if (soft == 1) ls_.in_soft = 1;
        } else if (!ls_.in_soft) {
          filter_add(rth, rph);
        }
        if (!soft) {
          cyc[6] += c.clock() - tls;
          if (theta <= 1e-2 * o.tol) {  // restoration phase called at an almost feasible point
            status = have_acc ? ST_ACCEPTABLE : ST_RESTORATION;
            if (have_acc) copy_arr(x, A(L.ax), D.n);
            break;
          }
          ls_.in_soft = 0; ls_.soft_cnt = 0; ls_.wd_short = 0; ls_.cnt_filter_rej = 0;
          if (rs) {
            resto_resto();
          } else {
            enter_resto(rth, rph, rgbd);
            rs_first = true;
          }
          mu_cache = -1.0;
          theta_cache = -1.0;
          ++it;
          continue;
        }
      }
      cyc[6] += c.clock() - tls;
      if (soft) {
        mu_cache = -1.0;
        theta_cache = -1.0;
        ++it;
        continue;
      }
      HTP_TRACE("[trace]   acc it=%d a=%.17g th_t=%.17g ph_t=%.17g ref_th=%.17g ref_ph=%.17g n_steps=%d\n", it, a_primal, th_t, ph_t, rth, rph, n_steps);
      long long tup = c.clock();
      const double a_dual = dual_steps(dx, ds, dR);
      accept_step(a_primal, a_dual, dx, ds, dyc, dyd, dR);
      if (n_steps == 0) ls_.wd_short = 0;
      if (n_steps > 0) ++ls_.wd_short;
      phi_cache = ph_t;
      mu_cache = mu;
      theta_cache = th_t;
      eval_grad_mode(x);
      cyc[7] += c.clock() - tup;
      ++it;
    }
    // honor_original_bounds: project into the unrelaxed bounds
    project_original_bounds();
    const double fobj = eval_f(x);
    if (c.lane == 0) {
      res.status = status;
      res.iters = it;
      res.n_factor = n_factor;
      res.n_resto = n_resto;
      res.objective = fobj;
      res.final_mu = mu;
      res.nlp_error = nlp_err;
      res.sf = sf;
    }
    c.sync();
  }

  // recompute original (unrelaxed) bounds and clip x
  HTP_HD HTP_FI void project_original_bounds() {
    gd* x = A(L.x);
    const double vmax = dabs(par(P_MAXV)), smax = dabs(par(P_MAXSTEER));
    const double amax = dabs(par(P_MAXACC)), wmax = dabs(par(P_MAXSR));
    const double twopi = 2.0 * M_PI;
    HTP_UNROLL
    for (int q = c.lane; q < D.n; q += c.width) {
      double lo = -HTP_INF, hi = HTP_INF;
      if (q < D.oU) {
        const int k = q % NS;
        if (k == 0) { lo = par(P_XLO); hi = par(P_XHI); }
        if (k == 1) { lo = par(P_YLO); hi = par(P_YHI); }
        if (k == 2) { lo = -vmax; hi = vmax; }
        if (k == 3) { lo = -twopi; hi = twopi; }
        if (k == 4) { lo = -smax; hi = smax; }
      } else if (q < D.oMU) {
        if ((q - D.oU) % 2 == 0) { lo = -amax; hi = amax; } else { lo = -wmax; hi = wmax; }
      } else if (q < D.oTAU) {
        lo = 0.0;
        if (PT) hi = 100000.0;
      } else if (q < D.oS) {
        lo = 0.05 / par(P_DT); hi = 1.0;
      }
      if (finite_(lo)) x[q] = dmax(x[q], lo);
      if (finite_(hi)) x[q] = dmin(x[q], hi);
    }
    c.sync();
  }
};

}  // namespace htp
