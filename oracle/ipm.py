"""Oracle: restatement of the IPOPT algorithm that R/obca_py/optimizer.py:489-507
runs through CasADi (`ca.nlpsol("solver", "ipopt", ...)`).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The algorithm lives in a third-party dependency that is absent here:
IPOPT (CasADi >= 3.6.3 bundles IPOPT 3.14.x, R/requirements.txt:9) with MUMPS.
This file restates its *published* algorithm -- A. Waechter, L. T. Biegler,
"On the implementation of an interior-point filter line-search algorithm for
large-scale nonlinear programming", Math. Prog. 106 (2006) -- and the IPOPT
3.14 defaults as CasADi calls it (optimizer.py:481-488 only sets
print_level/sb/max_cpu_time):

  * gradient-based NLP scaling (max gradient 100) at the user x0
  * bound_relax_factor 1e-8; bound_push = bound_frac = 1e-2 (x and slacks)
  * bound multipliers 1; least-squares equality/inequality multipliers,
    discarded if |y|_inf > 1e3
  * monotone Fiacco-McCormick barrier: mu0 = 0.1, kappa_eps 10, kappa_mu 0.2,
    theta_mu 1.5, mu floor tol/10, tau = max(0.99, 1-mu), fast decrease allowed
  * barrier objective with kappa_d = 1e-5 damping of one-sided bounds
  * primal-dual Newton step on the augmented system, inertia correction
    (delta_w: 1e-4 first, x1/3 decrease, x100 first / x8 increase;
     delta_c = 1e-8 mu^0.25 on singularity)
  * filter line search (gamma_theta 1e-5, gamma_phi 1e-8, delta 1, s_theta
    1.1, s_phi 2.3, eta_phi 1e-8, alpha_min_frac 0.05, theta_max/min
    1e4/1e-4 * max(1,theta0), obj_max_inc 5); the first trial step is always
    tested; up to 4 second-order corrections (kappa_soc 0.99); y stepped with
    alpha_primal; filter reset heuristic (max_filter_resets 5,
    filter_reset_trigger 5)
  * watchdog (watchdog_shortened_iter_trigger 10, watchdog_trial_iter_max 3)
  * tiny-step heuristic (tiny_step_tol 10 eps, tiny_step_y_tol 1e-2)
  * soft restoration phase (soft_resto_pderror_reduction_factor 0.9999,
    max_soft_resto_iters 10)
  * feasibility restoration phase (RestoIpoptNLP / MinC_1NrmRestorationPhase):
    min rho*sum(n+p) + eta(mu)/2 |D_R (x - x_R)|^2 s.t. c(x) + n_c - p_c = 0,
    d_L <= d(x) + n_d - p_d <= d_U, rho = 1000, eta = sqrt(mu),
    D_R = 1/max(1, |x_R|), mu_R = max(mu, |c|_inf, |d-s|_inf), n/p in closed
    form, bound multipliers min(rho, z), least-squares multipliers; it ends
    when the original theta drops below 0.9 theta_R and the point is
    acceptable to the original filter and iterate; back in the original
    problem the bound multipliers take one complementarity Newton step
    (reset to 1 if > 1000) and y = 0 (constr_mult_reset_threshold 0); inside
    the restoration phase a failed line search resets n, p in closed form
  * kappa_Sigma = 1e10 bound-multiplier safeguard
  * termination: scaled NLP error <= 1e-8 and unscaled dual_inf <= 1,
    constr_viol <= 1e-4, compl <= 1e-4; "acceptable" after 15 iterations at 1e-6;
    a failed restoration returns the last acceptable iterate if there is one
  * final x projected to the original bounds (honor_original_bounds)

The heuristics were restated from the IPOPT 3.14 sources as published
(IpBacktrackingLineSearch.cpp, IpFilterLSAcceptor.cpp, IpRestoMinC_1Nrm.cpp,
IpRestoIterateInitializer.cpp, IpRestoConvergenceCheck.cpp); no IPOPT
binary exists in this container, so their exact trajectories are parity
unpinned beyond the notebook's CasADi pin (tests/test_notebook_pins.py).

The KKT systems are solved with a dense Bunch-Kaufman LDL^T (scipy.linalg.ldl)
whose block-diagonal factor gives the exact inertia MUMPS reports, or with
oracle/structured.py.  The restoration problem's n/p variables are
eliminated onto a per-row diagonal of the constraint block (-(dc + e_r)),
which both KKT back ends take as a vector dc.
"""
import math

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp

from oracle import libm

EPS = np.finfo(float).eps

OPTS = dict(
    tol=1e-8, dual_inf_tol=1.0, constr_viol_tol=1e-4, compl_inf_tol=1e-4,
    acceptable_tol=1e-6, acceptable_iter=15, acceptable_constr_viol_tol=1e-2,
    acceptable_compl_inf_tol=1e-2, acceptable_dual_inf_tol=1e10,
    max_iter=3000, bound_relax_factor=1e-8, scaling_max_gradient=100.0, scaling_min_value=1e-8,
    bound_push=1e-2, bound_frac=1e-2, bound_mult_init_val=1.0, constr_mult_init_max=1e3,
    mu_init=0.1, kappa_eps=10.0, kappa_mu=0.2, theta_mu=1.5, tau_min=0.99, kappa_sigma=1e10,
    kappa_d=1e-5, s_max=100.0, gamma_theta=1e-5, gamma_phi=1e-8, delta=1.0, s_theta=1.1,
    s_phi=2.3, eta_phi=1e-8, alpha_min_frac=0.05, max_soc=4, kappa_soc=0.99, obj_max_inc=5.0,
    dw0=1e-4, dw_min=1e-20, dw_max=1e40, kw_minus=1.0 / 3.0, kw_plus=8.0, kw_plus_bar=100.0,
    dc_bar=1e-8, kappa_c=0.25,
    max_filter_resets=5, filter_reset_trigger=5,
    watchdog_shortened_iter_trigger=10, watchdog_trial_iter_max=3,
    tiny_step_tol=10.0 * EPS, tiny_step_y_tol=1e-2,
    soft_resto_pderror_reduction_factor=0.9999, max_soft_resto_iters=10,
    resto_penalty_parameter=1000.0, resto_proximity_weight=1.0, required_infeasibility_reduction=0.9,
    bound_mult_reset_threshold=1000.0, constr_mult_reset_threshold=0.0,
)

# solver statuses (include/htp.h HTP_STATUS_*)
SUCCESS, ACCEPTABLE, MAXITER, RESTO_FAILED, STEP_FAILED, BAD_INPUT, CPUTIME, INFEASIBLE, TINY_STEP = range(9)
STATUS = {SUCCESS: "Solve_Succeeded", ACCEPTABLE: "Solved_To_Acceptable_Level",
          MAXITER: "Maximum_Iterations_Exceeded", RESTO_FAILED: "Restoration_Failed",
          STEP_FAILED: "Error_In_Step_Computation", BAD_INPUT: "Invalid_Problem_Definition",
          CPUTIME: "Maximum_CpuTime_Exceeded", INFEASIBLE: "Infeasible_Problem_Detected",
          TINY_STEP: "Search_Direction_Becomes_Too_Small"}


def compare_le(lhs, rhs, basval):
    """IPOPT's Compare_le: lhs - rhs <= 10*eps*|basval|."""
    return lhs - rhs <= 10.0 * EPS * abs(basval)


def _inertia_of_ldl(d):
    pos = neg = zer = 0
    i, dim = 0, d.shape[0]
    while i < dim:
        if i + 1 < dim and d[i + 1, i] != 0.0:
            ev = np.linalg.eigvalsh(d[i:i + 2, i:i + 2])
            i += 2
        else:
            ev = [d[i, i]]
            i += 1
        for e in ev:
            pos += e > 0
            neg += e < 0
            zer += e == 0
    return int(pos), int(neg), int(zer)


class DenseKKT:
    """[W+Sx+dw, 0, Jc', Jd'; 0, Ss+dw, 0, -I; Jc, 0, -dc, 0; Jd, -I, 0, -dc];
    dc is a scalar or a per-row vector (restoration rows)."""

    def factor(self, Wm, Sx, Ss, Jc, Jd, dw, dc):
        Wm, Jc, Jd = (a.toarray() if hasattr(a, "toarray") else a for a in (Wm, Jc, Jd))
        n, ns, mc = Wm.shape[0], Ss.size, Jc.shape[0]
        dim = n + ns + mc + ns
        K = np.zeros((dim, dim))
        K[:n, :n] = Wm + np.diag(Sx + dw)
        K[n:n + ns, n:n + ns] = np.diag(Ss + dw)
        K[n + ns:n + ns + mc, :n] = Jc
        K[n + ns + mc:, :n] = Jd
        K[n + ns + mc:, n:n + ns] = -np.eye(ns)
        K[n + ns:, n + ns:] -= np.diag(np.broadcast_to(np.asarray(dc, dtype=float), (mc + ns,)))
        K = np.tril(K) + np.tril(K, -1).T
        lu, d, perm = sla.ldl(K, lower=True)
        self.fac = (lu, d, perm)
        self.dims = (n, ns, mc)
        return _inertia_of_ldl(d)

    def solve(self, rx, rs, rc, rd):
        lu, d, perm = self.fac
        b = np.concatenate([rx, rs, rc, rd])
        T = lu[perm]
        u = sla.solve_triangular(T, b[perm], lower=True, unit_diagonal=True)
        w = np.linalg.solve(d, u) if d.shape[0] < 4000 else sla.solve(d, u, assume_a="sym")
        v = sla.solve_triangular(T.T, w, lower=False, unit_diagonal=True)
        out = np.empty_like(v)
        out[perm] = v
        n, ns, mc = self.dims
        return out[:n], out[n:n + ns], out[n + ns:n + ns + mc], out[n + ns + mc:]


# ---------------------------------------------------------------------------
# The problems the interior-point loop iterates on (IPOPT's IpoptNLP objects)
# ---------------------------------------------------------------------------
class OrigProblem:
    """OrigIpoptNLP: the user NLP with gradient-based scaling and relaxed bounds."""

    is_resto = False

    def __init__(self, nlp, o, kkt):
        self.nlp, self.o, self.kkt = nlp, o, kkt
        gL, gU = nlp.g_L, nlp.g_U
        self.E = np.where(gL == gU)[0]
        self.I = np.where(gL != gU)[0]
        x0 = nlp.x0
        gf = nlp.grad_f(x0)
        mg = np.max(np.abs(gf)) if gf.size else 0.0
        sm = o["scaling_max_gradient"]
        self.sf = max(o["scaling_min_value"], sm / mg) if mg > sm else 1.0
        rowmax = np.asarray(abs(nlp.jac(x0).tocsr()).max(axis=1).todense()).ravel()
        sc = np.ones(nlp.m)
        big = rowmax > sm
        sc[big] = np.maximum(o["scaling_min_value"], sm / rowmax[big])
        self.sc = sc
        rf = o["bound_relax_factor"]
        xL, xU = nlp.x_L.copy(), nlp.x_U.copy()
        fl, fu = np.isfinite(xL), np.isfinite(xU)
        xL[fl] -= rf * np.maximum(1.0, np.abs(xL[fl]))
        xU[fu] += rf * np.maximum(1.0, np.abs(xU[fu]))
        self.xL, self.xU, self.hxL, self.hxU = xL, xU, fl, fu
        dL, dU = gL[self.I].copy(), gU[self.I].copy()
        fdl, fdu = np.isfinite(dL), np.isfinite(dU)
        dL[fdl] -= rf * np.maximum(1.0, np.abs(dL[fdl]))
        dU[fdu] += rf * np.maximum(1.0, np.abs(dU[fdu]))
        sI = sc[self.I]
        self.dL = np.where(fdl, dL * sI, -np.inf)
        self.dU = np.where(fdu, dU * sI, np.inf)
        self.hdL, self.hdU = fdl, fdu
        self.cE = gL[self.E]
        self.n, self.mc, self.md = nlp.n, self.E.size, self.I.size

    def f(self, x, mu):
        return self.sf * self.nlp.f(x)

    def grad_f(self, x, mu):
        return self.sf * self.nlp.grad_f(x)

    def cd(self, x):
        g = self.nlp.cons(x)
        return self.sc[self.E] * (g[self.E] - self.cE), self.sc[self.I] * g[self.I]

    def jac(self, x):
        J = (sp.diags(self.sc) @ self.nlp.jac(x)).tocsr()
        return J[self.E], J[self.I]

    def hess(self, x, yc, yd, mu, obj_factor=1.0):
        y = np.zeros(self.nlp.m)
        y[self.E] = yc * self.sc[self.E]
        y[self.I] = yd * self.sc[self.I]
        return self.nlp.hess(x, y, self.sf * obj_factor)

    def unscaled_viol(self, x, c=None, d=None):
        nlp = self.nlp
        g = nlp.cons(x)
        v = np.abs(g[self.E] - self.cE)
        gl, gu = nlp.g_L[self.I], nlp.g_U[self.I]
        w = np.maximum(0.0, np.maximum(gl - g[self.I], g[self.I] - gu))
        return max(np.max(v, initial=0.0), np.max(w, initial=0.0))

    def factor(self, W, Sx, Ss, Jc, Jd, dw, dc):
        return self.kkt.factor(W, Sx, Ss, Jc, Jd, dw, dc)

    def solve(self, rx, rs, rc, rd):
        return self.kkt.solve(rx, rs, rc, rd)


class RestoProblem:
    """RestoIpoptNLP over the (scaled) original problem: variables
    [x, n_c, p_c, n_d, p_d]; no further scaling or bound relaxation."""

    is_resto = True

    def __init__(self, orig, x_ref, o):
        self.orig, self.o = orig, o
        n, mc, md = orig.n, orig.mc, orig.md
        self.nx, self.mc, self.md = n, mc, md
        self.n = n + 2 * mc + 2 * md
        self.rho = o["resto_penalty_parameter"]
        self.x_ref = x_ref.copy()
        self.dr = 1.0 / np.maximum(1.0, np.abs(x_ref))
        z = np.zeros(2 * mc + 2 * md)
        self.xL = np.concatenate([orig.xL, z])
        self.xU = np.concatenate([orig.xU, z + np.inf])
        self.hxL = np.concatenate([orig.hxL, np.ones(z.size, bool)])
        self.hxU = np.concatenate([orig.hxU, np.zeros(z.size, bool)])
        self.dL, self.dU, self.hdL, self.hdU = orig.dL, orig.dU, orig.hdL, orig.hdU
        self.sf = 1.0

    def parts(self, X):
        n, mc, md = self.nx, self.mc, self.md
        return X[:n], X[n:n + mc], X[n + mc:n + 2 * mc], X[n + 2 * mc:n + 2 * mc + md], X[n + 2 * mc + md:]

    def eta(self, mu):
        return self.o["resto_proximity_weight"] * math.sqrt(mu)

    def f(self, X, mu):
        x, nc, pc, nd, pd = self.parts(X)
        t = self.dr * (x - self.x_ref)
        return self.rho * (nc.sum() + pc.sum() + nd.sum() + pd.sum()) + 0.5 * self.eta(mu) * (t @ t)

    def grad_f(self, X, mu):
        g = np.full(self.n, self.rho)
        x = X[:self.nx]
        g[:self.nx] = self.eta(mu) * self.dr * self.dr * (x - self.x_ref)
        return g

    def cd(self, X):
        x, nc, pc, nd, pd = self.parts(X)
        c, d = self.orig.cd(x)
        return c + nc - pc, d + nd - pd

    def jac(self, X):
        Jc, Jd = self.orig.jac(X[:self.nx])
        mc, md = self.mc, self.md
        Ic, Id = sp.identity(mc, format="csr"), sp.identity(md, format="csr")
        Zc, Zd = sp.csr_matrix((mc, md)), sp.csr_matrix((md, mc))
        return (sp.hstack([Jc, Ic, -Ic, Zc, Zc], format="csr"), sp.hstack([Jd, Zd, Zd, Id, -Id], format="csr"))

    def hess(self, X, yc, yd, mu, obj_factor=1.0):
        Wx = self.orig.hess(X[:self.nx], yc, yd, mu, obj_factor=0.0) + \
            sp.diags(obj_factor * self.eta(mu) * self.dr * self.dr)
        extra = self.n - self.nx
        return sp.block_diag([Wx, sp.csr_matrix((extra, extra))], format="csr")

    def unscaled_viol(self, X, c=None, d=None):
        if c is None:
            c, d = self.cd(X)
        w = np.maximum(0.0, np.maximum(np.where(self.hdL, self.dL - d, 0.0), np.where(self.hdU, d - self.dU, 0.0)))
        return max(np.max(np.abs(c), initial=0.0), np.max(w, initial=0.0))

    # n/p eliminated: (S_n + dw) dn + dy = r_n, (S_p + dw) dp - dy = r_p
    #   -> J dx - (dc + 1/(S_n+dw) + 1/(S_p+dw)) dy = r_c - r_n/(S_n+dw) + r_p/(S_p+dw)
    def factor(self, W, Sx, Ss, Jc, Jd, dw, dc):
        n, mc, md = self.nx, self.mc, self.md
        Wx = W.tocsr()[:n, :n]
        sn_c, sp_c = Sx[n:n + mc] + dw, Sx[n + mc:n + 2 * mc] + dw
        sn_d, sp_d = Sx[n + 2 * mc:n + 2 * mc + md] + dw, Sx[n + 2 * mc + md:] + dw
        self._s = (sn_c, sp_c, sn_d, sp_d)
        e = np.concatenate([1.0 / sn_c + 1.0 / sp_c, 1.0 / sn_d + 1.0 / sp_d])
        pos, neg, zer = self.orig.factor(Wx, Sx[:n], Ss, Jc[:, :n], Jd[:, :n], dw, dc + e)
        extra = np.concatenate(self._s)
        return pos + int(np.sum(extra > 0)), neg + int(np.sum(extra < 0)), zer + int(np.sum(extra == 0))

    def solve(self, rx, rs, rc, rd):
        n, mc, md = self.nx, self.mc, self.md
        sn_c, sp_c, sn_d, sp_d = self._s
        r_nc, r_pc = rx[n:n + mc], rx[n + mc:n + 2 * mc]
        r_nd, r_pd = rx[n + 2 * mc:n + 2 * mc + md], rx[n + 2 * mc + md:]
        dx, ds, dyc, dyd = self.orig.solve(rx[:n], rs, rc - r_nc / sn_c + r_pc / sp_c, rd - r_nd / sn_d + r_pd / sp_d)
        out = np.concatenate([dx, (r_nc - dyc) / sn_c, (r_pc + dyc) / sp_c, (r_nd - dyd) / sn_d, (r_pd + dyd) / sp_d])
        return out, ds, dyc, dyd


def _solve_quadratic(a, b):
    """IpRestoIterateInitializer's solve_quadratic: n = a + sqrt(a^2 + b)."""
    return a + np.sqrt(a * a + b)


# ---------------------------------------------------------------------------
class _Iterate:
    __slots__ = ("x", "s", "yc", "yd", "zL", "zU", "vL", "vU")

    def __init__(self, **kw):
        for k in self.__slots__:
            setattr(self, k, kw.get(k))

    def copy(self):
        return _Iterate(**{k: (None if getattr(self, k) is None else getattr(self, k).copy()) for k in self.__slots__})


class _Stop(Exception):
    def __init__(self, status):
        super().__init__(STATUS.get(status, str(status)))
        self.status = status


class _Ipm:
    """One interior-point run (the original problem, or the restoration problem
    with `parent` = the original run)."""

    def __init__(self, prob, o, counter, log, parent=None):
        self.p, self.o, self.counter, self.log, self.parent = prob, o, counter, log, parent
        self.filt = []
        self.dw_last = 0.0
        # line-search state (IpBacktrackingLineSearch / IpFilterLSAcceptor)
        self.last_mu = -1.0
        self.in_watchdog = False
        self.watchdog_shortened_iter = 0
        self.watchdog_trial_iter = 0
        self.tiny_step_last_iteration = False
        self.tiny_step_flag = False
        self.in_soft_resto = False
        self.soft_resto_counter = 0
        self.fallback = False
        self.last_rejection_due_to_filter = False
        self.count_successive_filter_rejections = 0
        self.n_filter_resets = 0
        self.acceptable_point = None
        self.root = parent.root if parent is not None else self
        self.last_x = None

    # ------------------------------------------------------------ helpers
    def slacks(self, x, s):
        p = self.p
        return (x - p.xL, p.xU - x, s - p.dL, p.dU - s)

    def push(self, v, lo, hi, hlo, hhi):
        o = self.o
        v = v.copy()
        pl = np.where(hlo, o["bound_push"] * np.maximum(1.0, np.abs(np.where(hlo, lo, 0.0))), 0.0)
        pu = np.where(hhi, o["bound_push"] * np.maximum(1.0, np.abs(np.where(hhi, hi, 0.0))), 0.0)
        both = hlo & hhi
        pl[both] = np.minimum(pl[both], o["bound_frac"] * (hi[both] - lo[both]))
        pu[both] = np.minimum(pu[both], o["bound_frac"] * (hi[both] - lo[both]))
        v = np.where(hlo, np.maximum(v, lo + pl), v)
        v = np.where(hhi, np.minimum(v, hi - pu), v)
        return v

    SLACK_MOVE = EPS ** 0.75

    def safe(self, v, z, bound, mu):
        """IpoptCalculatedQuantities::CalculateSafeSlack: a slack below
        eps*min(1, mu) becomes min(max(mu/z, s_min), slack + slack_move*max(1,|bound|))."""
        s_min = EPS * min(1.0, mu)
        m = v < s_min
        if not np.any(m):
            return v, m
        v = v.copy()
        v[m] = np.minimum(np.maximum(mu / z[m], s_min), np.maximum(v[m], 0.0) + self.SLACK_MOVE * np.maximum(1.0, np.abs(bound[m])))
        return v, m

    def _xmask(self, m):
        """bound mask without the restoration n/p entries (their slacks are not corrected)"""
        if self.p.is_resto:
            m = m.copy()
            m[self.p.nx:] = False
        return m

    def safe_slacks(self, x, s, it, mu):
        """Slacks at (x, s) with the safe-slack correction (multipliers of `it`)."""
        p = self.p
        xl, xu, sl, su = self.slacks(x, s)
        out = []
        for v, z, b, msk in ((xl, it.zL, p.xL, self._xmask(p.hxL)), (xu, it.zU, p.xU, self._xmask(p.hxU)),
                             (sl, it.vL, p.dL, p.hdL), (su, it.vU, p.dU, p.hdU)):
            vv = v.copy()
            if np.any(msk):
                vv[msk] = self.safe(v[msk], z[msk], b[msk], mu)[0]
            out.append(vv)
        return tuple(out)

    def adjust_bounds(self, x, s, it, mu):
        """After accepting (x, s): shift the bounds of corrected slacks (AdjustVariableBounds)."""
        p = self.p
        xl, xu, sl, su = self.slacks(x, s)
        for v, z, b, msk, sign, val in ((xl, it.zL, p.xL, self._xmask(p.hxL), -1, x), (xu, it.zU, p.xU, self._xmask(p.hxU), 1, x),
                                        (sl, it.vL, p.dL, p.hdL, -1, s), (su, it.vU, p.dU, p.hdU, 1, s)):
            idx = np.where(msk)[0]
            if idx.size == 0:
                continue
            vv, m = self.safe(v[idx], z[idx], b[idx], mu)
            if np.any(m):
                j = idx[m]
                b[j] = val[j] + sign * vv[m]

    def barrier(self, x, s, mu, it=None):
        p, o = self.p, self.o
        sl = self.slacks(x, s) if it is None else self.safe_slacks(x, s, it, mu)
        masks = (p.hxL, p.hxU, p.hdL, p.hdU)
        for v, m in zip(sl, masks):
            if np.any(v[m] <= 0):
                return np.inf
        val = p.f(x, mu)
        for v, m in zip(sl, masks):
            val -= mu * np.sum(libm.log(v[m]))
        kd = o["kappa_d"] * mu
        val += kd * np.sum(sl[0][p.hxL & ~p.hxU]) + kd * np.sum(sl[1][p.hxU & ~p.hxL])
        val += kd * np.sum(sl[2][p.hdL & ~p.hdU]) + kd * np.sum(sl[3][p.hdU & ~p.hdL])
        return val

    def grad_barrier(self, x, s, mu):
        p, o = self.p, self.o
        xl, xu, sl, su = self.slacks(x, s)
        kd = o["kappa_d"] * mu
        gx = p.grad_f(x, mu).copy()
        gx[p.hxL] -= mu / xl[p.hxL]
        gx[p.hxU] += mu / xu[p.hxU]
        gx[p.hxL & ~p.hxU] += kd
        gx[p.hxU & ~p.hxL] -= kd
        gs = np.zeros_like(s)
        gs[p.hdL] -= mu / sl[p.hdL]
        gs[p.hdU] += mu / su[p.hdU]
        gs[p.hdL & ~p.hdU] += kd
        gs[p.hdU & ~p.hdL] -= kd
        return gx, gs

    @staticmethod
    def theta(c, d, s):
        return np.sum(np.abs(c)) + np.sum(np.abs(d - s))

    def errors(self, it, c, d, Jc, Jd, mu):
        """Optimality/barrier errors; mu enters the complementarity only (the
        restoration objective's gradient is taken at the current barrier mu)."""
        p, o = self.p, self.o
        gx = p.grad_f(it.x, self.mu) + Jc.T @ it.yc + Jd.T @ it.yd - it.zL + it.zU
        gs = -it.yd - it.vL + it.vU
        dual = max(np.max(np.abs(gx), initial=0.0), np.max(np.abs(gs), initial=0.0))
        xl, xu, sl, su = self.slacks(it.x, it.s)
        comp = 0.0
        for v, z, m in ((xl, it.zL, p.hxL), (xu, it.zU, p.hxU), (sl, it.vL, p.hdL), (su, it.vU, p.hdU)):
            if np.any(m):
                comp = max(comp, np.max(np.abs(v[m] * z[m] - mu)))
        nz = p.hxL.sum() + p.hxU.sum() + p.hdL.sum() + p.hdU.sum()
        zsum = np.sum(np.abs(it.zL)) + np.sum(np.abs(it.zU)) + np.sum(np.abs(it.vL)) + np.sum(np.abs(it.vU))
        ysum = np.sum(np.abs(it.yc)) + np.sum(np.abs(it.yd))
        ny = it.yc.size + it.yd.size
        s_d = max(o["s_max"], (ysum + zsum) / max(1, ny + nz)) / o["s_max"]
        s_c = max(o["s_max"], zsum / max(1, nz)) / o["s_max"]
        prim_b = max(np.max(np.abs(c), initial=0.0), np.max(np.abs(d - it.s), initial=0.0))
        dv = np.maximum(0.0, np.maximum(np.where(p.hdL, p.dL - d, 0.0), np.where(p.hdU, d - p.dU, 0.0)))
        prim_nlp = max(np.max(np.abs(c), initial=0.0), np.max(dv, initial=0.0))
        return dict(dual=dual, comp=comp, s_d=s_d, s_c=s_c, prim_b=prim_b, prim_nlp=prim_nlp)

    def pd_error(self, it, c, d, Jc, Jd, mu, zref=None):
        """curr/trial_primal_dual_system_error(mu): averaged 1-norms of the dual
        infeasibility, primal infeasibility and relaxed complementarity (trial
        point: safe slacks with the current multipliers zref)."""
        p = self.p
        gx = p.grad_f(it.x, mu) + Jc.T @ it.yc + Jd.T @ it.yd - it.zL + it.zU
        gs = -it.yd - it.vL + it.vU
        nd_ = gx.size + gs.size
        dual = (np.sum(np.abs(gx)) + np.sum(np.abs(gs))) / max(1, nd_)
        npr = c.size + d.size
        prim = (np.sum(np.abs(c)) + np.sum(np.abs(d - it.s))) / npr if npr else 0.0
        xl, xu, sl, su = self.slacks(it.x, it.s) if zref is None else self.safe_slacks(it.x, it.s, zref, mu)
        cs, ncs = 0.0, 0
        for v, z, m in ((xl, it.zL, p.hxL), (xu, it.zU, p.hxU), (sl, it.vL, p.hdL), (su, it.vU, p.hdU)):
            cs += np.sum(np.abs(v[m] * z[m] - mu))
            ncs += int(m.sum())
        return dual + prim + (cs / ncs if ncs else 0.0)

    def frac_primal(self, it, dx, ds, tau):
        p = self.p
        xl, xu, sl, su = self.slacks(it.x, it.s)
        a = 1.0
        for v, dv, m, sg in ((xl, dx, p.hxL, 1), (xu, dx, p.hxU, -1), (sl, ds, p.hdL, 1), (su, ds, p.hdU, -1)):
            step = sg * dv
            sel = m & (step < 0)
            if np.any(sel):
                a = min(a, np.min(-tau * v[sel] / step[sel]))
        return a

    def frac_dual(self, it, dzs, tau):
        p = self.p
        a = 1.0
        for z, dz, m in zip((it.zL, it.zU, it.vL, it.vU), dzs, (p.hxL, p.hxU, p.hdL, p.hdU)):
            sel = m & (dz < 0)
            if np.any(sel):
                a = min(a, np.min(-tau * z[sel] / dz[sel]))
        return a

    def dz_of(self, it, dx, ds, mu):
        p = self.p
        xl, xu, sl, su = self.slacks(it.x, it.s)
        sxl, sxu = np.where(p.hxL, xl, 1.0), np.where(p.hxU, xu, 1.0)
        ssl, ssu = np.where(p.hdL, sl, 1.0), np.where(p.hdU, su, 1.0)
        return (np.where(p.hxL, (mu - it.zL * sxl - it.zL * dx) / sxl, 0.0),
                np.where(p.hxU, (mu - it.zU * sxu + it.zU * dx) / sxu, 0.0),
                np.where(p.hdL, (mu - it.vL * ssl - it.vL * ds) / ssl, 0.0),
                np.where(p.hdU, (mu - it.vU * ssu + it.vU * ds) / ssu, 0.0))

    def dual_step(self, it, a_primal, a_dual, dyc, dyd, dzs, mu, adjust=False):
        """PerformDualStep + the kappa_Sigma safeguard (`it` holds the new primal
        point and the old multipliers; safe slacks; adjust: shift the bounds)."""
        p, o = self.p, self.o
        xl, xu, sl, su = self.safe_slacks(it.x, it.s, it, mu)
        if adjust:
            self.adjust_bounds(it.x, it.s, it, mu)
        new = it.copy()
        new.yc = it.yc + a_primal * dyc
        new.yd = it.yd + a_primal * dyd
        new.zL = it.zL + a_dual * dzs[0]
        new.zU = it.zU + a_dual * dzs[1]
        new.vL = it.vL + a_dual * dzs[2]
        new.vU = it.vU + a_dual * dzs[3]
        ks = o["kappa_sigma"]
        for z, v, m in ((new.zL, xl, p.hxL), (new.zU, xu, p.hxU), (new.vL, sl, p.hdL), (new.vU, su, p.hdU)):
            z[m] = np.maximum(np.minimum(z[m], ks * mu / v[m]), mu / (ks * v[m]))
        return new

    def current_is_acceptable(self, e0, uviol):
        o, p = self.o, self.p
        nlp_err = max(e0["dual"] / e0["s_d"], e0["prim_nlp"], e0["comp"] / e0["s_c"])
        return (nlp_err <= o["acceptable_tol"] and e0["dual"] / p.sf <= o["acceptable_dual_inf_tol"]
                and uviol <= o["acceptable_constr_viol_tol"] and e0["comp"] / p.sf <= o["acceptable_compl_inf_tol"])

    # ------------------------------------------------------- filter acceptor
    def augment_filter(self, ref):
        theta, phi = ref[0], ref[1]
        self.filt.append(((1 - self.o["gamma_theta"]) * theta, phi - self.o["gamma_phi"] * theta))

    def is_ftype(self, ref, a):
        theta, _, gBD = ref
        return gBD < 0 and a * (-gBD) ** self.o["s_phi"] > self.o["delta"] * theta ** self.o["s_theta"]

    def armijo(self, ref, a, ph_t):
        return compare_le(ph_t - ref[1], self.o["eta_phi"] * a * ref[2], ref[1])

    def acceptable_to_iterate(self, ref, ph_t, th_t, from_resto=False):
        theta, phi, _ = ref
        o = self.o
        if not from_resto and ph_t > phi:
            basval = math.log10(abs(phi)) if abs(phi) > 10.0 else 1.0
            if math.log10(ph_t - phi) > o["obj_max_inc"] + basval:
                return False
        return (compare_le(th_t, (1 - o["gamma_theta"]) * theta, theta)
                or compare_le(ph_t - phi, -o["gamma_phi"] * theta, phi))

    def acceptable_to_filter(self, ph_t, th_t):
        return all(th_t < tf or ph_t < pf for (tf, pf) in self.filt)

    def check_trial(self, ref, a_test, th_t, ph_t):
        """FilterLSAcceptor::CheckAcceptabilityOfTrialPoint."""
        if th_t > self.theta_max or not np.isfinite(ph_t):
            return False
        theta = ref[0]
        if a_test > 0 and self.is_ftype(ref, a_test) and theta <= self.theta_min:
            ok = self.armijo(ref, a_test, ph_t)
        else:
            ok = self.acceptable_to_iterate(ref, ph_t, th_t)
        if not ok:
            self.last_rejection_due_to_filter = False
            return False
        if not self.acceptable_to_filter(ph_t, th_t):
            self.last_rejection_due_to_filter = True
            return False
        return True

    def update_for_next_iteration(self, ref, a_test, ph_t):
        o = self.o
        if not (self.is_ftype(ref, a_test) and self.armijo(ref, a_test, ph_t)):
            self.augment_filter(ref)
        if o["max_filter_resets"] > 0:
            if self.n_filter_resets < o["max_filter_resets"]:
                if self.last_rejection_due_to_filter:
                    self.count_successive_filter_rejections += 1
                    if self.count_successive_filter_rejections >= o["filter_reset_trigger"]:
                        self.filt = []
                        self.count_successive_filter_rejections = 0
                        self.n_filter_resets += 1
                else:
                    self.count_successive_filter_rejections = 0
            self.last_rejection_due_to_filter = False

    # ---------------------------------------------------------------- run
    def trial_values(self, x, s, mu):
        c, d = self.p.cd(x)
        th = self.theta(c, d, s)
        ph = self.barrier(x, s, mu, self.cur_it)
        return c, d, th, ph

    def init_orig(self):
        p, o = self.p, self.o
        nlp = p.nlp
        x = self.push(nlp.x0, p.xL, p.xU, p.hxL, p.hxU)
        c, d = p.cd(x)
        s = self.push(d, p.dL, p.dU, p.hdL, p.hdU)
        bmi = o["bound_mult_init_val"]
        it = _Iterate(x=x, s=s, yc=np.zeros(p.mc), yd=np.zeros(p.md),
                      zL=np.where(p.hxL, bmi, 0.0), zU=np.where(p.hxU, bmi, 0.0),
                      vL=np.where(p.hdL, bmi, 0.0), vU=np.where(p.hdU, bmi, 0.0))
        self.mu = o["mu_init"]
        self.ls_multipliers(it, o["constr_mult_init_max"])
        return it

    def ls_multipliers(self, it, max_abs):
        """Least-squares y: [I 0 Jc' Jd'; 0 I 0 -I; Jc 0 0 0; Jd -I 0 0]."""
        p = self.p
        Jc, Jd = p.jac(it.x)
        gf = p.grad_f(it.x, self.mu)
        inert = p.factor(sp.csr_matrix((p.n, p.n)), np.ones(p.n), np.ones(p.md), Jc, Jd, 0.0, 0.0)
        it.yc, it.yd = np.zeros(p.mc), np.zeros(p.md)
        if inert[1] == p.mc + p.md and inert[2] == 0:
            _, _, yc_, yd_ = p.solve(-(gf - it.zL + it.zU), -(-it.vL + it.vU), np.zeros(p.mc), np.zeros(p.md))
            if max(np.max(np.abs(yc_), initial=0.0), np.max(np.abs(yd_), initial=0.0)) <= max_abs:
                it.yc, it.yd = yc_, yd_

    def run(self, it):
        """Iterate from `it` (status on exit; raises _Stop for terminal statuses).
        Returns the final iterate (orig) / the resto iterate on success (resto)."""
        p, o = self.p, self.o
        self.tau = max(o["tau_min"], 1.0 - self.mu)
        c, d = p.cd(it.x)
        th0 = self.theta(c, d, it.s)
        self.theta_max = 1e4 * max(1.0, th0)
        self.theta_min = 1e-4 * max(1.0, th0)
        Jc, Jd = p.jac(it.x)
        first = True
        while True:
            k = self.counter[0]
            self.root.last_x = it.x[:p.nx] if p.is_resto else it.x
            e0 = self.errors(it, c, d, Jc, Jd, 0.0)
            nlp_err = max(e0["dual"] / e0["s_d"], e0["prim_nlp"], e0["comp"] / e0["s_c"])
            uviol = p.unscaled_viol(it.x, c, d)
            self.log.append(dict(it=k, resto=p.is_resto, mu=self.mu, err=nlp_err, theta=self.theta(c, d, it.s),
                                 dual=e0["dual"], comp=e0["comp"], prim=e0["prim_nlp"]))
            # ---- convergence check
            if p.is_resto:
                st = self.resto_check(it, first)
                if st == "converged":
                    return it
            optimal = (nlp_err <= o["tol"] and e0["dual"] / p.sf <= o["dual_inf_tol"]
                       and uviol <= o["constr_viol_tol"] and e0["comp"] / p.sf <= o["compl_inf_tol"])
            accept_lvl = self.current_is_acceptable(e0, uviol)
            if p.is_resto:
                if not first and (optimal or (accept_lvl and self.acc_count + 1 >= o["acceptable_iter"])):
                    # the restoration problem converged without reaching an acceptable original point
                    # RestoConvergenceCheck: orig_ip_cq->trial_primal_infeasibility(NORM_MAX) <= 1e2 tol
                    # -> RESTORATION_CONVERGED_TO_FEASIBLE_POINT, else LOCALLY_INFEASIBLE
                    ot = self.parent.orig_primal_inf_max(it.x[:p.nx], it.s)
                    self.parent_status = RESTO_FAILED if ot <= 1e2 * o["tol"] else INFEASIBLE
                    raise _Stop(self.parent_status)
                self.acc_count = self.acc_count + 1 if accept_lvl else 0
            else:
                if optimal:
                    self.final, self.status = it, SUCCESS
                    return it
                if accept_lvl:
                    self.acc_count += 1
                    if self.acc_count >= o["acceptable_iter"]:
                        self.final, self.status = it, ACCEPTABLE
                        return it
                else:
                    self.acc_count = 0
            if k >= o["max_iter"]:
                raise _Stop(MAXITER)
            first = False
            # ---- monotone barrier update
            while True:
                eb = self.errors(it, c, d, Jc, Jd, self.mu)
                berr = max(eb["dual"] / eb["s_d"], eb["prim_b"], eb["comp"] / eb["s_c"])
                if berr > o["kappa_eps"] * self.mu and not self.tiny_step_flag:
                    break
                new_mu = max(o["tol"] / 10.0, min(o["kappa_mu"] * self.mu, self.mu ** o["theta_mu"]))
                if new_mu == self.mu:
                    if self.tiny_step_flag:
                        raise _Stop(TINY_STEP)
                    break
                self.mu = new_mu
                self.tau = max(o["tau_min"], 1.0 - self.mu)
                self.filt = []
                self.tiny_step_flag = False
            self.tiny_step_flag = False
            mu, tau = self.mu, self.tau
            # ---- search direction with inertia correction
            W = p.hess(it.x, it.yc, it.yd, mu)
            xl, xu, sl, su = self.slacks(it.x, it.s)
            Sx = np.where(p.hxL, it.zL / np.where(p.hxL, xl, 1.0), 0.0) + \
                np.where(p.hxU, it.zU / np.where(p.hxU, xu, 1.0), 0.0)
            Ss = np.where(p.hdL, it.vL / np.where(p.hdL, sl, 1.0), 0.0) + \
                np.where(p.hdU, it.vU / np.where(p.hdU, su, 1.0), 0.0)
            gbx, gbs = self.grad_barrier(it.x, it.s, mu)
            rx = gbx + Jc.T @ it.yc + Jd.T @ it.yd
            rs = gbs - it.yd
            delta = None
            dw, dc = 0.0, 0.0
            while True:
                pos, neg, zer = p.factor(W, Sx, Ss, Jc, Jd, dw, dc)
                if neg == p.mc + p.md and zer == 0:
                    delta = p.solve(-rx, -rs, -c, -(d - it.s))
                    break
                if zer > 0 and dc == 0.0:
                    dc = o["dc_bar"] * mu ** o["kappa_c"]
                    continue
                if dw == 0.0:
                    dw = o["dw0"] if self.dw_last == 0.0 else max(o["dw_min"], o["kw_minus"] * self.dw_last)
                else:
                    dw = (o["kw_plus_bar"] if (self.dw_last == 0.0 or 1e5 * self.dw_last < dw) else o["kw_plus"]) * dw
                if dw > o["dw_max"]:
                    break
            if delta is None:
                self.fallback = True
            elif dw > 0.0:
                self.dw_last = dw
            self.kkt_state = (dw, dc, rx, rs)
            # ---- line search
            cur = dict(it=it, c=c, d=d, Jc=Jc, Jd=Jd, e0=e0, uviol=uviol)
            it, c, d = self.find_trial(cur, delta, gbx, gbs, rx, rs)
            Jc, Jd = p.jac(it.x)
            self.counter[0] += 1

    # ------------------------------------------------------ line search
    def find_trial(self, cur, delta, gbx, gbs, rx, rs):
        p, o = self.p, self.o
        it, c, d = cur["it"], cur["c"], cur["d"]
        mu, tau = self.mu, self.tau
        self.cur_it = it
        if not p.is_resto and self.current_is_acceptable(cur["e0"], cur["uviol"]):
            self.acceptable_point = it.copy()
        if self.last_mu != mu:
            self.in_watchdog = False
            self.watchdog_shortened_iter = 0
            self.last_mu = mu
        theta = self.theta(c, d, it.s)
        phi = self.barrier(it.x, it.s, mu)
        goto_resto = self.fallback
        self.fallback = False
        gBD = (gbx @ delta[0] + gbs @ delta[1]) if delta is not None else 0.0
        ref = self.wd_ref if self.in_watchdog else (theta, phi, gBD)
        accept = False
        n_steps = 0
        a_primal = 0.0
        tiny = (not goto_resto) and self.detect_tiny_step(it, delta, c, d)
        if self.in_watchdog and (goto_resto or tiny):
            it, c, d, delta, gbx, gbs, rx, rs = self.stop_watchdog()
            cur = dict(it=it, c=c, d=d)
            self.cur_it = it
            theta, phi = ref[0], ref[1]
            goto_resto = tiny = False
        if (o["watchdog_shortened_iter_trigger"] > 0 and not self.in_watchdog and not goto_resto and not tiny
                and not self.in_soft_resto and self.watchdog_shortened_iter >= o["watchdog_shortened_iter_trigger"]):
            self.start_watchdog(it, c, d, delta, (theta, phi, gBD), gbx, gbs, rx, rs)
        trial = None
        a_test = 0.0
        if tiny:
            a_primal = self.frac_primal(it, delta[0], delta[1], tau)
            xt, st = it.x + a_primal * delta[0], it.s + a_primal * delta[1]
            trial = (xt, st) + self.trial_values(xt, st, mu)
            if self.tiny_step_last_iteration:
                self.tiny_step_flag = True
            self.tiny_step_last_iteration = True
            accept = True
        else:
            self.tiny_step_last_iteration = False
        soft_step = False
        if not goto_resto and not tiny:
            if self.in_soft_resto:
                self.soft_resto_counter += 1
                if self.soft_resto_counter > o["max_soft_resto_iters"]:
                    accept = False
                else:
                    accept, satisfies, res = self.try_soft_resto_step(cur, delta, (theta, phi, gBD))
                    if accept:
                        soft_step = True
                        new_it, c2, d2 = res
                        if satisfies:
                            self.in_soft_resto = False
                            self.soft_resto_counter = 0
                        return new_it, c2, d2
            else:
                skip_first = False
                while True:
                    accept, n_steps, a_primal, a_test, trial, delta = self.backtrack(
                        it, c, d, delta, ref, skip_first, n_steps, rx, rs)
                    if self.in_watchdog:
                        if accept:
                            self.in_watchdog = False
                            break
                        self.watchdog_trial_iter += 1
                        if self.watchdog_trial_iter > o["watchdog_trial_iter_max"]:
                            it, c, d, delta, gbx, gbs, rx, rs = self.stop_watchdog()
                            cur = dict(it=it, c=c, d=d)
                            self.cur_it = it
                            ref = (self.wd_ref[0], self.wd_ref[1], self.wd_ref[2])
                            skip_first = True
                            continue
                        accept = True   # the watchdog takes the full step unchecked
                        break
                    break
        if not accept:
            if not self.in_soft_resto and o["soft_resto_pderror_reduction_factor"] > 0 and not goto_resto:
                self.augment_filter(ref)                      # PrepareRestoPhaseStart
                accept, satisfies, res = self.try_soft_resto_step(cur, delta, ref)
                if accept:
                    if not satisfies:
                        self.in_soft_resto = True
                    return res
            else:
                if not self.in_soft_resto:
                    self.augment_filter(ref)
            # ---- restoration phase
            if theta <= 1e-2 * o["tol"]:
                raise _Stop(self.restore_acceptable_point())
            self.in_soft_resto = False
            self.soft_resto_counter = 0
            self.watchdog_shortened_iter = 0
            self.count_successive_filter_rejections = 0
            if p.is_resto:
                return self.resto_resto(it)
            return self.restoration(it, (theta, phi, gBD))
        # ---- accepted (regular / watchdog / tiny step)
        if not tiny and not (self.in_watchdog and not accept):
            pass
        xt, st, ct, dt, _th, _ph = trial
        dx, ds, dyc, dyd = delta
        new = it.copy()
        new.x, new.s = xt, st
        # dual step along the (possibly corrected) direction actually taken
        dzs = self.dz_of(it, dx, ds, mu)
        a_dual = self.frac_dual(it, dzs, tau)
        new = self.dual_step(new, a_primal, a_dual, dyc, dyd, dzs, mu, adjust=True)
        if n_steps == 0:
            self.watchdog_shortened_iter = 0
        if n_steps > 0:
            self.watchdog_shortened_iter += 1
        return new, ct, dt

    def backtrack(self, it, c, d, delta, ref, skip_first, n_steps, rx, rs):
        """DoBacktrackingLineSearch (with second-order corrections)."""
        p, o = self.p, self.o
        mu, tau = self.mu, self.tau
        dx, ds = delta[0], delta[1]
        alpha_max = self.frac_primal(it, dx, ds, tau)
        if self.in_watchdog:
            alpha_min = alpha_max
        else:
            theta, _, gBD = ref
            alpha_min = o["gamma_theta"]
            if gBD < 0:
                alpha_min = min(o["gamma_theta"], o["gamma_phi"] * theta / (-gBD))
                if theta <= self.theta_min:
                    alpha_min = min(alpha_min, o["delta"] * theta ** o["s_theta"] / (-gBD) ** o["s_phi"])
            alpha_min *= o["alpha_min_frac"]
        alpha = alpha_max
        if skip_first:
            alpha *= 0.5
        accept = False
        trial = None
        a_test = alpha
        theta_curr = self.theta(c, d, it.s)
        while alpha > alpha_min or n_steps == 0:
            xt, st = it.x + alpha * dx, it.s + alpha * ds
            trial = (xt, st) + self.trial_values(xt, st, mu)
            a_test = self.wd_alpha_test if self.in_watchdog else alpha
            if self.check_trial(ref, a_test, trial[4], trial[5]):
                accept = True
                break
            if self.in_watchdog:
                break
            if alpha == alpha_max and theta_curr <= trial[4] and o["max_soc"] > 0:
                ok, soc_trial, soc_alpha, soc_delta = self.second_order_correction(it, c, d, trial, alpha, a_test, ref, rx, rs)
                if ok:
                    accept, trial, delta = True, soc_trial, soc_delta
                    alpha = soc_alpha
                    break
            alpha *= 0.5
            n_steps += 1
        if accept:
            self.update_for_next_iteration(ref, a_test, trial[5])
        return accept, n_steps, alpha, a_test, trial, delta

    def second_order_correction(self, it, c, d, trial, alpha, a_test, ref, rx, rs):
        p, o = self.p, self.o
        xt, st, ct, dt, th_t, _ = trial
        c_soc, d_soc = alpha * c + ct, alpha * (d - it.s) + (dt - st)
        th_old = ref[0]
        for _k in range(o["max_soc"]):
            sx, ss, syc, syd = p.solve(-rx, -rs, -c_soc, -d_soc)
            a_soc = self.frac_primal(it, sx, ss, self.tau)
            xs_, ss_ = it.x + a_soc * sx, it.s + a_soc * ss
            tr = (xs_, ss_) + self.trial_values(xs_, ss_, self.mu)
            if self.check_trial(ref, a_test, tr[4], tr[5]):
                return True, tr, a_soc, (sx, ss, syc, syd)
            if tr[4] > o["kappa_soc"] * th_old:
                break
            th_old = tr[4]
            c_soc, d_soc = a_soc * c_soc + tr[2], a_soc * d_soc + (tr[3] - ss_)
        return False, None, None, None

    def detect_tiny_step(self, it, delta, c, d):
        o = self.o
        if delta is None or o["tiny_step_tol"] == 0.0:
            return False
        if np.max(np.abs(delta[0]) / (1.0 + np.abs(it.x)), initial=0.0) > o["tiny_step_tol"]:
            return False
        if np.max(np.abs(delta[1]) / (1.0 + np.abs(it.s)), initial=0.0) > o["tiny_step_tol"]:
            return False
        if max(np.max(np.abs(delta[2]), initial=0.0), np.max(np.abs(delta[3]), initial=0.0)) >= o["tiny_step_y_tol"]:
            return False
        if max(np.max(np.abs(c), initial=0.0), np.max(np.abs(d - it.s), initial=0.0)) > 1e-4:
            return False
        return True

    def start_watchdog(self, it, c, d, delta, ref, gbx, gbs, rx, rs):
        self.in_watchdog = True
        self.wd_saved = (it.copy(), c.copy(), d.copy(), delta, gbx, gbs, rx, rs, self.kkt_state)
        self.wd_ref = ref
        self.watchdog_trial_iter = 0
        self.wd_alpha_test = self.frac_primal(it, delta[0], delta[1], self.tau)

    def stop_watchdog(self):
        """Resume from the stored iterate along the stored direction (re-factor
        the stored point's matrix for any second-order correction)."""
        self.in_watchdog = False
        it, c, d, delta, gbx, gbs, rx, rs, kst = self.wd_saved
        p = self.p
        dw, dc = kst[0], kst[1]
        W = p.hess(it.x, it.yc, it.yd, self.mu)
        xl, xu, sl, su = self.slacks(it.x, it.s)
        Sx = np.where(p.hxL, it.zL / np.where(p.hxL, xl, 1.0), 0.0) + np.where(p.hxU, it.zU / np.where(p.hxU, xu, 1.0), 0.0)
        Ss = np.where(p.hdL, it.vL / np.where(p.hdL, sl, 1.0), 0.0) + np.where(p.hdU, it.vU / np.where(p.hdU, su, 1.0), 0.0)
        Jc, Jd = p.jac(it.x)
        p.factor(W, Sx, Ss, Jc, Jd, dw, dc)
        self.watchdog_shortened_iter = 0
        self.wd_saved = None
        return it, c, d, delta, gbx, gbs, rx, rs

    def try_soft_resto_step(self, cur, delta, ref):
        """TrySoftRestoStep: the primal-dual step with alpha = min(primal, dual
        fraction to the boundary); accepted if it satisfies the original filter
        criteria or reduces the primal-dual error by the factor 0.9999."""
        p, o = self.p, self.o
        it, c, d = cur["it"], cur["c"], cur["d"]
        if delta is None:
            return False, False, None
        mu, tau = self.mu, self.tau
        dx, ds, dyc, dyd = delta
        dzs = self.dz_of(it, dx, ds, mu)
        a = min(self.frac_primal(it, dx, ds, tau), self.frac_dual(it, dzs, tau))
        new = it.copy()
        new.x, new.s = it.x + a * dx, it.s + a * ds
        new = self.dual_step(new, a, a, dyc, dyd, dzs, mu)
        ct, dt, th_t, ph_t = self.trial_values(new.x, new.s, mu)
        if self.check_trial(ref, 0.0, th_t, ph_t):
            self.adjust_bounds(new.x, new.s, it, mu)
            return True, True, (new, ct, dt)
        Jc, Jd = cur.get("Jc"), cur.get("Jd")
        if Jc is None:
            Jc, Jd = p.jac(it.x)
        Jct, Jdt = p.jac(new.x)
        if self.pd_error(new, ct, dt, Jct, Jdt, mu, zref=it) <= o["soft_resto_pderror_reduction_factor"] * \
                self.pd_error(it, c, d, Jc, Jd, mu):
            self.adjust_bounds(new.x, new.s, it, mu)
            return True, False, (new, ct, dt)
        return False, False, None

    def restore_acceptable_point(self):
        if self.acceptable_point is not None:
            self.final, self.status = self.acceptable_point, ACCEPTABLE
            return ACCEPTABLE
        return RESTO_FAILED

    # ------------------------------------------------- restoration phase
    def orig_theta(self, x, s):
        c, d = self.p.cd(x)
        return self.theta(c, d, s)

    def orig_primal_inf_max(self, x, s):
        """Max-norm primal infeasibility of the (scaled) original problem at (x, s)."""
        c, d = self.p.cd(x)
        return max(np.max(np.abs(c), initial=0.0), np.max(np.abs(d - s), initial=0.0))

    def restoration(self, it, ref):
        """MinC_1NrmRestorationPhase::PerformRestoration (original problem only)."""
        p, o = self.p, self.o
        rp = RestoProblem(p, it.x, o)
        c, d = p.cd(it.x)
        mu_r = max(self.mu, np.max(np.abs(c), initial=0.0), np.max(np.abs(d - it.s), initial=0.0))
        rho = rp.rho
        a = mu_r / (2.0 * rho) - 0.5 * c
        nc = _solve_quadratic(a, c * mu_r / (2.0 * rho))
        pc = c + nc
        dms = d - it.s
        a = mu_r / (2.0 * rho) - 0.5 * dms
        nd = _solve_quadratic(a, dms * mu_r / (2.0 * rho))
        pd = dms + nd
        X = np.concatenate([it.x, nc, pc, nd, pd])
        zL = np.concatenate([np.minimum(rho, it.zL), mu_r / nc, mu_r / pc, mu_r / nd, mu_r / pd])
        zU = np.concatenate([np.minimum(rho, it.zU), np.zeros(2 * p.mc + 2 * p.md)])
        rit = _Iterate(x=X, s=it.s.copy(), yc=None, yd=None, zL=zL,
                       zU=np.where(rp.hxU, zU, 0.0), vL=np.minimum(rho, it.vL), vU=np.minimum(rho, it.vU))
        sub = _Ipm(rp, o, self.counter, self.log, parent=self)
        sub.mu = mu_r
        sub.acc_count = 0
        sub.ls_multipliers(rit, o["constr_mult_init_max"])
        self.resto_ref = ref
        self.resto_theta0 = ref[0]
        self.counter[0] += 1     # the restoration phase starts with the next iteration number
        try:
            rend = sub.run(rit)
        except _Stop as e:
            if e.status in (RESTO_FAILED, INFEASIBLE, STEP_FAILED):
                st = self.restore_acceptable_point()
                raise _Stop(st if st == ACCEPTABLE else e.status)
            raise
        self.counter[0] -= 1     # IpData().Set_iter_count(resto_iter - 1)
        # back to the original problem: x, s from the restoration phase
        xr, sr = rend.x[:p.nx] if hasattr(p, "nx") else rend.x[:p.n], rend.s
        new = it.copy()
        new.x, new.s = xr.copy(), sr.copy()
        # bound multipliers: one complementarity Newton step for the whole primal change
        mu = self.mu
        cur_sl, tri_sl = self.slacks(it.x, it.s), self.slacks(new.x, new.s)
        dzs = []
        for z, cs, ts, m in zip((it.zL, it.zU, it.vL, it.vU), cur_sl, tri_sl, (p.hxL, p.hxU, p.hdL, p.hdU)):
            dz = np.zeros_like(z)
            dz[m] = (mu + z[m] * (cs[m] - ts[m])) / ts[m] - z[m]
            dzs.append(dz)
        a_dual = self.frac_dual(it, dzs, self.tau)
        new.zL, new.zU = it.zL + a_dual * dzs[0], it.zU + a_dual * dzs[1]
        new.vL, new.vU = it.vL + a_dual * dzs[2], it.vU + a_dual * dzs[3]
        bmax = max(np.max(np.abs(new.zL), initial=0.0), np.max(np.abs(new.zU), initial=0.0),
                   np.max(np.abs(new.vL), initial=0.0), np.max(np.abs(new.vU), initial=0.0))
        if bmax > o["bound_mult_reset_threshold"]:
            new.zL, new.zU = np.where(p.hxL, 1.0, 0.0), np.where(p.hxU, 1.0, 0.0)
            new.vL, new.vU = np.where(p.hdL, 1.0, 0.0), np.where(p.hdU, 1.0, 0.0)
        # constraint multipliers: constr_mult_reset_threshold = 0 -> zero
        new.yc, new.yd = np.zeros(p.mc), np.zeros(p.md)
        c2, d2 = p.cd(new.x)
        return new, c2, d2

    def resto_check(self, it, first):
        """RestoConvergenceCheck / RestoFilterConvergenceCheck (restoration run)."""
        if first:
            return "continue"
        par, p, o = self.parent, self.p, self.o
        x, s = it.x[:p.nx], it.s
        th_t = par.orig_theta(x, s)
        if th_t > o["required_infeasibility_reduction"] * par.resto_theta0:
            return "continue"
        ph_t = par.barrier(x, s, par.mu)
        if not par.acceptable_to_filter(ph_t, th_t):
            return "continue"
        if not par.acceptable_to_iterate(par.resto_ref, ph_t, th_t, from_resto=True):
            return "continue"
        return "converged"

    def resto_resto(self, it):
        """RestoRestorationPhase: n, p reset in closed form at the current x."""
        p = self.p
        x = it.x[:p.nx]
        c, d = p.orig.cd(x)
        mu, rho = self.mu, p.rho
        a = mu / (2.0 * rho) - 0.5 * c
        nc = _solve_quadratic(a, c * mu / (2.0 * rho))
        pc = c + nc
        dms = d - it.s
        a = mu / (2.0 * rho) - 0.5 * dms
        nd = _solve_quadratic(a, dms * mu / (2.0 * rho))
        pd = dms + nd
        new = it.copy()
        new.x = np.concatenate([x, nc, pc, nd, pd])
        zx = it.zL[:p.nx]
        new.zL = np.concatenate([zx, mu / nc, mu / pc, mu / nd, mu / pd])
        c2, d2 = p.cd(new.x)
        return new, c2, d2


class IpoptRestatement:
    """IPOPT 3.14 default algorithm on an NLP object (oracle/nlp.py API)."""

    def __init__(self, nlp, opts=None, kkt=None):
        self.nlp = nlp
        self.o = dict(OPTS)
        if opts:
            self.o.update(opts)
        self.kkt = kkt if kkt is not None else DenseKKT()
        self.log = []

    def solve(self):
        o, nlp = self.o, self.nlp
        prob = OrigProblem(nlp, o, self.kkt)
        self.sf, self.sc = prob.sf, prob.sc
        counter = [0]
        ipm = _Ipm(prob, o, counter, self.log)
        ipm.acc_count = 0
        it = ipm.init_orig()
        try:
            fin = ipm.run(it)
            status = ipm.status
        except _Stop as e:
            status = e.status
            if status == ACCEPTABLE and getattr(ipm, "final", None) is not None:
                fin = ipm.final
            else:  # the last iterate (of the restoration phase, if it failed there)
                fin = _Iterate(x=ipm.last_x, yc=None, yd=None)
        self.n_resto = sum(1 for i in range(1, len(self.log)) if self.log[i]["resto"] and not self.log[i - 1]["resto"])
        xf = fin.x.copy()
        lo, hi = nlp.x_L, nlp.x_U
        xf = np.where(np.isfinite(lo), np.maximum(xf, lo), xf)
        xf = np.where(np.isfinite(hi), np.minimum(xf, hi), xf)
        its = counter[0]
        self.iters, self.status, self.x, self.mu = its, status, xf, ipm.mu
        self.yc, self.yd = fin.yc, fin.yd
        return dict(status=status, status_str=STATUS[status], success=status in (SUCCESS, ACCEPTABLE), iters=its,
                    x=xf, f=nlp.f(xf), yc=fin.yc, yd=fin.yd, n_resto=self.n_resto)
