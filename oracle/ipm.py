"""Oracle: restatement of the IPOPT algorithm that R/obca_py/optimizer.py:489-507
runs through CasADi (`ca.nlpsol("solver", "ipopt", ...)`).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The algorithm lives in a third-party dependency that is absent here:
IPOPT (CasADi >= 3.6.3 bundles IPOPT 3.14.x, R/requirements.txt:9) with MUMPS.
This file restates its *published* algorithm -- A. Waechter, L. T. Biegler,
"On the implementation of an interior-point filter line-search algorithm for
large-scale nonlinear programming", Math. Prog. 106 (2006) -- with IPOPT 3.14's
default options (optimizer.py:481-488 only sets print_level/sb/max_cpu_time):

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
  * fraction-to-the-boundary (primal, dual separately); filter line search
    (gamma_theta 1e-5, gamma_phi 1e-8, delta 1, s_theta 1.1, s_phi 2.3,
    eta_phi 1e-8, alpha_min_frac 0.05, theta_max/min 1e4/1e-4 * max(1,theta0)),
    up to 4 second-order corrections (kappa_soc 0.99); y stepped with alpha_primal
  * kappa_Sigma = 1e10 bound-multiplier safeguard
  * termination: scaled NLP error <= 1e-8 and unscaled dual_inf <= 1,
    constr_viol <= 1e-4, compl <= 1e-4; "acceptable" after 15 iterations at 1e-6
  * final x projected to the original bounds (honor_original_bounds)

Not restated (documented in DESIGN.md): restoration phase (a failed line
search ends the solve with status RESTORATION_FAILED), watchdog, tiny-step
heuristic, iterative refinement, Hessian-degeneracy detection, slack_move.

The KKT systems are solved with a dense Bunch-Kaufman LDL^T (scipy.linalg.ldl)
whose block-diagonal factor gives the exact inertia MUMPS reports.
"""
import math

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp

EPS = np.finfo(float).eps

OPTS = dict(
    tol=1e-8, dual_inf_tol=1.0, constr_viol_tol=1e-4, compl_inf_tol=1e-4,
    acceptable_tol=1e-6, acceptable_iter=15, acceptable_constr_viol_tol=1e-2,
    acceptable_compl_inf_tol=1e-2, acceptable_dual_inf_tol=1e10,
    max_iter=3000, bound_relax_factor=1e-8, scaling_max_gradient=100.0, scaling_min_value=1e-8,
    bound_push=1e-2, bound_frac=1e-2, bound_mult_init_val=1.0, constr_mult_init_max=1e3,
    mu_init=0.1, kappa_eps=10.0, kappa_mu=0.2, theta_mu=1.5, tau_min=0.99, kappa_sigma=1e10,
    kappa_d=1e-5, s_max=100.0, gamma_theta=1e-5, gamma_phi=1e-8, delta=1.0, s_theta=1.1,
    s_phi=2.3, eta_phi=1e-8, alpha_min_frac=0.05, max_soc=4, kappa_soc=0.99,
    dw0=1e-4, dw_min=1e-20, dw_max=1e40, kw_minus=1.0 / 3.0, kw_plus=8.0, kw_plus_bar=100.0,
    dc_bar=1e-8, kappa_c=0.25,
)

STATUS = {0: "Solve_Succeeded", 1: "Solved_To_Acceptable_Level", 2: "Maximum_Iterations_Exceeded",
          3: "Restoration_Failed", 4: "Error_In_Step_Computation"}


def compare_le(lhs, rhs, basval):
    """IPOPT's Compare_le: lhs - rhs <= 10*eps*|basval|."""
    return lhs - rhs <= 10.0 * EPS * abs(basval)


class DenseKKT:
    """[W+Sx+dw, 0, Jc', Jd'; 0, Ss+dw, 0, -I; Jc, 0, -dc, 0; Jd, -I, 0, -dc]."""

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
        K[n + ns:, n + ns:] -= dc * np.eye(mc + ns)
        K = np.tril(K) + np.tril(K, -1).T
        lu, d, perm = sla.ldl(K, lower=True)
        # inertia from the 1x1 / 2x2 blocks of d
        pos = neg = zer = 0
        i = 0
        while i < dim:
            if i + 1 < dim and d[i + 1, i] != 0.0:
                ev = np.linalg.eigvalsh(d[i:i + 2, i:i + 2])
                i += 2
            else:
                ev = [d[i, i]]
                i += 1
            for e in ev:
                if e > 0:
                    pos += 1
                elif e < 0:
                    neg += 1
                else:
                    zer += 1
        self.fac = (lu, d, perm)
        self.dims = (n, ns, mc)
        return pos, neg, zer

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


class IpoptRestatement:
    """IPOPT 3.14 default algorithm on an NLP object (oracle/nlp.py API)."""

    def __init__(self, nlp, opts=None, kkt=None):
        self.nlp = nlp
        self.o = dict(OPTS)
        if opts:
            self.o.update(opts)
        self.kkt = kkt if kkt is not None else DenseKKT()
        self.log = []

    # ------------------------------------------------------------ setup
    def _setup(self):
        o, nlp = self.o, self.nlp
        gL, gU = nlp.g_L, nlp.g_U
        self.E = np.where(gL == gU)[0]
        self.I = np.where(gL != gU)[0]
        x0 = nlp.x0.copy()
        # gradient-based scaling at the user starting point
        gf = nlp.grad_f(x0)
        mg = np.max(np.abs(gf)) if gf.size else 0.0
        self.sf = max(o["scaling_min_value"], o["scaling_max_gradient"] / mg) if mg > o["scaling_max_gradient"] else 1.0
        J = nlp.jac(x0).tocsr()
        rowmax = np.zeros(nlp.m)
        absJ = abs(J)
        rowmax = np.asarray(absJ.max(axis=1).todense()).ravel()
        sc = np.ones(nlp.m)
        big = rowmax > o["scaling_max_gradient"]
        sc[big] = np.maximum(o["scaling_min_value"], o["scaling_max_gradient"] / rowmax[big])
        self.sc = sc
        # relaxed bounds
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

    def _push(self, v, lo, hi, hlo, hhi):
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

    # ------------------------------------------------------- evaluations
    def _eval(self, x):
        g = self.nlp.cons(x)
        c = self.sc[self.E] * (g[self.E] - self.cE)
        d = self.sc[self.I] * g[self.I]
        return c, d

    def _jac(self, x):
        J = sp.diags(self.sc) @ self.nlp.jac(x)
        J = J.tocsr()
        return J[self.E], J[self.I]

    def _hess(self, x, yc, yd):
        y = np.zeros(self.nlp.m)
        y[self.E] = yc * self.sc[self.E]
        y[self.I] = yd * self.sc[self.I]
        return self.nlp.hess(x, y, self.sf)

    def _slacks(self, x, s):
        return (x - self.xL, self.xU - x, s - self.dL, self.dU - s)

    def _barrier(self, x, s, mu):
        o = self.o
        sl = self._slacks(x, s)
        masks = (self.hxL, self.hxU, self.hdL, self.hdU)
        val = self.sf * self.nlp.f(x)
        for v, m in zip(sl, masks):
            val -= mu * np.sum(np.log(v[m]))
        kd = o["kappa_d"] * mu
        val += kd * np.sum(sl[0][self.hxL & ~self.hxU]) + kd * np.sum(sl[1][self.hxU & ~self.hxL])
        val += kd * np.sum(sl[2][self.hdL & ~self.hdU]) + kd * np.sum(sl[3][self.hdU & ~self.hdL])
        return val

    def _grad_barrier(self, x, s, mu):
        o = self.o
        xl, xu, sl, su = self._slacks(x, s)
        kd = o["kappa_d"] * mu
        gx = self.sf * self.nlp.grad_f(x)
        gx[self.hxL] -= mu / xl[self.hxL]
        gx[self.hxU] += mu / xu[self.hxU]
        gx[self.hxL & ~self.hxU] += kd
        gx[self.hxU & ~self.hxL] -= kd
        gs = np.zeros_like(s)
        gs[self.hdL] -= mu / sl[self.hdL]
        gs[self.hdU] += mu / su[self.hdU]
        gs[self.hdL & ~self.hdU] += kd
        gs[self.hdU & ~self.hdL] -= kd
        return gx, gs

    def _theta(self, c, d, s):
        return np.sum(np.abs(c)) + np.sum(np.abs(d - s))

    # ------------------------------------------------------------- errors
    def _errors(self, x, s, yc, yd, zL, zU, vL, vU, c, d, Jc, Jd, mu):
        o = self.o
        gx = self.sf * self.nlp.grad_f(x) + Jc.T @ yc + Jd.T @ yd - zL + zU
        gs = -yd - vL + vU
        dual = max(np.max(np.abs(gx), initial=0.0), np.max(np.abs(gs), initial=0.0))
        xl, xu, sl, su = self._slacks(x, s)
        comp = 0.0
        for v, z, m in ((xl, zL, self.hxL), (xu, zU, self.hxU), (sl, vL, self.hdL), (su, vU, self.hdU)):
            if np.any(m):
                comp = max(comp, np.max(np.abs(v[m] * z[m] - mu)))
        nz = self.hxL.sum() + self.hxU.sum() + self.hdL.sum() + self.hdU.sum()
        zsum = np.sum(np.abs(zL)) + np.sum(np.abs(zU)) + np.sum(np.abs(vL)) + np.sum(np.abs(vU))
        ysum = np.sum(np.abs(yc)) + np.sum(np.abs(yd))
        ny = yc.size + yd.size
        s_d = max(o["s_max"], (ysum + zsum) / max(1, ny + nz)) / o["s_max"]
        s_c = max(o["s_max"], zsum / max(1, nz)) / o["s_max"]
        prim_barrier = max(np.max(np.abs(c), initial=0.0), np.max(np.abs(d - s), initial=0.0))
        # NLP constraint violation (uses d(x), not s)
        dv = np.maximum(0.0, np.maximum(np.where(self.hdL, self.dL - d, 0.0), np.where(self.hdU, d - self.dU, 0.0)))
        prim_nlp = max(np.max(np.abs(c), initial=0.0), np.max(dv, initial=0.0))
        return dict(dual=dual, comp=comp, s_d=s_d, s_c=s_c, prim_b=prim_barrier, prim_nlp=prim_nlp)

    def _unscaled_viol(self, x):
        g = self.nlp.cons(x)
        v = np.abs(g[self.E] - self.cE)
        gl, gu = self.nlp.g_L[self.I], self.nlp.g_U[self.I]
        w = np.maximum(0.0, np.maximum(gl - g[self.I], g[self.I] - gu))
        return max(np.max(v, initial=0.0), np.max(w, initial=0.0))

    # ------------------------------------------------------------ solve
    def solve(self):
        o, nlp = self.o, self.nlp
        self._setup()
        x = self._push(nlp.x0, self.xL, self.xU, self.hxL, self.hxU)
        c, d = self._eval(x)
        s = self._push(d, self.dL, self.dU, self.hdL, self.hdU)
        n, mc, md = nlp.n, self.E.size, self.I.size
        bmi = o["bound_mult_init_val"]
        zL = np.where(self.hxL, bmi, 0.0)
        zU = np.where(self.hxU, bmi, 0.0)
        vL = np.where(self.hdL, bmi, 0.0)
        vU = np.where(self.hdU, bmi, 0.0)
        Jc, Jd = self._jac(x)

        # least-squares multipliers: [I 0 Jc' Jd'; 0 I 0 -I; Jc 0 0 0; Jd -I 0 0]
        gfs = self.sf * nlp.grad_f(x)
        Wls = sp.csr_matrix((n, n))
        inert = self.kkt.factor(Wls, np.ones(n), np.ones(md), Jc, Jd, 0.0, 0.0)
        yc = np.zeros(mc)
        yd = np.zeros(md)
        if inert[1] == mc + md and inert[2] == 0:
            _, _, yc_, yd_ = self.kkt.solve(-(gfs - zL + zU), -(-vL + vU), np.zeros(mc), np.zeros(md))
            # the LS system returns the multipliers in the constraint slots
            if max(np.max(np.abs(yc_), initial=0.0), np.max(np.abs(yd_), initial=0.0)) <= o["constr_mult_init_max"]:
                yc, yd = yc_, yd_

        mu = o["mu_init"]
        tau = max(o["tau_min"], 1.0 - mu)
        theta0 = self._theta(c, d, s)
        theta_max = 1e4 * max(1.0, theta0)
        theta_min = 1e-4 * max(1.0, theta0)
        filt = []
        dw_last = 0.0
        acc_count = 0
        status = 2
        it = 0
        self.n_factor = 0
        for it in range(o["max_iter"] + 1):
            e0 = self._errors(x, s, yc, yd, zL, zU, vL, vU, c, d, Jc, Jd, 0.0)
            nlp_err = max(e0["dual"] / e0["s_d"], e0["prim_nlp"], e0["comp"] / e0["s_c"])
            uviol = self._unscaled_viol(x)
            self.log.append(dict(it=it, mu=mu, err=nlp_err, f=nlp.f(x), theta=self._theta(c, d, s)))
            if (nlp_err <= o["tol"] and e0["dual"] / self.sf <= o["dual_inf_tol"]
                    and uviol <= o["constr_viol_tol"] and e0["comp"] / self.sf <= o["compl_inf_tol"]):
                status = 0
                break
            if (nlp_err <= o["acceptable_tol"] and e0["dual"] / self.sf <= o["acceptable_dual_inf_tol"]
                    and uviol <= o["acceptable_constr_viol_tol"] and e0["comp"] / self.sf <= o["acceptable_compl_inf_tol"]):
                acc_count += 1
                if acc_count >= o["acceptable_iter"]:
                    status = 1
                    break
            else:
                acc_count = 0
            if it == o["max_iter"]:
                status = 2
                break

            # ---- monotone barrier update (fast decrease allowed)
            while True:
                eb = self._errors(x, s, yc, yd, zL, zU, vL, vU, c, d, Jc, Jd, mu)
                berr = max(eb["dual"] / eb["s_d"], eb["prim_b"], eb["comp"] / eb["s_c"])
                if berr > o["kappa_eps"] * mu:
                    break
                new_mu = max(o["tol"] / 10.0, min(o["kappa_mu"] * mu, mu ** o["theta_mu"]))
                if new_mu == mu:
                    break
                mu = new_mu
                tau = max(o["tau_min"], 1.0 - mu)
                filt = []

            # ---- search direction with inertia correction
            Wm = self._hess(x, yc, yd)
            xl, xu, sl, su = self._slacks(x, s)
            Sx = np.where(self.hxL, zL / np.where(self.hxL, xl, 1.0), 0.0) + np.where(self.hxU, zU / np.where(self.hxU, xu, 1.0), 0.0)
            Ss = np.where(self.hdL, vL / np.where(self.hdL, sl, 1.0), 0.0) + np.where(self.hdU, vU / np.where(self.hdU, su, 1.0), 0.0)
            gbx, gbs = self._grad_barrier(x, s, mu)
            rx = gbx + Jc.T @ yc + Jd.T @ yd
            rs = gbs - yd
            rc = c
            rd = d - s
            dw, dc = 0.0, 0.0
            ok = False
            while True:
                pos, neg, zer = self.kkt.factor(Wm, Sx, Ss, Jc, Jd, dw, dc)
                self.n_factor += 1
                if neg == mc + md and zer == 0:
                    ok = True
                    break
                if zer > 0 and dc == 0.0:
                    dc = o["dc_bar"] * mu ** o["kappa_c"]
                    continue
                if dw == 0.0:
                    dw = o["dw0"] if dw_last == 0.0 else max(o["dw_min"], o["kw_minus"] * dw_last)
                else:
                    dw = (o["kw_plus_bar"] if (dw_last == 0.0 or 1e5 * dw_last < dw) else o["kw_plus"]) * dw
                if dw > o["dw_max"]:
                    break
            if not ok:
                status = 4
                break
            if dw > 0.0:
                dw_last = dw
            dx, ds, dyc, dyd = self.kkt.solve(-rx, -rs, -rc, -rd)

            sxl = np.where(self.hxL, xl, 1.0)
            sxu = np.where(self.hxU, xu, 1.0)
            ssl = np.where(self.hdL, sl, 1.0)
            ssu = np.where(self.hdU, su, 1.0)

            def dz_of(dx_, ds_):
                dzL = np.where(self.hxL, (mu - zL * sxl - zL * dx_) / sxl, 0.0)
                dzU = np.where(self.hxU, (mu - zU * sxu + zU * dx_) / sxu, 0.0)
                dvL = np.where(self.hdL, (mu - vL * ssl - vL * ds_) / ssl, 0.0)
                dvU = np.where(self.hdU, (mu - vU * ssu + vU * ds_) / ssu, 0.0)
                return dzL, dzU, dvL, dvU

            def frac_primal(dx_, ds_):
                a = 1.0
                for v, dv, m, sg in ((xl, dx_, self.hxL, 1), (xu, dx_, self.hxU, -1),
                                     (sl, ds_, self.hdL, 1), (su, ds_, self.hdU, -1)):
                    step = sg * dv
                    sel = m & (step < 0)
                    if np.any(sel):
                        a = min(a, np.min(-tau * v[sel] / step[sel]))
                return a

            def frac_dual(dzs):
                a = 1.0
                for z, dz, m in zip((zL, zU, vL, vU), dzs, (self.hxL, self.hxU, self.hdL, self.hdU)):
                    sel = m & (dz < 0)
                    if np.any(sel):
                        a = min(a, np.min(-tau * z[sel] / dz[sel]))
                return a

            # ---- filter line search
            phi = self._barrier(x, s, mu)
            theta = self._theta(c, d, s)
            gBD = gbx @ dx + gbs @ ds
            alpha_max = frac_primal(dx, ds)
            a_min = o["gamma_theta"]
            if gBD < 0:
                a_min = min(o["gamma_theta"], o["gamma_phi"] * theta / (-gBD))
                if theta <= theta_min:
                    a_min = min(a_min, o["delta"] * theta ** o["s_theta"] / (-gBD) ** o["s_phi"])
            a_min *= o["alpha_min_frac"]

            def is_ftype(a):
                return gBD < 0 and a * (-gBD) ** o["s_phi"] > o["delta"] * theta ** o["s_theta"]

            def acceptable(a, xt, st):
                ct, dt = self._eval(xt)
                th_t = self._theta(ct, dt, st)
                if np.any(self._slacks(xt, st)[0][self.hxL] <= 0) or np.any(self._slacks(xt, st)[1][self.hxU] <= 0):
                    return False, th_t
                ph_t = self._barrier(xt, st, mu)
                if not np.isfinite(ph_t) or th_t > theta_max:
                    return False, th_t
                if a > 0 and is_ftype(a) and theta <= theta_min:
                    ok_ = compare_le(ph_t - phi, o["eta_phi"] * a * gBD, phi)
                else:
                    ok_ = (compare_le(th_t, (1 - o["gamma_theta"]) * theta, theta)
                           or compare_le(ph_t - phi, -o["gamma_phi"] * theta, phi))
                if not ok_:
                    return False, th_t
                for (tf, pf) in filt:
                    if not (th_t < tf or ph_t < pf):
                        return False, th_t
                return True, th_t

            alpha = alpha_max
            accepted = False
            step = (dx, ds, dyc, dyd)
            a_primal = alpha
            first = True
            while alpha >= a_min:
                xt, st = x + alpha * dx, s + alpha * ds
                acc, th_t = acceptable(alpha, xt, st)
                if acc:
                    accepted, a_primal, a_test = True, alpha, alpha
                    break
                if first and th_t >= theta and o["max_soc"] > 0:
                    # second-order correction
                    ct, dt = self._eval(xt)
                    c_soc, d_soc = alpha * c + ct, alpha * (d - s) + (dt - st)
                    th_old = theta
                    for _k in range(o["max_soc"]):
                        sx, ss, syc, syd = self.kkt.solve(-rx, -rs, -c_soc, -d_soc)
                        a_soc = frac_primal(sx, ss)
                        xs_, ss_ = x + a_soc * sx, s + a_soc * ss
                        acc, th_soc = acceptable(alpha, xs_, ss_)
                        if acc:
                            accepted, a_primal, a_test = True, a_soc, alpha
                            step = (sx, ss, syc, syd)
                            break
                        if th_soc > o["kappa_soc"] * th_old:
                            break
                        th_old = th_soc
                        cs_, ds_ = self._eval(xs_)
                        c_soc, d_soc = a_soc * c_soc + cs_, a_soc * d_soc + (ds_ - ss_)
                    if accepted:
                        break
                first = False
                alpha *= 0.5
            if not accepted:
                status = 3
                break
            # filter augmentation
            if not (is_ftype(a_test) and compare_le(self._barrier(x + a_primal * step[0], s + a_primal * step[1], mu) - phi,
                                                       o["eta_phi"] * a_test * gBD, phi)):
                filt.append(((1 - o["gamma_theta"]) * theta, phi - o["gamma_phi"] * theta))

            dx, ds, dyc, dyd = step
            dzs = dz_of(dx, ds)
            a_dual = frac_dual(dzs)
            x = x + a_primal * dx
            s = s + a_primal * ds
            yc = yc + a_primal * dyc
            yd = yd + a_primal * dyd
            zL = zL + a_dual * dzs[0]
            zU = zU + a_dual * dzs[1]
            vL = vL + a_dual * dzs[2]
            vU = vU + a_dual * dzs[3]
            # kappa_Sigma safeguard
            ks = o["kappa_sigma"]
            xl, xu, sl, su = self._slacks(x, s)
            for z, v, m in ((zL, xl, self.hxL), (zU, xu, self.hxU), (vL, sl, self.hdL), (vU, su, self.hdU)):
                z[m] = np.maximum(np.minimum(z[m], ks * mu / v[m]), mu / (ks * v[m]))
            c, d = self._eval(x)
            Jc, Jd = self._jac(x)

        # honor_original_bounds
        xf = x.copy()
        lo, hi = nlp.x_L, nlp.x_U
        xf = np.where(np.isfinite(lo), np.maximum(xf, lo), xf)
        xf = np.where(np.isfinite(hi), np.minimum(xf, hi), xf)
        self.iters = it
        self.status = status
        self.x = xf
        self.mu = mu
        self.yc, self.yd = yc, yd
        return dict(status=status, status_str=STATUS[status], success=status in (0, 1), iters=it,
                    x=xf, f=nlp.f(xf), yc=yc, yd=yd)
