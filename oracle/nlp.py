"""Oracle: numpy restatement of the OBCA NLP of R/obca_py/optimizer.py.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Everything below follows optimizer.py line by line:

* variable order, x0 and bounds ............ set_initial_guess :228-290,
                                             generate_variables :292-354
* constraint order and bounds ............... generate_constraints :356-425
* objective ................................. generate_objective :427-473
* dynamics (Euler / RK2-midpoint w/ time scale) kinematic_model :9-36, :364-377

Derivatives: dynamics by sympy (exact symbolic differentiation of the same
expressions), collision constraints and objective by hand; every derivative
is checked against finite differences in tests/test_oracle_nlp.py.

Instance format (plain dict, shared by tests / bench / shim):
    init_traj (N,5) float64 [x, y, v, theta, steer]
    obs_A list of (e_m,2), obs_b list of (e_m,)      obstacle halfspaces
    body_G list of (e_n,2), body_g list of (e_n,)    vehicle-body halfspaces
    dT, Q (2,2), R (2,2), W (2,2), wheelbase, max_steer, max_velocity,
    max_accel, max_steer_rate, min_dist, x_bound (2,), y_bound (2,)
    optional: init_control (N-1,2), init_mu (N,mu_count), init_lambda (N,lam_count)
"""
import functools

import numpy as np
import scipy.sparse as sp
import sympy

from oracle import libm

NS, NC = 5, 2
SLACK_WEIGHT = 5000.0  # optimizer.py:472


# --------------------------------------------------------------------------
# dynamics: optimizer.py:9-36 (f) and :364-377 (Euler / RK2 midpoint)
# --------------------------------------------------------------------------
@functools.lru_cache(maxsize=None)
def _dyn_funcs(topt):
    px, py, v, th, de, a, om, tau, dT, L = sympy.symbols("px py v th de a om tau dT L")
    ys = sympy.symbols("y0:5")
    x = sympy.Matrix([px, py, v, th, de])
    u = sympy.Matrix([a, om])

    def f(s, c):
        return sympy.Matrix([s[2] * sympy.cos(s[3]), s[2] * sympy.sin(s[3]), c[0],
                             s[2] * sympy.tan(s[4]) / L, c[1]])

    if topt:
        h = dT * tau
        F = x + h * f(x + sympy.Rational(1, 2) * h * f(x, u), u)
        w = [px, py, v, th, de, a, om, tau]
    else:
        F = x + dT * f(x, u)
        w = [px, py, v, th, de, a, om]
    J = F.jacobian(w)
    phi = sum(ys[k] * F[k] for k in range(5))
    H = sympy.hessian(phi, w)
    args = w + [dT, L] + list(ys)
    mods = [{"sin": libm.sin, "cos": libm.cos, "tan": libm.tan}, "numpy"]   # oracle/libm.py: numpy or glibc
    fF = sympy.lambdify(args, list(F), mods)
    fJ = sympy.lambdify(args, [J[i, j] for i in range(5) for j in range(len(w))], mods)
    fH = sympy.lambdify(args, [H[i, j] for i in range(len(w)) for j in range(len(w))], mods)
    return fF, fJ, fH, len(w)


def _bcast(vals, shape):
    return np.stack([np.broadcast_to(np.asarray(vv, dtype=np.float64), shape) for vv in vals], axis=-1)


def dynamics(W, dT, L, topt):
    """W: (k, 7|8) stage vectors [x(5), u(2), (tau)] -> F (k,5)."""
    fF, _, _, nw = _dyn_funcs(bool(topt))
    args = [W[:, j] for j in range(nw)] + [dT, L] + [0.0] * 5
    return _bcast(fF(*args), (W.shape[0],))


def dynamics_jac(W, dT, L, topt):
    fF, fJ, _, nw = _dyn_funcs(bool(topt))
    args = [W[:, j] for j in range(nw)] + [dT, L] + [0.0] * 5
    return _bcast(fJ(*args), (W.shape[0],)).reshape(W.shape[0], 5, nw)


def dynamics_hess(W, Y, dT, L, topt):
    """sum_k Y[:,k] * d2F_k/dw2 -> (k, nw, nw)."""
    _, _, fH, nw = _dyn_funcs(bool(topt))
    args = [W[:, j] for j in range(nw)] + [dT, L] + [Y[:, k] for k in range(5)]
    return _bcast(fH(*args), (W.shape[0],)).reshape(W.shape[0], nw, nw)


# --------------------------------------------------------------------------
class ObcaNLP:
    """The NLP exactly as optimizer.py hands it to nlpsol (:476-507)."""

    def __init__(self, inst):
        self.inst = inst
        tr = np.asarray(inst["init_traj"], dtype=np.float64)
        self.N = N = tr.shape[0]
        if N < 1:
            raise Exception("[OBCA] Initial guess is empty!")  # optimizer.py:233-234
        self.dT = float(inst["dT"])
        self.Q = np.asarray(inst["Q"], dtype=np.float64)
        self.R = np.asarray(inst["R"], dtype=np.float64)
        self.W = np.asarray(inst["W"], dtype=np.float64)
        self.topt = self.W[1, 1] != 0  # optimizer.py:109
        self.L = float(inst["wheelbase"])
        self.A = [np.asarray(a, dtype=np.float64) for a in inst["obs_A"]]
        self.b = [np.asarray(a, dtype=np.float64) for a in inst["obs_b"]]
        self.G = [np.asarray(a, dtype=np.float64) for a in inst["body_G"]]
        self.gb = [np.asarray(a, dtype=np.float64) for a in inst["body_g"]]
        self.M, self.K = len(self.A), len(self.G)
        self.eo = np.array([a.shape[0] for a in self.A], dtype=int)
        self.eb = np.array([a.shape[0] for a in self.G], dtype=int)
        self.TEo, self.TEb = int(self.eo.sum()), int(self.eb.sum())
        self.off_o = np.concatenate([[0], np.cumsum(self.eo)[:-1]]).astype(int)
        self.off_b = np.concatenate([[0], np.cumsum(self.eb)[:-1]]).astype(int)
        self.mu_count = self.TEb * self.M  # optimizer.py:267
        self.lam_count = self.TEo * self.K  # optimizer.py:268

        # variable offsets (optimizer.py:292-354)
        self.oX = 0
        self.oU = NS * N
        self.oMU = self.oU + NC * (N - 1)
        self.oLAM = self.oMU + N * self.mu_count
        self.oTAU = self.oLAM + N * self.lam_count
        self.oS = self.oTAU + ((N - 1) if self.topt else 0)
        self.n = self.oS + NS

        # constraint offsets (optimizer.py:356-425)
        self.gDyn = NS
        self.gTerm = NS + NS * (N - 1)
        self.gCol = self.gTerm + NS
        self.npair = N * self.M * self.K
        self.m = self.gCol + 4 * self.npair

        self._build_pairs()
        self._build_bounds()
        self._build_x0()

    # ---------------------------------------------------------------- layout
    def _build_pairs(self):
        N, M, K = self.N, self.M, self.K
        P = []
        for i in range(N):
            for m in range(M):
                for n in range(K):
                    mu0 = self.oMU + i * self.mu_count + m * self.TEb + self.off_b[n]
                    la0 = self.oLAM + i * self.lam_count + n * self.TEo + self.off_o[m]
                    P.append((i, m, n, mu0, la0))
        self.pairs = P
        # pairs of one (obstacle m, body n) share A, b, G, g: the vectorised loops run per group
        pi = np.array([q[0] for q in P], dtype=int)
        self.pgroups = []
        for m in range(M):
            for n in range(K):
                sel = np.arange(len(P))[m * K + n::M * K]
                self.pgroups.append((m, n, sel, pi[sel], np.array([P[q][3] for q in sel], dtype=int),
                                     np.array([P[q][4] for q in sel], dtype=int)))

    def _build_bounds(self):
        inst, N = self.inst, self.N
        xb = inst.get("x_bound", [-np.inf, np.inf])
        yb = inst.get("y_bound", [-np.inf, np.inf])
        if xb[1] < xb[0]:
            raise Exception("[OBCA] The x_bound is infeasible!")
        if yb[1] < yb[0]:
            raise Exception("[OBCA] The y_bound is infeasible!")
        vmax = abs(inst["max_velocity"])
        smax = abs(inst["max_steer"])
        amax = abs(inst["max_accel"])
        wmax = abs(inst["max_steer_rate"])
        lb = np.full(self.n, -np.inf)
        ub = np.full(self.n, np.inf)
        st_lb = np.array([xb[0], yb[0], -vmax, -2 * np.pi, -smax])
        st_ub = np.array([xb[1], yb[1], vmax, 2 * np.pi, smax])
        lb[: NS * N] = np.tile(st_lb, N)
        ub[: NS * N] = np.tile(st_ub, N)
        lb[self.oU:self.oMU] = np.tile([-amax, -wmax], N - 1)
        ub[self.oU:self.oMU] = np.tile([amax, wmax], N - 1)
        lb[self.oMU:self.oTAU] = 0.0
        if self.topt:
            lb[self.oTAU:self.oS] = 0.05 / self.dT
            ub[self.oTAU:self.oS] = 1.0
        self.x_L, self.x_U = lb, ub

        dmin = inst.get("min_dist", 0.1)
        if dmin is None or dmin < 0:
            dmin = 0.1
        gl = np.zeros(self.m)
        gu = np.zeros(self.m)
        c = self.gCol + 4 * np.arange(self.npair)
        gl[c + 0], gu[c + 0] = 0.0, 1.0
        gl[c + 3], gu[c + 3] = dmin, np.inf
        self.g_L, self.g_U = gl, gu
        self.dmin = dmin

    def _build_x0(self):
        inst, N = self.inst, self.N
        tr = np.asarray(inst["init_traj"], dtype=np.float64)
        x0 = np.zeros(self.n)
        x0[: NS * N] = tr.reshape(-1)
        ic = inst.get("init_control")
        if ic is not None:
            ic = np.asarray(ic, dtype=np.float64)
            if ic.shape != (N - 1, NC):
                raise Exception("[OBCA] The control input dimension does not match!")
            x0[self.oU:self.oMU] = ic.reshape(-1)
        imu, ilam = inst.get("init_mu"), inst.get("init_lambda")
        if imu is None:
            x0[self.oMU:self.oTAU] = 0.1
        else:
            imu, ilam = np.asarray(imu), np.asarray(ilam)
            if imu.shape != (N, self.mu_count) or ilam.shape != (N, self.lam_count):
                raise Exception("[OBCA] The dual variable dimension does not match!")
            x0[self.oMU:self.oLAM] = imu.reshape(-1)
            x0[self.oLAM:self.oTAU] = ilam.reshape(-1)
        if self.topt:
            x0[self.oTAU:self.oS] = 1.0
        self.x0 = x0
        self.init_state = tr[0].copy()
        self.end_state = tr[-1].copy()

    # --------------------------------------------------------------- helpers
    def split(self, x):
        N = self.N
        X = x[: NS * N].reshape(N, NS)
        U = x[self.oU:self.oMU].reshape(N - 1, NC)
        tau = x[self.oTAU:self.oS] if self.topt else np.ones(N - 1)
        s = x[self.oS:self.oS + NS]
        return X, U, tau, s

    def _stage_w(self, x):
        X, U, tau, _ = self.split(x)
        cols = [X[:-1], U] + ([tau[:, None]] if self.topt else [])
        return np.hstack(cols)

    def _pair_vals(self, x):
        """Per-pair (w = A^T lam, A t - b, mu, lam) for the collision rows."""
        X = x[: NS * self.N].reshape(self.N, NS)
        out = []
        for (i, m, n, mu0, la0) in self.pairs:
            A, b, G, g = self.A[m], self.b[m], self.G[n], self.gb[n]
            mu = x[mu0:mu0 + len(g)]
            la = x[la0:la0 + len(b)]
            out.append((i, m, n, mu0, la0, A, b, G, g, mu, la, X[i]))
        return out

    # ------------------------------------------------------------- objective
    def f(self, x):
        N, dT, Wm = self.N, self.dT, self.W
        X, U, tau, s = self.split(x)
        h = dT * tau if self.topt else np.full(N - 1, dT)
        obj = 0.0
        if self.topt:
            obj += np.sum(h * Wm[1, 1])
        obj += np.einsum("ij,jk,ik->", U, self.Q, U)
        if N > 2:
            jerk = (U[1:] - U[:-1]) / h[:-1, None]
            obj += np.einsum("ij,jk,ik->", jerk, self.R, jerk)
        obj += np.sum((X[:-1, 2] * h) ** 2) * Wm[0, 0]
        obj += SLACK_WEIGHT * np.dot(s, s)
        return float(obj)

    def grad_f(self, x):
        N, dT, Wm = self.N, self.dT, self.W
        X, U, tau, s = self.split(x)
        h = dT * tau if self.topt else np.full(N - 1, dT)
        gr = np.zeros(self.n)
        gU = U @ (self.Q + self.Q.T)
        gtau = np.zeros(N - 1)
        if self.topt:
            gtau += dT * Wm[1, 1]
        if N > 2:
            Rs = self.R + self.R.T
            du = U[1:] - U[:-1]
            hh = h[:-1]
            gj = (du @ Rs) / (hh ** 2)[:, None]
            gU[1:] += gj
            gU[:-1] -= gj
            if self.topt:
                Jv = np.einsum("ij,jk,ik->i", du, self.R, du) / hh ** 2
                gtau[:-1] += -2.0 * Jv / tau[:-1]
        v = X[:-1, 2]
        gv = 2.0 * Wm[0, 0] * v * h ** 2
        if self.topt:
            gtau += 2.0 * Wm[0, 0] * v ** 2 * dT ** 2 * tau
        gr[self.oU:self.oMU] = gU.reshape(-1)
        gr[2:NS * (N - 1):NS] = gv
        if self.topt:
            gr[self.oTAU:self.oS] = gtau
        gr[self.oS:self.oS + NS] = 2.0 * SLACK_WEIGHT * s
        return gr

    # ----------------------------------------------------------- constraints
    def cons(self, x):
        N = self.N
        X, U, tau, s = self.split(x)
        out = np.zeros(self.m)
        out[:NS] = X[0] - self.init_state
        if N > 1:
            F = dynamics(self._stage_w(x), self.dT, self.L, self.topt)
            out[self.gDyn:self.gTerm] = (X[1:] - F).reshape(-1)
        out[self.gTerm:self.gCol] = X[-1] - self.end_state + s
        for (m, n, sel, i, mu0, la0) in self.pgroups:
            A, b, G, g = self.A[m], self.b[m], self.G[n], self.gb[n]
            la = x[la0[:, None] + np.arange(len(b))]
            mu = x[mu0[:, None] + np.arange(len(g))]
            st = X[i]
            w = la @ A
            c, sn = libm.cos(st[:, 3]), libm.sin(st[:, 3])
            r = self.gCol + 4 * sel
            out[r] = w[:, 0] * w[:, 0] + w[:, 1] * w[:, 1]
            out[r + 1] = mu @ G[:, 0] + (c * w[:, 0] + sn * w[:, 1])
            out[r + 2] = mu @ G[:, 1] + (-sn * w[:, 0] + c * w[:, 1])
            out[r + 3] = -(mu @ g) + np.einsum("pj,pj->p", st[:, :2] @ A.T - b, la)
        return out

    def jac(self, x):
        """Sparse (m x n) Jacobian of g."""
        N = self.N
        rows, cols, vals = [], [], []

        def put(r, c, v):
            rows.append(np.ravel(r))
            cols.append(np.ravel(c))
            vals.append(np.ravel(np.asarray(v, dtype=np.float64)))

        put(np.arange(NS), np.arange(NS), np.ones(NS))
        if N > 1:
            Wst = self._stage_w(x)
            Jd = dynamics_jac(Wst, self.dT, self.L, self.topt)  # (N-1,5,nw)
            nw = Jd.shape[2]
            for i in range(N - 1):
                r0 = self.gDyn + NS * i
                put(r0 + np.arange(NS), NS * (i + 1) + np.arange(NS), np.ones(NS))
                cidx = list(NS * i + np.arange(NS)) + [self.oU + NC * i, self.oU + NC * i + 1]
                if self.topt:
                    cidx.append(self.oTAU + i)
                rr = np.repeat(r0 + np.arange(NS), nw)
                cc = np.tile(np.array(cidx), NS)
                put(rr, cc, -Jd[i].reshape(-1))
        put(self.gTerm + np.arange(NS), NS * (N - 1) + np.arange(NS), np.ones(NS))
        put(self.gTerm + np.arange(NS), self.oS + np.arange(NS), np.ones(NS))
        X = x[: NS * N].reshape(N, NS)
        for (m, n, sel, i, mu0, la0) in self.pgroups:
            A, b, G, g = self.A[m], self.b[m], self.G[n], self.gb[n]
            em, en = len(b), len(g)
            la = x[la0[:, None] + np.arange(em)]
            st = X[i]
            w = la @ A
            c, sn = libm.cos(st[:, 3]), libm.sin(st[:, 3])
            r = (self.gCol + 4 * sel)[:, None]
            lai = la0[:, None] + np.arange(em)
            mui = mu0[:, None] + np.arange(en)
            one_e, one_n = np.ones((1, em)), np.ones((1, en))
            put((r * one_e).ravel(), lai.ravel(), (2.0 * w @ A.T).ravel())
            put((r + 1) * one_n, mui, np.broadcast_to(G[:, 0], mui.shape))
            put((r + 2) * one_n, mui, np.broadcast_to(G[:, 1], mui.shape))
            put((r + 1) * one_e, lai, c[:, None] * A[:, 0] + sn[:, None] * A[:, 1])
            put((r + 2) * one_e, lai, -sn[:, None] * A[:, 0] + c[:, None] * A[:, 1])
            put(r[:, 0] + 1, NS * i + 3, -sn * w[:, 0] + c * w[:, 1])
            put(r[:, 0] + 2, NS * i + 3, -c * w[:, 0] - sn * w[:, 1])
            put((r + 3) * one_n, mui, np.broadcast_to(-g, mui.shape))
            put((r + 3) * one_e, lai, st[:, :2] @ A.T - b)
            put(np.repeat(r[:, 0] + 3, 2), (NS * i[:, None] + np.arange(2)).ravel(), w.ravel())
        Jm = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                           shape=(self.m, self.n))
        return Jm.tocsr()

    # --------------------------------------------------------------- Hessian
    def hess(self, x, y, obj_factor=1.0):
        """Full symmetric sparse Hessian of obj_factor*f + y^T g."""
        N, dT, Wm = self.N, self.dT, self.W
        X, U, tau, s = self.split(x)
        rows, cols, vals = [], [], []

        def add(r, c, v):
            r = np.atleast_1d(r)
            c = np.atleast_1d(c)
            v = np.broadcast_to(np.asarray(v, dtype=np.float64), np.broadcast(r, c).shape)
            rr, cc = np.broadcast_arrays(r, c)
            rows.append(rr.ravel())
            cols.append(cc.ravel())
            vals.append(v.ravel())

        sig = obj_factor
        h = dT * tau if self.topt else np.full(N - 1, dT)
        Qs = self.Q + self.Q.T
        Rs = self.R + self.R.T
        for i in range(N - 1):
            ui = self.oU + NC * i + np.arange(NC)
            add(ui[:, None], ui[None, :], sig * Qs)
            vi = NS * i + 2
            add(vi, vi, sig * 2.0 * Wm[0, 0] * h[i] ** 2)
            if self.topt:
                ti = self.oTAU + i
                add(ti, ti, sig * 2.0 * Wm[0, 0] * X[i, 2] ** 2 * dT ** 2)
                add([vi, ti], [ti, vi], sig * 4.0 * Wm[0, 0] * X[i, 2] * dT ** 2 * tau[i])
        for i in range(N - 2):
            ui = self.oU + NC * i + np.arange(NC)
            uj = ui + NC
            hh = h[i]
            blk = Rs / hh ** 2
            add(ui[:, None], ui[None, :], sig * blk)
            add(uj[:, None], uj[None, :], sig * blk)
            add(ui[:, None], uj[None, :], -sig * blk)
            add(uj[:, None], ui[None, :], -sig * blk)
            if self.topt:
                ti = self.oTAU + i
                du = U[i + 1] - U[i]
                Jv = du @ self.R @ du / hh ** 2
                add(ti, ti, sig * 6.0 * Jv / tau[i] ** 2)
                gdu = -2.0 * (Rs @ du) / (hh ** 2 * tau[i])  # d2/(d du d tau)
                add(uj, ti, sig * gdu)
                add(ti, uj, sig * gdu)
                add(ui, ti, -sig * gdu)
                add(ti, ui, -sig * gdu)
        add(self.oS + np.arange(NS), self.oS + np.arange(NS), sig * 2.0 * SLACK_WEIGHT)

        if N > 1:
            Wst = self._stage_w(x)
            Yd = y[self.gDyn:self.gTerm].reshape(N - 1, NS)
            Hd = dynamics_hess(Wst, -Yd, self.dT, self.L, self.topt)  # rows are x_{i+1} - F
            for i in range(N - 1):
                cidx = list(NS * i + np.arange(NS)) + [self.oU + NC * i, self.oU + NC * i + 1]
                if self.topt:
                    cidx.append(self.oTAU + i)
                ci = np.array(cidx)
                add(ci[:, None], ci[None, :], Hd[i])

        for (m, n, sel, i, mu0, la0) in self.pgroups:
            A, b = self.A[m], self.b[m]
            em = len(b)
            r = self.gCol + 4 * sel
            y1, y2a, y2b, y3 = y[r], y[r + 1], y[r + 2], y[r + 3]
            la = x[la0[:, None] + np.arange(em)]
            w = la @ A
            c, sn = libm.cos(X[i, 3]), libm.sin(X[i, 3])
            lai = la0[:, None] + np.arange(em)
            th = NS * i + 3
            AA = 2.0 * A @ A.T
            add(lai[:, :, None], lai[:, None, :], y1[:, None, None] * AA)
            # d/dlam of y2^T dR^T/dth A^T lam:  dR^T' y2 = [-sn y2a - c y2b, c y2a - sn y2b]
            gx, gy = -sn * y2a - c * y2b, c * y2a - sn * y2b
            v_thl = gx[:, None] * A[:, 0] + gy[:, None] * A[:, 1]
            add(lai, th[:, None], v_thl)
            add(th[:, None], lai, v_thl)
            # d2/dth2: -y2^T R^T w
            add(th, th, -(y2a * (c * w[:, 0] + sn * w[:, 1]) + y2b * (-sn * w[:, 0] + c * w[:, 1])))
            for k in range(2):
                add(lai, (NS * i + k)[:, None], y3[:, None] * A[:, k])
                add((NS * i + k)[:, None], lai, y3[:, None] * A[:, k])
        Hm = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                           shape=(self.n, self.n))
        return Hm.tocsr()

    # --------------------------------------------------------------- counts
    def counts(self):
        eq = int(np.sum(self.g_L == self.g_U))
        return {"n_var": self.n, "n_eq": eq, "n_ineq": self.m - eq}

    def unpack(self, x):
        """Solution dict slicing as optimizer.py:514-569."""
        N = self.N
        X, U, tau, s = self.split(x)
        return {
            "x_opt": X[:, 0].copy(), "y_opt": X[:, 1].copy(), "v_opt": X[:, 2].copy(),
            "theta_opt": X[:, 3].copy(), "steer_angle_opt": X[:, 4].copy(),
            "accel_opt": U[:, 0].copy(), "steer_rate_opt": U[:, 1].copy(),
            "mu_opt": x[self.oMU:self.oLAM].reshape(N, self.mu_count).copy(),
            "lambda_opt": x[self.oLAM:self.oTAU].reshape(N, self.lam_count).copy(),
            "time_scale_opt": (tau.copy() if self.topt else np.ones(N - 1)),
            "slack_opt": s.copy(),
        }
