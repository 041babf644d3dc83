"""Oracle: numpy restatement of the point-formulation OBCA NLP of
R/obca_py/optimizer_points.py.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows optimizer_points.py line by line:

* vehicle vertices ....................... get_vehicle_vertices :35-50 (done by the
                                           caller: inst["vertices"], convex hull)
* variable order, x0 and bounds ........... initialize_manual :52-108, generate_variable :229-255
                                           X (5N), U (2(N-1)), LAMBDA obstacle-major
                                           (index N*sum_{j'<j} n_j' + i*n_j + e)
* constraint order and bounds ............. generate_constrain :257-327
                                           X0 = init, Euler dynamics, X_{N-1} = end (hard),
                                           then per obstacle j, step i, vertex k:
                                           ||A'lam||^2 in [0, 1] and (A(R v_k + t) - b).lam in
                                           [MIN_DISTANCE_TO_OBS, 100000]
* objective ............................... generate_object :193-227
                                           sum_{i<N-2} dsr^2 + da^2 + sum_{i<N-1} 20 (v_i dT)^2
The reference ignores init_dual_var (LAMBDA starts at 0.1) and never reads
`r`, `q`; both are kept that way.

Instance format (plain dict):
    init_traj (N,5), obs_A list of (e_j,2), obs_b list of (e_j,), vertices (KV,2),
    dT, wheelbase, max_steer, max_velocity, max_accel, max_steer_rate, min_dist,
    x_bound (2,), y_bound (2,), optional init_control (N-1,2)
"""
import numpy as np
import scipy.sparse as sp

from .nlp import NC, NS, dynamics, dynamics_hess, dynamics_jac

LAMBDA_MAX = 100000.0   # optimizer_points.py:255
DIST_MAX = 100000.0     # optimizer_points.py:327


class PointNLP:
    """The NLP exactly as optimizer_points.py hands it to nlpsol (:157-173)."""

    topt = False

    def __init__(self, inst):
        self.inst = inst
        tr = np.asarray(inst["init_traj"], dtype=np.float64)
        self.N = N = tr.shape[0]
        if N < 1:
            raise ValueError("empty init guess")  # build_model :118-120
        self.dT = float(inst["dT"])
        self.L = float(inst["wheelbase"])
        self.A = [np.asarray(a, dtype=np.float64) for a in inst["obs_A"]]
        self.b = [np.asarray(a, dtype=np.float64) for a in inst["obs_b"]]
        self.V = np.asarray(inst["vertices"], dtype=np.float64)
        self.M, self.KV = len(self.A), self.V.shape[0]
        self.eo = np.array([a.shape[0] for a in self.A], dtype=int)
        self.TEo = int(self.eo.sum())
        self.off_o = np.concatenate([[0], np.cumsum(self.eo)[:-1]]).astype(int)

        self.oU = NS * N
        self.oLAM = self.oU + NC * (N - 1)
        self.n = self.oLAM + N * self.TEo
        self.gDyn = NS
        self.gTerm = NS + NS * (N - 1)
        self.gCol = self.gTerm + NS
        self.nblk = N * self.M
        self.m = self.gCol + 2 * self.KV * self.nblk
        self.blocks = [(j, i, self.oLAM + N * self.off_o[j] + i * self.eo[j])
                       for j in range(self.M) for i in range(N)]
        self._build_bounds()
        self._build_x0()

    def _build_bounds(self):
        inst, N = self.inst, self.N
        xb = inst.get("x_bound", [-9999999, 9999999])
        yb = inst.get("y_bound", [-9999999, 9999999])
        vmax, smax = inst["max_velocity"], inst["max_steer"]
        amax, wmax = inst["max_accel"], inst["max_steer_rate"]
        lb = np.empty(self.n)
        ub = np.empty(self.n)
        lb[:NS * N] = np.tile([xb[0], yb[0], -vmax, -2 * np.pi, -smax], N)
        ub[:NS * N] = np.tile([xb[1], yb[1], vmax, 2 * np.pi, smax], N)
        lb[self.oU:self.oLAM] = np.tile([-amax, -wmax], N - 1)
        ub[self.oU:self.oLAM] = np.tile([amax, wmax], N - 1)
        lb[self.oLAM:] = 0.0
        ub[self.oLAM:] = LAMBDA_MAX
        self.x_L, self.x_U = lb, ub
        self.dmin = float(inst["min_dist"])
        gl = np.zeros(self.m)
        gu = np.zeros(self.m)
        r = self.gCol + 2 * np.arange(self.KV * self.nblk)
        gl[r], gu[r] = 0.0, 1.0
        gl[r + 1], gu[r + 1] = self.dmin, DIST_MAX
        self.g_L, self.g_U = gl, gu

    def _build_x0(self):
        inst, N = self.inst, self.N
        tr = np.asarray(inst["init_traj"], dtype=np.float64)
        x0 = np.zeros(self.n)
        x0[:NS * N] = tr.reshape(-1)
        ic = inst.get("init_control")
        if ic is not None:
            x0[self.oU:self.oLAM] = np.asarray(ic, dtype=np.float64).reshape(-1)
        x0[self.oLAM:] = 0.1
        self.x0 = x0
        self.init_state = tr[0].copy()
        self.end_state = tr[-1].copy()

    # --------------------------------------------------------------- helpers
    def split(self, x):
        X = x[:NS * self.N].reshape(self.N, NS)
        U = x[self.oU:self.oLAM].reshape(self.N - 1, NC)
        return X, U

    def _stage_w(self, x):
        X, U = self.split(x)
        return np.hstack([X[:-1], U])

    def _block_vals(self, x):
        X, _ = self.split(x)
        for p, (j, i, la0) in enumerate(self.blocks):
            A, b = self.A[j], self.b[j]
            la = x[la0:la0 + len(b)]
            yield p, j, i, la0, A, b, la, X[i]

    @staticmethod
    def _rot(th):
        c, s = np.cos(th), np.sin(th)
        return c, s, np.array([[c, -s], [s, c]]), np.array([[-s, -c], [c, -s]])

    # ------------------------------------------------------------- objective
    def f(self, x):
        X, U = self.split(x)
        obj = 0.0
        if self.N > 2:
            du = U[1:] - U[:-1]
            obj += float(np.sum(du[:, 1] * du[:, 1] + du[:, 0] * du[:, 0]))
        obj += float(np.sum((X[:-1, 2] * self.dT) ** 2 * 20))
        return obj

    def grad_f(self, x):
        X, U = self.split(x)
        g = np.zeros(self.n)
        gU = np.zeros_like(U)
        if self.N > 2:
            du = U[1:] - U[:-1]
            gU[1:] += 2.0 * du
            gU[:-1] -= 2.0 * du
        g[self.oU:self.oLAM] = gU.reshape(-1)
        g[2:NS * (self.N - 1):NS] = 40.0 * X[:-1, 2] * self.dT * self.dT
        return g

    # ----------------------------------------------------------- constraints
    def cons(self, x):
        N = self.N
        X, _ = self.split(x)
        out = np.zeros(self.m)
        out[:NS] = X[0] - self.init_state
        if N > 1:
            F = dynamics(self._stage_w(x), self.dT, self.L, False)
            out[self.gDyn:self.gTerm] = (X[1:] - F).reshape(-1)
        out[self.gTerm:self.gCol] = X[-1] - self.end_state
        for p, j, i, la0, A, b, la, st in self._block_vals(x):
            _, _, R, _ = self._rot(st[3])
            w = A.T @ la
            for k in range(self.KV):
                vt = R @ self.V[k] + st[:2]
                r = self.gCol + 2 * (self.KV * p + k)
                out[r] = w @ w
                out[r + 1] = (A @ vt - b) @ la
        return out

    def jac(self, x):
        N = self.N
        rows, cols, vals = [], [], []

        def put(r, c, v):
            rows.append(np.atleast_1d(r))
            cols.append(np.atleast_1d(c))
            vals.append(np.atleast_1d(np.asarray(v, dtype=np.float64)))

        put(np.arange(NS), np.arange(NS), np.ones(NS))
        if N > 1:
            Jd = dynamics_jac(self._stage_w(x), self.dT, self.L, False)
            nw = Jd.shape[2]
            for i in range(N - 1):
                r0 = self.gDyn + NS * i
                put(r0 + np.arange(NS), NS * (i + 1) + np.arange(NS), np.ones(NS))
                cidx = np.array(list(NS * i + np.arange(NS)) + [self.oU + NC * i, self.oU + NC * i + 1])
                put(np.repeat(r0 + np.arange(NS), nw), np.tile(cidx, NS), -Jd[i].reshape(-1))
        put(self.gTerm + np.arange(NS), NS * (N - 1) + np.arange(NS), np.ones(NS))
        for p, j, i, la0, A, b, la, st in self._block_vals(x):
            _, _, R, dR = self._rot(st[3])
            w = A.T @ la
            lai = la0 + np.arange(len(b))
            for k in range(self.KV):
                r = self.gCol + 2 * (self.KV * p + k)
                vt = R @ self.V[k] + st[:2]
                put(np.full(len(b), r), lai, 2.0 * A @ w)
                put(np.full(len(b), r + 1), lai, A @ vt - b)
                put([r + 1, r + 1, r + 1], [NS * i, NS * i + 1, NS * i + 3], [w[0], w[1], w @ (dR @ self.V[k])])
        Jm = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                           shape=(self.m, self.n))
        return Jm.tocsr()

    def hess(self, x, y, obj_factor=1.0):
        N = self.N
        X, _ = self.split(x)
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
        for i in range(N - 1):
            add(NS * i + 2, NS * i + 2, sig * 40.0 * self.dT * self.dT)
        I2 = 2.0 * np.eye(NC)
        for i in range(N - 2):
            ui = self.oU + NC * i + np.arange(NC)
            uj = ui + NC
            add(ui[:, None], ui[None, :], sig * I2)
            add(uj[:, None], uj[None, :], sig * I2)
            add(ui[:, None], uj[None, :], -sig * I2)
            add(uj[:, None], ui[None, :], -sig * I2)
        if N > 1:
            Yd = y[self.gDyn:self.gTerm].reshape(N - 1, NS)
            Hd = dynamics_hess(self._stage_w(x), -Yd, self.dT, self.L, False)
            for i in range(N - 1):
                ci = np.array(list(NS * i + np.arange(NS)) + [self.oU + NC * i, self.oU + NC * i + 1])
                add(ci[:, None], ci[None, :], Hd[i])
        for p, j, i, la0, A, b, la, st in self._block_vals(x):
            _, _, R, dR = self._rot(st[3])
            w = A.T @ la
            lai = la0 + np.arange(len(b))
            th = NS * i + 3
            for k in range(self.KV):
                r = self.gCol + 2 * (self.KV * p + k)
                y1, y3 = y[r], y[r + 1]
                add(lai[:, None], lai[None, :], y1 * 2.0 * A @ A.T)
                dv = dR @ self.V[k]
                for c in range(2):
                    add(lai, NS * i + c, y3 * A[:, c])
                    add(NS * i + c, lai, y3 * A[:, c])
                add(lai, th, y3 * (A @ dv))
                add(th, lai, y3 * (A @ dv))
                add(th, th, -y3 * (w @ (R @ self.V[k])))
        Hm = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                           shape=(self.n, self.n))
        return Hm.tocsr()

    def counts(self):
        eq = int(np.sum(self.g_L == self.g_U))
        return {"n_var": self.n, "n_eq": eq, "n_ineq": self.m - eq}

    def unpack(self, x):
        """solve :175-191 slicing: x/y/v/theta/steer_opt, a_opt, steerate_opt."""
        X, U = self.split(x)
        return {"x_opt": X[:, 0].copy(), "y_opt": X[:, 1].copy(), "v_opt": X[:, 2].copy(),
                "theta_opt": X[:, 3].copy(), "steer_opt": X[:, 4].copy(),
                "a_opt": U[:, 0].copy(), "steerate_opt": U[:, 1].copy(),
                "lambda_opt": x[self.oLAM:].copy()}
