"""Oracle: structure-exploiting solve of the IPOPT augmented system for the
OBCA NLP (oracle/nlp.py layout).  Same interface as ipm.DenseKKT.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  It is the numpy blueprint
of the HIP kernel's linear algebra and the CPU baseline at full config sizes.

Elimination order (each step is a Schur complement, so by Sylvester's law the
inertia of the full matrix is the sum of the inertias of the eliminated
blocks -- the exact inertia IPOPT/MUMPS reports, whenever every eliminated
block is nonsingular):

 1. inequality slacks s (Ds = Sigma_s + dw > 0)      -> +m_d positive
    inequality multipliers y_d (-(1/Ds + dc) < 0)     -> +m_d negative
    Hbar = W + Sigma_x + dw + Jd' diag(1/Ed) Jd
 2. "local blocks", eliminated onto their stage variables p:
      collision pair (i,m,n): z = [mu_mn (e_n), lam_mn (e_m)], rows c2 (2 eq),
                              p = (x_i, y_i, theta_i)
      terminal:               z = slack_e (5), rows terminal (5 eq),
                              p = x_{N-1}
    Kloc = [Hbar_zz, Cz'; Cz, -dc]  (inertia by eigvalsh), B = [Hbar_zp; Cp]
 3. stage block-tridiagonal system, block i = [y_i (init / dyn_{i-1} rows),
    x_i, u_i, tau_i]; block LDL^T (D_{i+1} = K_{i+1,i+1} - L D_i^{-1} L'),
    inertia of each D_i by eigvalsh.
"""
import numpy as np
import scipy.linalg as sla

from .nlp import NS, NC


def _eig_inertia(Ms):
    """Inertia from a Bunch-Kaufman LDL^T (scale-robust, unlike eigvalsh)."""
    _, d, _ = sla.ldl(Ms, lower=True)
    pos = neg = zer = 0
    i, n = 0, d.shape[0]
    while i < n:
        if i + 1 < n and d[i + 1, i] != 0.0:
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


class StructuredKKTLoop:
    """Per-block reference loop (the round-1/2 oracle); kept to cross-check StructuredKKT."""

    def __init__(self, nlp):
        self.nlp = nlp
        N = nlp.N
        gL, gU = nlp.g_L, nlp.g_U
        E = np.where(gL == gU)[0]
        I = np.where(gL != gU)[0]
        posE = -np.ones(nlp.m, dtype=int)
        posE[E] = np.arange(E.size)
        self.posE = posE
        # local blocks: collision pairs (uniform sizes are not required)
        self.loc = []
        for p, (i, m, n, mu0, la0) in enumerate(nlp.pairs):
            en, em = nlp.eb[n], nlp.eo[m]
            z = np.concatenate([mu0 + np.arange(en), la0 + np.arange(em)])
            r = nlp.gCol + 4 * p
            self.loc.append((z, posE[[r + 1, r + 2]], np.array([NS * i, NS * i + 1, NS * i + 3])))
        # terminal block
        self.loc.append((nlp.oS + np.arange(NS), posE[nlp.gTerm + np.arange(NS)], NS * (N - 1) + np.arange(NS)))
        # stage blocks
        self.stage_vars, self.stage_rows = [], []
        for i in range(N):
            v = list(NS * i + np.arange(NS))
            if i < N - 1:
                v += [nlp.oU + NC * i, nlp.oU + NC * i + 1]
                if nlp.topt:
                    v.append(nlp.oTAU + i)
            rows = np.arange(NS) if i == 0 else nlp.gDyn + NS * (i - 1) + np.arange(NS)
            self.stage_vars.append(np.array(v))
            self.stage_rows.append(posE[rows])
        self.n_stage = sum(len(v) for v in self.stage_vars)

    def factor(self, Wm, Sx, Ss, Jc, Jd, dw, dc):
        nlp = self.nlp
        Wm, Jc, Jd = Wm.tocsr(), Jc.tocsr(), Jd.tocsr()
        n, mc, md = Wm.shape[0], Jc.shape[0], Jd.shape[0]
        # dc: scalar, or per row [equality rows (E order), inequality rows] (restoration phase)
        dcv = np.broadcast_to(np.asarray(dc, dtype=float), (mc + md,))
        dcc, dcd = dcv[:mc], dcv[mc:]
        Ds = Ss + dw
        Ed = 1.0 / Ds + dcd
        import scipy.sparse as sp
        Hb = (Wm + sp.diags(Sx + dw) + Jd.T @ sp.diags(1.0 / Ed) @ Jd).tocsr()
        pos, neg, zer = md, md, 0
        Hd = Hb.toarray() if n <= 6000 else None
        self._Hb, self._Jc, self._Jd, self._Ds, self._Ed, self._dc = Hb, Jc, Jd, Ds, Ed, dc
        Jcd = Jc.toarray() if n <= 6000 else None

        def hsub(r, c):
            if Hd is not None:
                return Hd[np.ix_(r, c)]
            return Hb[r][:, c].toarray()

        def jsub(r, c):
            if Jcd is not None:
                return Jcd[np.ix_(r, c)]
            return Jc[r][:, c].toarray()

        self.locfac = []
        schur = {}
        for (z, rows, p) in self.loc:
            nz, nr = z.size, rows.size
            K = np.zeros((nz + nr, nz + nr))
            K[:nz, :nz] = hsub(z, z)
            Cz = jsub(rows, z)
            K[nz:, :nz] = Cz
            K[:nz, nz:] = Cz.T
            K[nz:, nz:] = -np.diag(dcc[rows])
            B = np.vstack([hsub(z, p), jsub(rows, p)])
            a, b_, c_ = _eig_inertia(K)
            pos, neg, zer = pos + a, neg + b_, zer + c_
            if c_:
                return pos, neg, zer
            KiB = np.linalg.solve(K, B)
            self.locfac.append((K, B, KiB))
            key = tuple(p)
            schur[key] = schur.get(key, 0.0) + B.T @ KiB
        # stage blocks
        N = nlp.N
        self.D, self.Lo = [], []
        prev = None
        for i in range(N):
            v, r = self.stage_vars[i], self.stage_rows[i]
            nv, nr = v.size, r.size
            K = np.zeros((nr + nv, nr + nv))
            K[:nr, :nr] = -np.diag(dcc[r])
            Jr = jsub(r, v)
            K[:nr, nr:] = Jr
            K[nr:, :nr] = Jr.T
            K[nr:, nr:] = hsub(v, v)
            # add the Schur complements of local blocks attached to this stage
            for key, S in schur.items():
                kk = np.array(key)
                if np.all(np.isin(kk, v)):
                    idx = nr + np.searchsorted(v, kk) if np.all(np.diff(v) > 0) else nr + np.array([list(v).index(q) for q in kk])
                    K[np.ix_(idx, idx)] -= S
            if prev is not None:
                pv, pr, Dp = prev
                # off-diagonal block: rows [y_i, v_i] x cols [y_{i-1}, v_{i-1}]
                Off = np.zeros((nr + nv, pr.size + pv.size))
                Off[:nr, pr.size:] = jsub(r, pv)
                Off[nr:, pr.size:] = hsub(v, pv)
                try:
                    LD = np.linalg.solve(Dp, Off.T).T
                except np.linalg.LinAlgError:   # exactly singular previous block: reported as singular
                    return pos, neg, zer + 1
                K = K - LD @ Off.T
                self.Lo.append((Off, LD))
            a, b_, c_ = _eig_inertia(K)
            pos, neg, zer = pos + a, neg + b_, zer + c_
            if c_:          # singular stage block: reported as such (IPOPT then perturbs delta_c)
                return pos, neg, zer
            self.D.append(K)
            prev = (v, r, K)
        return pos, neg, zer

    def solve(self, bx, bs, bc, bd):
        nlp = self.nlp
        Jd, Ds, Ed = self._Jd, self._Ds, self._Ed
        bxb = bx + Jd.T @ ((bd + bs / Ds) / Ed)
        bcb = bc.copy()
        # local block rhs
        rloc = []
        stage_rhs = {}
        for (z, rows, p), (K, B, KiB) in zip(self.loc, self.locfac):
            bl = np.concatenate([bxb[z], bcb[rows]])
            Kib = np.linalg.solve(K, bl)
            rloc.append(Kib)
            for j, q in enumerate(p):
                stage_rhs[q] = stage_rhs.get(q, 0.0) + B[:, j] @ Kib
        # stage rhs
        N = nlp.N
        R = []
        for i in range(N):
            v, r = self.stage_vars[i], self.stage_rows[i]
            rv = np.concatenate([bcb[r], np.array([bxb[q] - stage_rhs.get(q, 0.0) for q in v])])
            R.append(rv)
        # forward
        V = [R[0]]
        for i in range(1, N):
            Off, LD = self.Lo[i - 1]
            V.append(R[i] - LD @ V[i - 1])
        X = [None] * N
        X[N - 1] = np.linalg.solve(self.D[N - 1], V[N - 1])
        for i in range(N - 2, -1, -1):
            Off, LD = self.Lo[i]
            X[i] = np.linalg.solve(self.D[i], V[i] - Off.T @ X[i + 1])
        dx = np.zeros(nlp.n)
        dyc = np.zeros(bc.size)
        for i in range(N):
            v, r = self.stage_vars[i], self.stage_rows[i]
            dyc[r] = X[i][:r.size]
            dx[v] = X[i][r.size:]
        # local back-substitution
        for (z, rows, p), (K, B, KiB), Kib in zip(self.loc, self.locfac, rloc):
            w = Kib - KiB @ dx[p]
            dx[z] = w[:z.size]
            dyc[rows] = w[z.size:]
        dyd = (Jd @ dx - bd - bs / Ds) / Ed
        ds = (bs + dyd) / Ds
        return dx, ds, dyc, dyd


def _gather(M, R, C):
    """Dense values M[R, C] of a CSR matrix for broadcast index arrays R, C."""
    R, C = np.broadcast_arrays(np.asarray(R), np.asarray(C))
    if R.size == 0:
        return np.zeros(R.shape)
    return np.asarray(M[R.ravel(), C.ravel()]).reshape(R.shape)


def _ldl_nopiv(K):
    """Batched unpivoted LDL^T pivots of symmetric K (B, n, n) -> d (B, n) (no interchanges)."""
    A = K.copy()
    n = A.shape[1]
    d = np.zeros(A.shape[:2])
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        for k in range(n):
            d[:, k] = A[:, k, k]
            if k + 1 < n:
                l = A[:, k + 1:, k] / d[:, k, None]
                A[:, k + 1:, k + 1:] -= l[:, :, None] * A[:, None, k, k + 1:]
    return d


class StructuredKKT:
    """Same elimination and inertia as StructuredKKTLoop, batched over the collision pairs.

    The pairs of one (obstacle m, body n) share a block shape and are handled as one stack:
    the dense blocks are gathered from the sparse matrices in one indexing call, the inertia of
    a block comes from its unpivoted LDL^T when every multiplier pivot is positive (then the
    block is [H, C'; C, -dc] with H positive definite, a stable factorisation whose pivot signs
    are the exact inertia) and from the Bunch-Kaufman LDL^T otherwise, and the solves run
    through numpy's batched LU.  Schur complements enter the stage blocks in the loop
    version's order (pairs of stage i in (m, n) order, then the terminal block)."""

    def __init__(self, nlp):
        self.nlp = nlp
        N = nlp.N
        gL, gU = nlp.g_L, nlp.g_U
        E = np.where(gL == gU)[0]
        posE = -np.ones(nlp.m, dtype=int)
        posE[E] = np.arange(E.size)
        self.posE = posE
        P = len(nlp.pairs)
        pi = np.array([q[0] for q in nlp.pairs], dtype=int)
        pm = np.array([q[1] for q in nlp.pairs], dtype=int)
        pn = np.array([q[2] for q in nlp.pairs], dtype=int)
        mu0 = np.array([q[3] for q in nlp.pairs], dtype=int)
        la0 = np.array([q[4] for q in nlp.pairs], dtype=int)
        self.groups = []
        for m in range(nlp.M):
            for n in range(nlp.K):
                sel = np.where((pm == m) & (pn == n))[0]
                if sel.size == 0:
                    continue
                en, em = int(nlp.eb[n]), int(nlp.eo[m])
                Z = np.concatenate([mu0[sel, None] + np.arange(en), la0[sel, None] + np.arange(em)], axis=1)
                r = nlp.gCol + 4 * sel
                Rw = posE[np.stack([r + 1, r + 2], axis=1)]
                Pv = np.stack([NS * pi[sel], NS * pi[sel] + 1, NS * pi[sel] + 3], axis=1)
                self.groups.append(dict(sel=sel, stage=pi[sel], Z=Z, R=Rw, P=Pv))
        self.npair = P
        self.term = (nlp.oS + np.arange(NS), posE[nlp.gTerm + np.arange(NS)], NS * (N - 1) + np.arange(NS))
        self.stage_vars, self.stage_rows = [], []
        for i in range(N):
            v = list(NS * i + np.arange(NS))
            if i < N - 1:
                v += [nlp.oU + NC * i, nlp.oU + NC * i + 1]
                if nlp.topt:
                    v.append(nlp.oTAU + i)
            rows = np.arange(NS) if i == 0 else nlp.gDyn + NS * (i - 1) + np.arange(NS)
            self.stage_vars.append(np.array(v))
            self.stage_rows.append(posE[rows])
        self.n_stage = sum(len(v) for v in self.stage_vars)

    def factor(self, Wm, Sx, Ss, Jc, Jd, dw, dc):
        import scipy.sparse as sp
        nlp = self.nlp
        Wm, Jc, Jd = Wm.tocsr(), Jc.tocsr(), Jd.tocsr()
        n, mc, md = Wm.shape[0], Jc.shape[0], Jd.shape[0]
        dcv = np.broadcast_to(np.asarray(dc, dtype=float), (mc + md,))
        dcc, dcd = dcv[:mc], dcv[mc:]
        Ds = Ss + dw
        Ed = 1.0 / Ds + dcd
        Hb = (Wm + sp.diags(Sx + dw) + Jd.T @ sp.diags(1.0 / Ed) @ Jd).tocsr()
        self._Hb, self._Jc, self._Jd, self._Ds, self._Ed, self._dc = Hb, Jc, Jd, Ds, Ed, dc
        pos, neg, zer = md, md, 0
        N = nlp.N
        schur = np.zeros((N, 3, 3))
        self.gfac = []
        for g in self.groups:
            Z, Rw, Pv = g["Z"], g["R"], g["P"]
            nz, nr = Z.shape[1], Rw.shape[1]
            B_ = Z.shape[0]
            K = np.zeros((B_, nz + nr, nz + nr))
            K[:, :nz, :nz] = _gather(Hb, Z[:, :, None], Z[:, None, :])
            Cz = _gather(Jc, Rw[:, :, None], Z[:, None, :])
            K[:, nz:, :nz] = Cz
            K[:, :nz, nz:] = np.transpose(Cz, (0, 2, 1))
            K[:, nz:, nz:] = -dcc[Rw][:, :, None] * np.eye(nr)
            Bm = np.concatenate([_gather(Hb, Z[:, :, None], Pv[:, None, :]),
                                 _gather(Jc, Rw[:, :, None], Pv[:, None, :])], axis=1)
            d = _ldl_nopiv(K)
            ok = np.all(d[:, :nz] > 0, axis=1) & np.all(np.isfinite(d), axis=1) & np.all(d != 0, axis=1)
            pos += int(np.sum(d[ok] > 0))
            neg += int(np.sum(d[ok] < 0))
            for b in np.where(~ok)[0]:
                a, b_, c_ = _eig_inertia(K[b])
                pos, neg, zer = pos + a, neg + b_, zer + c_
            if zer:
                return pos, neg, zer
            KiB = np.linalg.solve(K, Bm)
            S = np.einsum("bki,bkj->bij", Bm, KiB)
            np.add.at(schur, g["stage"], S)
            self.gfac.append((K, Bm, KiB))
        # terminal block
        z, rows, p = self.term
        nz, nr = z.size, rows.size
        K = np.zeros((nz + nr, nz + nr))
        K[:nz, :nz] = _gather(Hb, z[:, None], z[None, :])
        Cz = _gather(Jc, rows[:, None], z[None, :])
        K[nz:, :nz] = Cz
        K[:nz, nz:] = Cz.T
        K[nz:, nz:] = -np.diag(dcc[rows])
        Bt = np.vstack([_gather(Hb, z[:, None], p[None, :]), _gather(Jc, rows[:, None], p[None, :])])
        a, b_, c_ = _eig_inertia(K)
        pos, neg, zer = pos + a, neg + b_, zer + c_
        if c_:
            return pos, neg, zer
        KiBt = np.linalg.solve(K, Bt)
        self.tfac = (K, Bt, KiBt)
        St = Bt.T @ KiBt
        # stage blocks
        self.D, self.Lo = [], []
        prev = None
        sidx = np.array([0, 1, 3])
        for i in range(N):
            v, r = self.stage_vars[i], self.stage_rows[i]
            nv, nr = v.size, r.size
            K = np.zeros((nr + nv, nr + nv))
            K[:nr, :nr] = -np.diag(dcc[r])
            Jr = _gather(Jc, r[:, None], v[None, :])
            K[:nr, nr:] = Jr
            K[nr:, :nr] = Jr.T
            K[nr:, nr:] = _gather(Hb, v[:, None], v[None, :])
            if self.npair:
                K[np.ix_(nr + sidx, nr + sidx)] -= schur[i]
            if i == N - 1:
                K[nr:nr + NS, nr:nr + NS] -= St
            if prev is not None:
                pv, pr, Dp = prev
                Off = np.zeros((nr + nv, pr.size + pv.size))
                Off[:nr, pr.size:] = _gather(Jc, r[:, None], pv[None, :])
                Off[nr:, pr.size:] = _gather(Hb, v[:, None], pv[None, :])
                try:
                    LD = np.linalg.solve(Dp, Off.T).T
                except np.linalg.LinAlgError:   # exactly singular previous block: reported as singular
                    return pos, neg, zer + 1
                K = K - LD @ Off.T
                self.Lo.append((Off, LD))
            a, b_, c_ = _eig_inertia(K)
            pos, neg, zer = pos + a, neg + b_, zer + c_
            if c_:          # singular stage block: reported as such (IPOPT then perturbs delta_c)
                return pos, neg, zer
            self.D.append(K)
            prev = (v, r, K)
        return pos, neg, zer

    def solve(self, bx, bs, bc, bd):
        nlp = self.nlp
        Jd, Ds, Ed = self._Jd, self._Ds, self._Ed
        bxb = bx + Jd.T @ ((bd + bs / Ds) / Ed)
        bcb = bc.copy()
        srhs = np.zeros(nlp.n)
        kibs = []
        for g, (K, Bm, KiB) in zip(self.groups, self.gfac):
            bl = np.concatenate([bxb[g["Z"]], bcb[g["R"]]], axis=1)
            Kib = np.linalg.solve(K, bl[:, :, None])[:, :, 0]
            kibs.append(Kib)
            np.add.at(srhs, g["P"], np.einsum("bkj,bk->bj", Bm, Kib))
        z, rows, p = self.term
        Kt, Bt, KiBt = self.tfac
        Kibt = np.linalg.solve(Kt, np.concatenate([bxb[z], bcb[rows]]))
        srhs[p] += Bt.T @ Kibt
        N = nlp.N
        V = []
        for i in range(N):
            v, r = self.stage_vars[i], self.stage_rows[i]
            rv = np.concatenate([bcb[r], bxb[v] - srhs[v]])
            V.append(rv if i == 0 else rv - self.Lo[i - 1][1] @ V[i - 1])
        X = [None] * N
        X[N - 1] = np.linalg.solve(self.D[N - 1], V[N - 1])
        for i in range(N - 2, -1, -1):
            Off, LD = self.Lo[i]
            X[i] = np.linalg.solve(self.D[i], V[i] - Off.T @ X[i + 1])
        dx = np.zeros(nlp.n)
        dyc = np.zeros(bc.size)
        for i in range(N):
            v, r = self.stage_vars[i], self.stage_rows[i]
            dyc[r] = X[i][:r.size]
            dx[v] = X[i][r.size:]
        for g, (K, Bm, KiB), Kib in zip(self.groups, self.gfac, kibs):
            w = Kib - np.einsum("bij,bj->bi", KiB, dx[g["P"]])
            nz = g["Z"].shape[1]
            dx[g["Z"]] = w[:, :nz]
            dyc[g["R"]] = w[:, nz:]
        w = Kibt - KiBt @ dx[p]
        dx[z] = w[:z.size]
        dyc[rows] = w[z.size:]
        dyd = (Jd @ dx - bd - bs / Ds) / Ed
        ds = (bs + dyd) / Ds
        return dx, ds, dyc, dyd


class StructuredPointKKT:
    """The augmented system of the point formulation (oracle/nlp_points.py, optimizer_points.py) by the
    same eliminations: inequality slacks / multipliers, then the lambda-only local blocks of every
    (obstacle j, step i) onto (x_i, y_i, theta_i) -- no equality rows, so each block is the positive
    definite Hbar_zz -- then a block LDL^T over the N stage blocks plus one block for the hard
    terminal rows X_{N-1} = end (coupled to x_{N-1}).  Inertia: unpivoted LDL^T pivots of the local
    blocks when all are positive, Bunch-Kaufman otherwise; Bunch-Kaufman on every stage block."""

    def __init__(self, nlp):
        self.nlp = nlp
        N = nlp.N
        E = np.where(nlp.g_L == nlp.g_U)[0]
        posE = -np.ones(nlp.m, dtype=int)
        posE[E] = np.arange(E.size)
        self.groups = []
        for j in range(nlp.M):
            sel = np.array([p for p, (jj, i, la0) in enumerate(nlp.blocks) if jj == j], dtype=int)
            i = np.array([nlp.blocks[p][1] for p in sel], dtype=int)
            la0 = np.array([nlp.blocks[p][2] for p in sel], dtype=int)
            Z = la0[:, None] + np.arange(int(nlp.eo[j]))
            Pv = np.stack([NS * i, NS * i + 1, NS * i + 3], axis=1)
            self.groups.append(dict(stage=i, Z=Z, P=Pv))
        self.stage_vars, self.stage_rows = [], []
        for i in range(N):
            v = list(NS * i + np.arange(NS))
            if i < N - 1:
                v += [nlp.oU + NC * i, nlp.oU + NC * i + 1]
            rows = np.arange(NS) if i == 0 else nlp.gDyn + NS * (i - 1) + np.arange(NS)
            self.stage_vars.append(np.array(v))
            self.stage_rows.append(posE[rows])
        self.stage_vars.append(np.zeros(0, dtype=int))                    # terminal block: rows only
        self.stage_rows.append(posE[nlp.gTerm + np.arange(NS)])

    def factor(self, Wm, Sx, Ss, Jc, Jd, dw, dc):
        import scipy.sparse as sp
        nlp = self.nlp
        Wm, Jc, Jd = Wm.tocsr(), Jc.tocsr(), Jd.tocsr()
        mc, md = Jc.shape[0], Jd.shape[0]
        dcv = np.broadcast_to(np.asarray(dc, dtype=float), (mc + md,))
        dcc, dcd = dcv[:mc], dcv[mc:]
        Ds = Ss + dw
        Ed = 1.0 / Ds + dcd
        Hb = (Wm + sp.diags(Sx + dw) + Jd.T @ sp.diags(1.0 / Ed) @ Jd).tocsr()
        self._Jd, self._Ds, self._Ed = Jd, Ds, Ed
        pos, neg, zer = md, md, 0
        N = nlp.N
        schur = np.zeros((N, 3, 3))
        self.gfac = []
        for g in self.groups:
            Z, Pv = g["Z"], g["P"]
            K = _gather(Hb, Z[:, :, None], Z[:, None, :])
            Bm = _gather(Hb, Z[:, :, None], Pv[:, None, :])
            d = _ldl_nopiv(K)
            ok = np.all(d > 0, axis=1) & np.all(np.isfinite(d), axis=1)
            pos += int(np.sum(d[ok] > 0))
            for b in np.where(~ok)[0]:
                a, b_, c_ = _eig_inertia(K[b])
                pos, neg, zer = pos + a, neg + b_, zer + c_
            if zer:
                return pos, neg, zer
            KiB = np.linalg.solve(K, Bm)
            np.add.at(schur, g["stage"], np.einsum("bki,bkj->bij", Bm, KiB))
            self.gfac.append((K, Bm, KiB))
        self.D, self.Lo = [], []
        prev = None
        sidx = np.array([0, 1, 3])
        for i in range(N + 1):
            v, r = self.stage_vars[i], self.stage_rows[i]
            nv, nr = v.size, r.size
            K = np.zeros((nr + nv, nr + nv))
            K[:nr, :nr] = -np.diag(dcc[r])
            Jr = _gather(Jc, r[:, None], v[None, :])
            K[:nr, nr:] = Jr
            K[nr:, :nr] = Jr.T
            K[nr:, nr:] = _gather(Hb, v[:, None], v[None, :])
            if i < N:
                K[np.ix_(nr + sidx, nr + sidx)] -= schur[i]
            if prev is not None:
                pv, pr, Dp = prev
                Off = np.zeros((nr + nv, pr.size + pv.size))
                Off[:nr, pr.size:] = _gather(Jc, r[:, None], pv[None, :])
                Off[nr:, pr.size:] = _gather(Hb, v[:, None], pv[None, :])
                try:
                    LD = np.linalg.solve(Dp, Off.T).T
                except np.linalg.LinAlgError:   # exactly singular previous block: reported as singular
                    return pos, neg, zer + 1
                K = K - LD @ Off.T
                self.Lo.append((Off, LD))
            a, b_, c_ = _eig_inertia(K)
            pos, neg, zer = pos + a, neg + b_, zer + c_
            if c_:          # singular stage block: reported as such (IPOPT then perturbs delta_c)
                return pos, neg, zer
            self.D.append(K)
            prev = (v, r, K)
        return pos, neg, zer

    def solve(self, bx, bs, bc, bd):
        nlp = self.nlp
        Jd, Ds, Ed = self._Jd, self._Ds, self._Ed
        bxb = bx + Jd.T @ ((bd + bs / Ds) / Ed)
        srhs = np.zeros(nlp.n)
        kibs = []
        for g, (K, Bm, KiB) in zip(self.groups, self.gfac):
            Kib = np.linalg.solve(K, bxb[g["Z"]][:, :, None])[:, :, 0]
            kibs.append(Kib)
            np.add.at(srhs, g["P"], np.einsum("bkj,bk->bj", Bm, Kib))
        nb = len(self.D)
        V = []
        for i in range(nb):
            v, r = self.stage_vars[i], self.stage_rows[i]
            rv = np.concatenate([bc[r], bxb[v] - srhs[v]])
            V.append(rv if i == 0 else rv - self.Lo[i - 1][1] @ V[i - 1])
        X = [None] * nb
        X[nb - 1] = np.linalg.solve(self.D[nb - 1], V[nb - 1])
        for i in range(nb - 2, -1, -1):
            Off, LD = self.Lo[i]
            X[i] = np.linalg.solve(self.D[i], V[i] - Off.T @ X[i + 1])
        dx = np.zeros(nlp.n)
        dyc = np.zeros(bc.size)
        for i in range(nb):
            v, r = self.stage_vars[i], self.stage_rows[i]
            dyc[r] = X[i][:r.size]
            dx[v] = X[i][r.size:]
        for g, (K, Bm, KiB), Kib in zip(self.groups, self.gfac, kibs):
            dx[g["Z"]] = Kib - np.einsum("bij,bj->bi", KiB, dx[g["P"]])
        dyd = (Jd @ dx - bd - bs / Ds) / Ed
        ds = (bs + dyd) / Ds
        return dx, ds, dyc, dyd
