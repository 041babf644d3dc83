"""TEST-ONLY helpers for the Reeds-Shepp parity tests: golden fixtures and the
oracle in the CSR layout of htp_rs_all_paths_batch, comparison, seeded query
generators and the reference's own check_path properties
(R/path_planner/utils/reeds_shepp.py:668-690)."""
import math
import os

import numpy as np

from oracle import reeds_shepp as ors

HERE = os.path.dirname(os.path.abspath(__file__))
SEG = {"L": 0, "S": 1, "R": 2, "_": 3}
FIELDS_EXACT = ("path_offsets", "status", "ctypes", "point_offsets", "directions")
FIELDS_FLOAT = ("lengths", "L", "x", "y", "yaw", "cs")


def golden():
    g = np.load(os.path.join(HERE, "golden", "rs_calc_all_paths.npz"))
    pts = g["points"]
    out = {"queries": g["cases"], "path_offsets": g["path_offsets"].astype(np.int64),
           "status": np.zeros(len(g["cases"]), np.int32), "lengths": g["lengths"], "L": g["L"],
           "ctypes": np.array([[SEG[c] for c in s] for s in g["ctypes"]], np.int8).reshape(-1, 5),
           "point_offsets": g["point_offsets"].astype(np.int64), "x": pts[:, 0], "y": pts[:, 1],
           "yaw": pts[:, 2], "directions": pts[:, 3].astype(np.int8), "cs": pts[:, 4]}
    return out


def oracle_csr(queries):
    po, pt, st = [0], [0], []
    cols = {k: [] for k in ("lengths", "ctypes", "L", "x", "y", "yaw", "cs", "directions")}
    for q in np.asarray(queries, dtype=np.float64):
        try:
            paths = calc_all_paths_all_samples(*[float(v) for v in q])
            st.append(2 if any(p.x is None for p in paths) else 0)
        except AssertionError:
            paths = []
            st.append(1)
        for p in paths:
            if p.x is None:  # the reference raises IndexError here; the ABI keeps the path with no samples
                p.x = p.y = p.yaw = p.cs = p.directions = []
            n = len(p.lengths)
            cols["lengths"].append(list(p.lengths) + [0.0] * (5 - n))
            cols["ctypes"].append([SEG[c] for c in p.ctypes] + [3] * (5 - n))
            cols["L"].append(p.L)
            for k in ("x", "y", "yaw", "cs", "directions"):
                cols[k].extend(getattr(p, k))
            pt.append(pt[-1] + len(p.x))
        po.append(po[-1] + len(paths))
    out = {"path_offsets": np.array(po, np.int64), "point_offsets": np.array(pt, np.int64),
           "status": np.array(st, np.int32),
           "lengths": np.array(cols["lengths"], np.float64).reshape(-1, 5),
           "ctypes": np.array(cols["ctypes"], np.int8).reshape(-1, 5), "L": np.array(cols["L"], np.float64),
           "directions": np.array(cols["directions"], np.int8)}
    for k in ("x", "y", "yaw", "cs"):
        out[k] = np.array(cols[k], np.float64)
    return out


def calc_all_paths_all_samples(sx, sy, syaw, gx, gy, gyaw, maxc, step_size):
    """ors.calc_all_paths, but a path whose sampler would raise IndexError
    (every sample at local x == 0.0) gets x = None instead of aborting the
    query -- the CSR convention of htp_rs_all_paths_batch (status 2)."""
    import math
    dx, dy, dth = gx - sx, gy - sy, gyaw - syaw
    c, s = math.cos(syaw), math.sin(syaw)
    paths = ors.admissible_words((c * dx + s * dy) * maxc, (-s * dx + c * dy) * maxc, dth)
    cq, sq = math.cos(-syaw), math.sin(-syaw)
    for p in paths:
        try:
            lx, ly, lyaw, cs, dirs = ors.local_course(p.L, p.lengths, p.ctypes, maxc, step_size * maxc)
            p.x = [cq * a + sq * b + sx for a, b in zip(lx, ly)]
            p.y = [-sq * a + cq * b + sy for a, b in zip(lx, ly)]
            p.yaw = [ors.pi_2_pi(a + syaw) for a in lyaw]
            p.cs, p.directions = cs, dirs
        except IndexError:
            p.x = None
        p.lengths = [a / maxc for a in p.lengths]
        p.L = p.L / maxc
    return paths


def compare(a, b, atol=0.0):
    """List of mismatch descriptions (empty = parity).  Structure (offsets,
    status, ctypes, directions) must be identical; values equal (atol=0) or
    within atol."""
    errs = []
    for k in FIELDS_EXACT:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        if x.shape != y.shape or not np.array_equal(x, y):
            if k in ("path_offsets", "point_offsets", "status") and x.shape == y.shape:
                bad = np.nonzero(x != y)[0]
                errs.append(f"{k}: {len(bad)} differ, first at {bad[:5].tolist()}")
            else:
                errs.append(f"{k}: shape {x.shape} vs {y.shape}")
            return errs  # later fields are misaligned
    for k in FIELDS_FLOAT:
        x, y = np.asarray(a[k], np.float64), np.asarray(b[k], np.float64)
        if k == "yaw":  # pi_2_pi output: +-pi are the same angle
            d = np.abs(np.angle(np.exp(1j * (x - y)))) if x.size else np.zeros(0)
        else:
            d = np.abs(x - y)
        m = float(d.max()) if d.size else 0.0
        if (atol == 0.0 and not np.array_equal(x, y)) or m > atol:
            errs.append(f"{k}: max |diff| {m:.3e} > {atol}")
    return errs


def random_queries(n, seed, box=8.0, degenerate=True):
    """Seeded pose pairs: general poses, near-coincident, pure rotations,
    pure translations along the heading, far goals, varied curvature/step.

    degenerate=False drops the pure rotations and straight-ahead goals: those
    sit exactly on the words' tie-breaks (t == 0, symmetric t == v, sample
    position == segment end), where a last-ulp difference between the device's
    and glibc's trig functions legitimately flips a comparison."""
    rng = np.random.default_rng(seed)
    q = np.zeros((n, 8))
    q[:, 0:2] = rng.uniform(-box, box, (n, 2))
    q[:, 2] = rng.uniform(-math.pi, math.pi, n)
    q[:, 3:5] = rng.uniform(-box, box, (n, 2))
    q[:, 5] = rng.uniform(-math.pi, math.pi, n)
    q[:, 6] = rng.choice([math.tan(0.55) / 1.9, math.tan(0.5) / 1.9, 0.5, 1.0 / 3.2, 0.2], n)
    q[:, 7] = rng.choice([0.2, 0.1, 0.05, 0.3], n)
    kind = rng.integers(0, 8, n)
    if not degenerate:
        kind[(kind == 2) | (kind == 3)] = 0
    near = kind == 1
    q[near, 3:5] = q[near, 0:2] + rng.normal(0, 0.05, (near.sum(), 2))
    rot = kind == 2
    q[rot, 3:5] = q[rot, 0:2]
    q[rot, 5] = q[rot, 2] + rng.uniform(0.1, 3.0, rot.sum())
    fwd = kind == 3
    dist = rng.uniform(0.5, 10.0, fwd.sum())
    q[fwd, 3] = q[fwd, 0] + dist * np.cos(q[fwd, 2])
    q[fwd, 4] = q[fwd, 1] + dist * np.sin(q[fwd, 2])
    q[fwd, 5] = q[fwd, 2]
    far = kind == 4
    q[far, 3:5] = q[far, 0:2] + rng.uniform(-300, 300, (far.sum(), 2))
    return q


def check_path_properties(csr, queries, tol=0.01, report=None, goal=True):
    """reeds_shepp.check_path (:668-690) as far as the reference satisfies it:
    every path starts at the start pose; on general-position queries, words
    with a straight segment end at the goal pose.  (The reference's CCC/CCCC
    words can miss the goal, its samples can be further apart than step_size,
    and on degenerate queries S-words can miss too -- parity keeps all of that,
    so those parts of check_path are not asserted.)  Returns the number of
    violating paths."""
    bad = 0
    po, pt = csr["path_offsets"], csr["point_offsets"]
    for i, q in enumerate(np.asarray(queries)):
        for p in range(int(po[i]), int(po[i + 1])):
            a, b = int(pt[p]), int(pt[p + 1]) - 1
            if b < a:
                bad += 1
                continue
            ok = (abs(csr["x"][a] - q[0]) <= 1e-9 and abs(csr["y"][a] - q[1]) <= 1e-9)
            if goal and 1 in csr["ctypes"][p]:
                ok = ok and (abs(csr["x"][b] - q[3]) <= tol and abs(csr["y"][b] - q[4]) <= tol
                             and abs(math.remainder(csr["yaw"][b] - q[5], 2 * math.pi)) <= tol)
            if not ok:
                bad += 1
                if report is not None and len(report) < 5:
                    report.append((i, q.tolist(), "".join("LSR_"[c] for c in csr["ctypes"][p]),
                                   csr["lengths"][p].tolist(), b - a + 1,
                                   [csr["x"][a], csr["y"][a], csr["x"][b], csr["y"][b], csr["yaw"][b]]))
    return bad
