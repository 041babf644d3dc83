"""Deterministic synthetic headland-turn workload.

Problem `pid` is drawn from Philox(key=[20251015, pid]) so a problem is
identical for any batch composition and any GPU count.

Two scene builders:

* `config_instance` / `make_orchard_instance` -- the BASELINE configs A-E.  The
  scene and the warm start come from the reference's own producers, restated in
  path_planner/ (see the block comment above make_orchard_instance): tree rows
  (map_utils.create_tree_rows), row poses (get_base_pose), the Dubins /
  circle-back / fish-tail planners of safety_forward_path_plan.py and
  OBCA_warm_start.py, get_init_ref_path, and OGE_OBCA's obstacle producer
  (create_boundary_polygons, get_obstacle_tree_rows, get_obstacles_for_OBCA).
* `make_instance` -- hand-placed rectangle scenes (headland boundary quad, the
  up bound quad, tree-row rectangles, far dummy quads) with closed-form
  warm starts; small-shape parity tests and the smoke test use it:
  - "dubins": the shortest Dubins word (pydubins);
  - "circleback": forward arc R_f by theta, reverse arc R_b by pi - theta,
    Dubins lead-in (safety_forward_path_plan.py:395-454);
  - "fishtail": a three-arc C|C|C K-turn at the minimum radius joined to the
    row poses by straights;
  - "mixed": one of the three per problem (its own Philox stream, key + 1).
  The path is sampled to exactly N poses and turned into [x, y, v, theta, steer]
  as R/obca_py/util.py:62-113 does; the boundary sits behind the warm start's
  swept footprint with a random margin.
"""
import math

import numpy as np

from . import geometry

TWO_PI = 2.0 * math.pi

MOWER = [[-1.84, 0.5], 1.0, 1.1]           # R/test/obca.ipynb (mowing preset)
PRUNER = [[3.259, -0.175], 1.325, 0.3]     # R/test/obca.ipynb:133 (summer pruning)
IMPLEMENTS = {"none": None, "mower": MOWER, "pruner": PRUNER}

# Vehicle of SURVEY 8(d) / R/test/obca.ipynb:142
VEHICLE = dict(max_steer=0.55, wheelbase=1.9, axle_to_front=2.85, axle_to_back=0.55, width=1.48)

# OBCA weights of R/test/obca.ipynb:370-371,413-415
DEFAULT_WEIGHTS = dict(dT=0.4, Q=np.diag([1.0, 1.0]), R=np.diag([0.1, 0.1]), W=np.diag([10.0, 0.1]))


# ----------------------------------------------------------------- Dubins
def _mod2pi(x):
    return x - TWO_PI * math.floor(x / TWO_PI)


def dubins_words(q0, q1, r):
    """All admissible Dubins words (pydubins / Shkel-Lumelsky formulation).
    Returns list of (name, (t, p, q)) in normalised (r=1) lengths."""
    dx, dy = q1[0] - q0[0], q1[1] - q0[1]
    D = math.hypot(dx, dy)
    d = D / r
    th = _mod2pi(math.atan2(dy, dx)) if D > 0 else 0.0
    a = _mod2pi(q0[2] - th)
    b = _mod2pi(q1[2] - th)
    sa, sb, ca, cb = math.sin(a), math.sin(b), math.cos(a), math.cos(b)
    cab = math.cos(a - b)
    out = []
    p2 = 2 + d * d - 2 * cab + 2 * d * (sa - sb)
    if p2 >= 0:
        t1 = math.atan2(cb - ca, d + sa - sb)
        out.append(("LSL", (_mod2pi(-a + t1), math.sqrt(p2), _mod2pi(b - t1))))
    p2 = 2 + d * d - 2 * cab + 2 * d * (sb - sa)
    if p2 >= 0:
        t1 = math.atan2(ca - cb, d - sa + sb)
        out.append(("RSR", (_mod2pi(a - t1), math.sqrt(p2), _mod2pi(-b + t1))))
    p2 = -2 + d * d + 2 * cab + 2 * d * (sa + sb)
    if p2 >= 0:
        p = math.sqrt(p2)
        t2 = math.atan2(-ca - cb, d + sa + sb) - math.atan2(-2.0, p)
        out.append(("LSR", (_mod2pi(-a + t2), p, _mod2pi(-_mod2pi(b) + t2))))
    p2 = d * d - 2 + 2 * cab - 2 * d * (sa + sb)
    if p2 >= 0:
        p = math.sqrt(p2)
        t2 = math.atan2(ca + cb, d - sa - sb) - math.atan2(2.0, p)
        out.append(("RSL", (_mod2pi(a - t2), p, _mod2pi(b - t2))))
    t0 = (6.0 - d * d + 2 * cab + 2 * d * (sa - sb)) / 8.0
    if abs(t0) <= 1:
        p = _mod2pi(TWO_PI - math.acos(t0))
        t = _mod2pi(a - math.atan2(ca - cb, d - sa + sb) + p / 2.0)
        out.append(("RLR", (t, p, _mod2pi(a - b - t + p))))
    t0 = (6.0 - d * d + 2 * cab + 2 * d * (sb - sa)) / 8.0
    if abs(t0) <= 1:
        p = _mod2pi(TWO_PI - math.acos(t0))
        t = _mod2pi(-a - math.atan2(ca - cb, d + sa - sb) + p / 2.0)
        out.append(("LRL", (t, p, _mod2pi(_mod2pi(b) - a - t + p))))
    return out


def dubins_shortest(q0, q1, r):
    words = dubins_words(q0, q1, r)
    name, seg = min(words, key=lambda w: sum(w[1]))
    return name, seg


def dubins_sample(q0, r, name, seg, s):
    """Pose + curvature at arc lengths s (metres) along a Dubins word (vectorised)."""
    t = np.asarray(s, dtype=np.float64) / r
    x = np.zeros_like(t)
    y = np.zeros_like(t)
    th = np.full_like(t, q0[2])
    kap = np.zeros_like(t)
    rem = t.copy()
    for typ, ln in zip(name, seg):
        st = np.minimum(rem, ln)
        act = rem > 0
        if typ == "L":
            nx, ny, nth, k = x + np.sin(th + st) - np.sin(th), y - np.cos(th + st) + np.cos(th), th + st, 1.0 / r
        elif typ == "R":
            nx, ny, nth, k = x - np.sin(th - st) + np.sin(th), y + np.cos(th - st) - np.cos(th), th - st, -1.0 / r
        else:
            nx, ny, nth, k = x + np.cos(th) * st, y + np.sin(th) * st, th, 0.0
        x, y, th = np.where(act, nx, x), np.where(act, ny, y), np.where(act, nth, th)
        kap = np.where(act, k, kap)
        rem = rem - st
    return np.stack([q0[0] + x * r, q0[1] + y * r, th, kap], axis=1)


# ------------------------------------------------- arc/straight segment paths
def segments_sample(q0, segs, s):
    """Pose, steering curvature and gear at arc lengths s (metres, along |path|) of a
    path of segments (kappa, u): kappa = steering curvature (dtheta per signed metre),
    u = signed length (u < 0 drives in reverse).  Returns (P, 5) [x, y, theta, kappa, dir]."""
    s = np.asarray(s, dtype=np.float64)
    out = np.zeros((s.size, 5))
    x, y, th = float(q0[0]), float(q0[1]), float(q0[2])
    start = 0.0
    for j, (kap, u) in enumerate(segs):
        ln = abs(u)
        sgn = 1.0 if u >= 0 else -1.0
        last = j == len(segs) - 1
        sel = (s >= start) & ((s < start + ln) | last)
        t = np.clip(s[sel] - start, 0.0, ln) * sgn
        if kap != 0.0:
            th1 = th + kap * t
            out[sel, 0] = x + (np.sin(th1) - math.sin(th)) / kap
            out[sel, 1] = y - (np.cos(th1) - math.cos(th)) / kap
            out[sel, 2] = th1
        else:
            out[sel, 0] = x + t * math.cos(th)
            out[sel, 1] = y + t * math.sin(th)
            out[sel, 2] = th
        out[sel, 3] = kap
        out[sel, 4] = sgn
        if kap != 0.0:
            th1 = th + kap * u
            x, y = x + (math.sin(th1) - math.sin(th)) / kap, y - (math.cos(th1) - math.cos(th)) / kap
            th = th1
        else:
            x, y = x + u * math.cos(th), y + u * math.sin(th)
        start += ln
    return out


def _seg_end(q0, segs):
    return segments_sample(q0, segs, [sum(abs(u) for _, u in segs)])[0]


def dubins_segments(q0, q1, r):
    """Shortest Dubins word as segments (steering curvature +1/r = L)."""
    name, seg = dubins_shortest(q0, q1, r)
    return [({"L": 1.0 / r, "R": -1.0 / r, "S": 0.0}[ch], ln * r) for ch, ln in zip(name, seg)]


def circle_back_segments(ps, pe, r, step=0.1):
    """safety_forward_path_plan.py:395-454 (get_circle_back_path_full, NEAR side, exit heading pi,
    enter heading 0): forward arc (Rf, theta) toward the next rows, reverse arc (Rb, pi - theta),
    Dubins lead-in to the row pose; None when the rows are 2R or more apart (the reference's Dubins
    fallback)."""
    w = abs(pe[1] - ps[1])
    if w >= 2.0 * r:
        return None
    Rf = Rb = r
    while True:
        theta = math.pi / 2 + math.asin((Rb + w - Rf) / (Rf + Rb))
        if ps[0] - (Rf + Rb) * math.cos(theta - math.pi / 2) < pe[0] - step:
            break
        Rf *= 1.05
        Rb *= 1.05
    turn = 1.0 if pe[1] - ps[1] > 0 else -1.0   # steer sign of get_steer_dir_for_enter_calculation (heading pi)
    segs = [(-turn / Rf, Rf * theta), (turn / Rb, -Rb * (math.pi - theta))]
    q = _seg_end(ps, segs)
    return segs + [sg for sg in dubins_segments((q[0], q[1], q[2]), pe, r) if sg[1] > 1e-12]


def fishtail_segments(ps, pe, r):
    """Three-arc C|C|C K-turn at the minimum radius: forward arc a, reverse arc pi - 2a, forward
    arc a (heading pi -> 0), a chosen by bisection so the lateral shift equals the row offset, then
    straights along the row axis so it starts at the exit pose and ends at the enter pose.  None
    when the rows are 2R or more apart."""
    w = pe[1] - ps[1]
    turn = 1.0 if w > 0 else -1.0
    if abs(w) >= 2.0 * r:
        return None

    def arcs(a):
        return [(-turn / r, r * a), (turn / r, -r * (math.pi - 2 * a)), (-turn / r, r * a)]

    lo, hi = 0.0, math.pi / 2   # signed lateral shift grows from -2r (a = 0) to 2r (a = pi/2)
    for _ in range(80):
        mid = 0.5 * (lo + hi)
        dy = _seg_end((0.0, 0.0, ps[2]), arcs(mid))[1]
        if turn * dy < abs(w):
            lo = mid
        else:
            hi = mid
    segs = arcs(0.5 * (lo + hi))
    dx = _seg_end((0.0, 0.0, ps[2]), segs)[0]
    lead = ps[0] + dx - pe[0]            # forward along heading pi before the arcs (moves -x)
    out = []
    if lead > 0:
        out.append((0.0, lead))
    out += segs
    if lead < 0:
        out.append((0.0, -lead))          # forward along heading 0 after the arcs
    return out


TURN_TYPES = ("dubins", "circleback", "fishtail")


# ------------------------------------------------------------ angle helpers
def wrap_angle(a):
    """R/obca_py/util.py:7-13 (Python floored modulo)."""
    return (np.asarray(a) + math.pi) % TWO_PI - math.pi


def process_angle(raw):
    """R/obca_py/util.py:16-43: wrap each angle, then unwrap the sequence."""
    w = wrap_angle(np.asarray(raw, dtype=np.float64))
    out = np.zeros_like(w)
    if w.size:
        out[0] = w[0]
        for i in range(1, w.size):
            out[i] = out[i - 1] + wrap_angle(w[i] - w[i - 1])
    return out


# ------------------------------------------------------------- polygon ops
def _polys_at(poly, poses):
    """poly (k,2) placed at every pose (P,3) -> (P,k,2)."""
    c, s = np.cos(poses[:, 2]), np.sin(poses[:, 2])
    px = poly[None, :, 0] * c[:, None] - poly[None, :, 1] * s[:, None] + poses[:, 0:1]
    py = poly[None, :, 0] * s[:, None] + poly[None, :, 1] * c[:, None] + poses[:, 1:2]
    return np.stack([px, py], axis=2)


def _min_sat_gap(F, Q):
    """Smallest separating-axis gap between each convex polygon F[p] (P,k,2)
    and the convex polygon Q (m,2); >0 means every pair is disjoint."""
    def axes(poly):  # (..., e, 2) unit outward-ish normals
        E = np.roll(poly, -1, axis=-2) - poly
        nrm = np.stack([E[..., 1], -E[..., 0]], axis=-1)
        return nrm / np.linalg.norm(nrm, axis=-1, keepdims=True)
    best = np.full(F.shape[0], -np.inf)
    for ax in (axes(F), np.broadcast_to(axes(Q), (F.shape[0],) + Q.shape)):
        pa = np.einsum("pkd,ped->pke", F, ax)            # (P,k,e)
        pb = np.einsum("md,ped->pme", Q, ax)             # (P,m,e)
        gap = np.maximum(pb.min(1) - pa.max(1), pa.min(1) - pb.max(1))  # (P,e)
        best = np.maximum(best, gap.max(1))
    return best.min()


def _rect(x0, x1, y0, y1):
    return np.array([[x0, y0], [x0, y1], [x1, y1], [x1, y0]], dtype=np.float64)


# ---------------------------------------------------------------- instance
def make_instance(pid, N=80, M=6, implement="none", key=20251015, turn="dubins", **over):
    """One OBCA instance (oracle/nlp.py instance format) for problem id `pid`; `turn` is one of
    TURN_TYPES or "mixed" (see the module docstring)."""
    rng = np.random.Generator(np.random.Philox(key=[key, pid]))
    if turn == "mixed":
        turn = TURN_TYPES[int(np.random.Generator(np.random.Philox(key=[key + 1, pid])).integers(0, 3))]
    if turn not in TURN_TYPES:
        raise ValueError("unknown turn type %r" % (turn,))
    veh = dict(VEHICLE)
    r_min = veh["wheelbase"] / math.tan(veh["max_steer"])
    body = geometry.body_rectangle(veh["axle_to_front"], veh["axle_to_back"], veh["width"])
    polys = [body]
    feat = IMPLEMENTS[implement]
    if feat is not None:
        polys.append(geometry.implement_rectangle(feat))

    for _attempt in range(64):
        rows = 8
        row_w = rng.uniform(2.2, 3.5)
        slope = math.radians(rng.uniform(-15.0, 15.0))
        l_std = [0.0, 1.0][int(rng.integers(0, 2))]
        tree_w, row_len = 0.3, 20.0
        xs0 = np.array([row_w * math.tan(slope) * i + rng.uniform(-l_std, l_std) for i in range(rows)])
        ys0 = row_w * np.arange(rows)
        s_row = int(rng.integers(0, 5))
        e_row = min(s_row + int(rng.integers(1, 4)), rows - 2)
        if turn != "dubins":   # fish-tail / circle-back turns go to the adjacent row
            e_row = s_row + 1
        exit_off = rng.uniform(-1.0, 1.0)
        enter_off = rng.uniform(0.0, 3.66)
        margin = rng.uniform(0.3, 1.0)

        near = lambda r: np.array([(xs0[r] + xs0[r + 1]) / 2.0, (ys0[r] + ys0[r + 1]) / 2.0])
        ps = near(s_row) + np.array([-1.0, 0.0]) * exit_off   # LEAVE, yaw = pi
        pe = near(e_row) - np.array([1.0, 0.0]) * enter_off   # ENTER, yaw = 0
        q0 = (ps[0], ps[1], math.pi)
        q1 = (pe[0], pe[1], 0.0)
        segs = None
        if turn == "circleback":
            segs = circle_back_segments(q0, q1, r_min)
        elif turn == "fishtail":
            segs = fishtail_segments(q0, q1, r_min)
        if segs is None:   # "dubins", or rows 2R or more apart (the reference's Dubins fallback)
            used = "dubins"
            name, seg = dubins_shortest(q0, q1, r_min)
            Lp = sum(seg) * r_min
            smp = dubins_sample(q0, r_min, name, seg, np.linspace(0.0, Lp, N))
            gear = np.ones(N)
        else:
            used = turn
            name = "".join("S" if k == 0.0 else ("L" if k > 0 else "R") + ("-" if u < 0 else "+") for k, u in segs)
            Lp = sum(abs(u) for _, u in segs)
            smp = segments_sample(q0, segs, np.linspace(0.0, Lp, N))
            gear = smp[:, 4]
        # footprint of the warm start (every pose, body + implements)
        foot = [_polys_at(p, smp[:, :3]) for p in polys]
        allpts = np.concatenate([f.reshape(-1, 2) for f in foot])
        x_b = allpts[:, 0].min() - margin
        obstacles = [_rect(x_b - 2.0, x_b, ys0.min() - 8.0, ys0.max() + 8.0)]
        row_order = list(range(s_row + 1, e_row + 1)) + [s_row, e_row + 1]
        for rr in [s_row - 1, e_row + 2]:
            if 0 <= rr < rows:
                row_order.append(rr)
        row_rects = [_rect(xs0[r] - 0.2, xs0[r] + row_len + 0.2, ys0[r] - tree_w / 2, ys0[r] + tree_w / 2)
                     for r in row_order]
        up = _rect(xs0.min() - 8.0, xs0.max() + row_len + 8.0, ys0.max() + row_w, ys0.max() + row_w + 1.0)
        cand = obstacles + row_rects + [up]
        ok = all(_min_sat_gap(f, o) > 0.02 for o in cand[:M] for f in foot)
        if ok:
            break
    cand = cand[:M]
    k = 0
    while len(cand) < M:  # far dummy quads
        cx = ps[0] + 60.0 + 5.0 * k
        cand.append(_rect(cx, cx + 1.0, ps[1] + 60.0, ps[1] + 61.0))
        k += 1

    dT = float(over.get("dT", DEFAULT_WEIGHTS["dT"]))
    ds = Lp / (N - 1)
    desired_v = min(ds / dT, 0.9)
    traj = np.zeros((N, 5))
    traj[:, 0], traj[:, 1] = smp[:, 0], smp[:, 1]
    traj[:, 2] = desired_v * gear
    traj[:, 3] = process_angle(smp[:, 2])
    traj[:, 4] = np.arctan(veh["wheelbase"] * smp[:, 3])
    traj[0, 2] = traj[-1, 2] = 0.0
    traj[0, 4] = 0.0

    obs_A, obs_b = zip(*[geometry.polytope_halfspaces(o) for o in cand])
    body_G, body_g = zip(*[geometry.polytope_halfspaces(p) for p in polys])
    inst = dict(
        init_traj=traj, obs_A=list(obs_A), obs_b=list(obs_b), body_G=list(body_G), body_g=list(body_g),
        obstacles=cand, dT=dT, Q=DEFAULT_WEIGHTS["Q"].copy(), R=DEFAULT_WEIGHTS["R"].copy(),
        W=DEFAULT_WEIGHTS["W"].copy(), wheelbase=veh["wheelbase"], max_steer=veh["max_steer"],
        max_velocity=1.0, max_accel=1.0, max_steer_rate=0.7, min_dist=0.1,
        x_bound=[-np.inf, np.inf], y_bound=[-np.inf, np.inf],
        meta=dict(pid=pid, turn=used, dubins=name, length=Lp, start=q0, goal=q1, s_row=s_row, e_row=e_row),
    )
    for kk, vv in over.items():
        inst[kk] = vv
    return inst


def make_points_instance(pid, N=80, M=6, implement="none", key=20251015, **over):
    """The same synthetic headland turn in the point formulation (oracle/nlp_points.py instance
    format, R/obca_py/optimizer_points.py): obstacle halfspaces, vehicle hull vertices
    (get_vehicle_vertices :35-50), the reference's default x/y bounds (initialize_manual :52-62)."""
    base = make_instance(pid, N=N, M=M, implement=implement, key=key)
    veh = VEHICLE
    # hard start/end constraints (no terminal slack): give the turn time enough to be feasible
    # (cruise <= 0.5 m/s, MAX_VELOCITY 1, MAX_ACCEL 1, MAX_STEER_RATE 0.7)
    ds = base["meta"]["length"] / (N - 1)
    dT = float(over.get("dT", max(base["dT"], ds / 0.5)))
    traj = base["init_traj"].copy()
    traj[1:-1, 2] = ds / dT
    polys = [geometry.body_rectangle(veh["axle_to_front"], veh["axle_to_back"], veh["width"])]
    if IMPLEMENTS[implement] is not None:
        polys.append(geometry.implement_rectangle(IMPLEMENTS[implement]))
    inst = dict(
        init_traj=traj, obs_A=base["obs_A"], obs_b=base["obs_b"], obstacles=base["obstacles"],
        vertices=geometry.vehicle_hull_vertices(polys), dT=dT, wheelbase=veh["wheelbase"],
        max_steer=veh["max_steer"], max_velocity=1.0, max_accel=1.0, max_steer_rate=0.7, min_dist=0.1,
        x_bound=[-9999999.0, 9999999.0], y_bound=[-9999999.0, 9999999.0], meta=base["meta"],
    )
    for kk, vv in over.items():
        inst[kk] = vv
    return inst


# ------------------------------------------------ the reference's own scene producers
# Configs A-E are built by the reference's planners and obstacle producer (restated in
# path_planner/), not by the hand-placed rectangles of make_instance:
#   tree rows ........ map_utils.create_tree_rows (R/path_planner/utils/map_utils.py:45-61)
#   row poses ........ get_base_pose (map_utils.py:228-271), NEAR side
#   warm start ....... dubins:     get_warm_start_path_dubins (R/path_planner/OBCA_warm_start.py:166-174)
#                      circleback: get_circle_back_path_full (R/path_planner/safety_forward_path_plan.py:395-454)
#                      fishtail:   get_start_end_pose_for_reeds_shepp (:300-364) + the Reeds-Shepp word with the
#                                  least backward length among the collision-free ones + Dubins lead-in/out
#                                  (R/test/classic_planner.ipynb cells 10-11)
#   init guess ....... get_init_ref_path (R/obca_py/util.py:62-113) at desired_v = ds / dT, resampled to N rows
#   obstacles ........ orchard_environment_OBCA.create_boundary_polygons / get_obstacle_tree_rows /
#                      get_obstacles_for_OBCA (R/path_planner/OGE_OBCA.py:306-373,477-677)
# The reference's global np.random draws (create_tree_rows :33, create_headland_countour_lines
# orchard_geometry_environment.py:71) come from an MT19937 stream seeded per problem from its Philox
# stream, so a problem is identical for any batch composition and any GPU count.
_CPU_LIB = None
SAFETY_BOUND = 0.2   # orchard_environment_OBCA.SAFETY_BOUND: the row rectangles' margin past the row ends


def _cpu_lib():
    global _CPU_LIB
    if _CPU_LIB is None:
        import ctypes
        import os
        so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhtp_cpu.so")
        lib = ctypes.CDLL(so)
        f = lib.htp_cpu_rs_all_paths
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 11
        _CPU_LIB = lib
    return _CPU_LIB


class _RSPath:
    __slots__ = ("lengths", "ctypes", "L", "x", "y", "yaw", "cs", "directions")


def host_rs_all_paths(sx, sy, syaw, gx, gy, gyaw, maxc, step_size):
    """calc_all_paths (R/path_planner/utils/reeds_shepp.py:39-65) on the host through the CPU build of
    csrc/rs_core.h (libhtp_cpu.so) -- the generator runs before the GPU is touched."""
    import ctypes  # noqa: F401
    f = _cpu_lib().htp_cpu_rs_all_paths
    q = np.array([sx, sy, syaw, gx, gy, gyaw, maxc, step_size], dtype=np.float64)
    n_p, n_q = np.zeros(1, np.int32), np.zeros(1, np.int64)
    cp, cq = 48, 4096
    for _ in range(2):
        ln, ct, L = np.zeros((cp, 5)), np.zeros((cp, 5), np.int8), np.zeros(cp)
        off = np.zeros(cp + 1, np.int64)
        x, y, yaw, cs = (np.zeros(cq) for _ in range(4))
        d = np.zeros(cq, np.int8)
        st = f(q.ctypes.data, cp, cq, n_p.ctypes.data, n_q.ctypes.data, ln.ctypes.data, ct.ctypes.data,
               L.ctypes.data, off.ctypes.data, x.ctypes.data, y.ctypes.data, yaw.ctypes.data, cs.ctypes.data,
               d.ctypes.data)
        if cp >= n_p[0] and cq >= n_q[0]:
            break
        cp, cq = int(n_p[0]), int(n_q[0])
    if st != 0:
        raise ValueError("[synth] Reeds-Shepp sampler status %d" % st)
    out = []
    for k in range(int(n_p[0])):
        p = _RSPath()
        nseg = int(np.count_nonzero(ct[k] != 3))
        a, b = int(off[k]), int(off[k + 1])
        p.lengths, p.ctypes, p.L = ln[k, :nseg].copy(), ["LSR-"[t] for t in ct[k, :nseg]], float(L[k])
        p.x, p.y, p.yaw, p.cs, p.directions = x[a:b].copy(), y[a:b].copy(), yaw[a:b].copy(), cs[a:b].copy(), \
            d[a:b].astype(np.float64)
        out.append(p)
    return out


class _legacy_random:
    """Seed numpy's global MT19937 stream (the reference draws from np.random.*) and restore it after."""

    def __init__(self, seed):
        self.seed = int(seed)

    def __enter__(self):
        self.saved = np.random.get_state()
        np.random.seed(self.seed)

    def __exit__(self, *exc):
        np.random.set_state(self.saved)
        return False


def _fishtail_path(tree_rows, s_row, e_row, car, empty, env, start, end, exit_off, enter_off):
    """classic_planner.ipynb cells 10-11 (R/path_planner/safety_forward_path_plan.py:300-364 + the word
    choice): rows [x, y, yaw, k, dir] or None when no Reeds-Shepp word clears the rows."""
    from .path_planner import map_utils
    from .path_planner import safety_forward_path_plan as sfp
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        safe_start, safe_end, leave_off, enter_off = sfp.get_start_end_pose_for_reeds_shepp(
            tree_rows, s_row, e_row, car, env, max_steer_angle=0.55, side=map_utils.NEAR_SIDE,
            extra_offset_enter_dist=enter_off, extra_offset_leave_dist=exit_off)
    paths = host_rs_all_paths(safe_start[0], safe_start[1], safe_start[2], safe_end[0], safe_end[1], safe_end[2],
                              car.curvature, 0.1)
    optimal, best = None, 99999
    for p in paths:
        traj = np.array([p.x, p.y, p.yaw]).T
        if env.check_path_feasibility(empty, traj, boundary_check=False):
            lengths = np.array(p.lengths)
            cost = np.abs(lengths[lengths < 0].sum())
            if cost < best:
                optimal, best = p, cost
    if optimal is None:
        return None
    path = np.array([optimal.x, optimal.y, optimal.yaw, optimal.cs, optimal.directions]).T
    r = 1.0 / car.curvature
    if leave_off > 0.1:
        path = np.vstack([sfp.get_dubins_path_full(start, safe_start, r)[:-1], path])
    if enter_off > 0.1:
        path = np.vstack([path, sfp.get_dubins_path_full(safe_end, end, r)[1:]])
    return path


def _warm_start_path(turn, tree_rows, s_row, e_row, car, empty, env, start, end, exit_off, enter_off):
    from .path_planner import map_utils
    from .path_planner import safety_forward_path_plan as sfp
    r = 1.0 / car.curvature
    if turn == "fishtail":
        return _fishtail_path(tree_rows, s_row, e_row, car, empty, env, start, end, exit_off, enter_off)
    if turn == "circleback":
        return sfp.get_circle_back_path_full(start, end, r, car, side=map_utils.NEAR_SIDE, step_size=0.1)
    return sfp.get_dubins_path_full(start, end, r, step_size=0.1)      # OBCA_warm_start.py:166-174


def _resample_rows(ref, N):
    """get_init_ref_path output (rows [x, y, v, theta, steer]) -> exactly N rows at even arc length
    (x, y, theta, steer interpolated; v = the gear speed of the covering row; v[0] = v[-1] = steer[0] = 0)."""
    seg = np.hypot(np.diff(ref[:, 0]), np.diff(ref[:, 1]))
    s = np.concatenate([[0.0], np.cumsum(seg)])
    t = np.linspace(0.0, s[-1], N)
    out = np.zeros((N, 5))
    for c in (0, 1, 3, 4):
        out[:, c] = np.interp(t, s, ref[:, c])
    idx = np.clip(np.searchsorted(s, t, side="right"), 1, len(s) - 1)
    v = ref[idx, 2]
    v = np.where(v == 0.0, ref[idx - 1, 2], v)
    out[:, 2] = v
    out[0, 2] = out[-1, 2] = 0.0
    out[0, 4] = 0.0
    return out


def _split_quads(poly):
    """A convex k-gon (k >= 5) as overlapping convex quads [v0, v_i, v_i+1, v_i+2] whose union is the
    polygon: the OBCA distance constraint to each piece holds iff it holds to the union, so the
    free space is unchanged while every obstacle slot of a batch keeps 4 edges."""
    P = np.asarray(poly, dtype=np.float64)
    if P.shape[0] <= 4:
        return [P]
    out, i = [], 1
    while True:
        j = min(i, P.shape[0] - 3)
        out.append(np.vstack([P[0], P[j], P[j + 1], P[j + 2]]))
        if j + 2 >= P.shape[0] - 1:
            return out
        i += 2


def _needed_headland(tree_rows, pts, angle):
    """Smallest headland_width whose field boundary (get_map_exterior_pts :288-334, near side) leaves
    every point inside: boundary x(y) = near row end x(y) - width / |sin(angle)|."""
    ys, xs = tree_rows[:, 0, 1], tree_rows[:, 0, 0]
    o = np.argsort(ys)
    xr = np.interp(pts[:, 1], ys[o], xs[o])
    return float(np.max(xr - pts[:, 0])) * abs(math.sin(angle))


def _tree_row_range(tree_rows, start, end):
    """Row indices [a, c) get_obstacle_tree_rows (OGE_OBCA.py:477-591) turns into obstacles."""
    hi, lo = max(start[1], end[1]), min(start[1], end[1])
    idxs = np.sort(np.where((tree_rows[:, 0, 1] > lo) & (tree_rows[:, 0, 1] < hi))[0])
    n = len(tree_rows)
    if idxs[0] == idxs[-1]:
        return max(idxs[-1] - 2, 0), min(idxs[-1] + 2, n - 1)
    return max(idxs[0] - 2, 0), min(idxs[-1] + 3, n - 1)


def make_orchard_instance(pid, N=80, M=6, implement="none", key=20251015, turn="dubins", **over):
    """One OBCA instance whose scene and warm start come from the reference's producers (see the block
    comment above).  Draws per attempt: row width U[2.2, 3.5], slope U[-15, 15] deg, l_std in {0, 1},
    start row 0..4, row jump 1..3 (1 for fish-tail / circle-back), leave offset U[-1, 1], enter offset
    U[0, 3.66], boundary margin U[0.3, 1.0].  The headland is 6 m (the notebooks' value) or wider when the
    warm start needs it (boundary = margin behind its footprint); an attempt is redrawn when the planner
    finds no path, when its path fails the reference's footprint predicate against the tree rows
    (check_path_feasibility, implements included), or when the OBCA init guess reaches deeper than the
    rows' SAFETY_BOUND into an obstacle -- as in the reference, the warm start may start inside that
    0.2 m margin, which OBCA (min_dist 0.1) then clears.  Obstacles: the
    producer's list in its order (k-gons split into overlapping quads); with more than M the M closest to
    the warm start are kept, with fewer the other tree rows of the orchard (nearest first) and the other
    bound quad are added (far dummy quads only if the orchard has none left)."""
    from .path_planner import map_utils
    from .path_planner.car_model import CarModel
    from .path_planner.OGE_OBCA import orchard_environment_OBCA
    from .obca_py.util import get_init_ref_path

    rng = np.random.Generator(np.random.Philox(key=[key, pid]))
    if turn == "mixed":
        turn = TURN_TYPES[int(np.random.Generator(np.random.Philox(key=[key + 1, pid])).integers(0, 3))]
    if turn not in TURN_TYPES:
        raise ValueError("unknown turn type %r" % (turn,))
    veh = dict(VEHICLE)
    feat = IMPLEMENTS[implement]
    car = CarModel(max_steer=veh["max_steer"], wheel_base=veh["wheelbase"], axle_to_front=veh["axle_to_front"],
                   axle_to_back=veh["axle_to_back"], width=veh["width"],
                   aux_poly_features=[feat] if feat is not None else [], with_aux=feat is not None)
    empty = CarModel(max_steer=veh["max_steer"], wheel_base=veh["wheelbase"], axle_to_front=veh["axle_to_front"],
                     axle_to_back=veh["axle_to_back"], width=veh["width"], with_aux=False)
    polys = [geometry.body_rectangle(veh["axle_to_front"], veh["axle_to_back"], veh["width"])]
    if feat is not None:
        polys.append(geometry.implement_rectangle(feat))
    dT = float(over.get("dT", DEFAULT_WEIGHTS["dT"]))
    rows_n, row_len, tree_w = max(8, M), 20.0, 0.3   # 8 rows; more when M asks for more obstacles
    cand = None
    for _attempt in range(64):
        row_w = rng.uniform(2.2, 3.5)
        slope = math.radians(rng.uniform(-15.0, 15.0))
        l_std = [0.0, 1.0][int(rng.integers(0, 2))]
        s_row = int(rng.integers(0, 5))
        e_row = min(s_row + int(rng.integers(1, 4)), rows_n - 2)
        if turn != "dubins":
            e_row = s_row + 1
        exit_off = rng.uniform(-1.0, 1.0)
        enter_off = rng.uniform(0.0, 3.66)
        margin = rng.uniform(0.3, 1.0)
        seed = int(rng.integers(0, 2 ** 31 - 1))
        with _legacy_random(seed):
            tree_rows = map_utils.create_tree_rows(rows_n, row_w, row_len, slope_angle=slope, l_std=l_std)
        start = map_utils.get_base_pose(s_row, tree_rows, exit_off, side=map_utils.NEAR_SIDE,
                                        pose_type=map_utils.LEAVE_POSE)
        end = map_utils.get_base_pose(e_row, tree_rows, enter_off, side=map_utils.NEAR_SIDE,
                                      pose_type=map_utils.ENTER_POSE)
        env = orchard_environment_OBCA(tree_rows, [], tree_width=tree_w, headland_width=6.0)
        try:
            path = _warm_start_path(turn, tree_rows, s_row, e_row, car, empty, env, start, end, exit_off, enter_off)
        except (ValueError, IndexError, ZeroDivisionError, RuntimeError):
            path = None
        if path is None or len(path) < 4:
            continue
        # the reference's own footprint predicate on the whole warm start (tree rows, implements included;
        # orchard_geometry_environment.py:423-458): a planner output that fails it is redrawn
        if not env.check_path_feasibility(car, path[:, :3], boundary_check=False, aux_check=True):
            continue
        # a forward Dubins turn is the reference's first choice only when it clears the rows buffered to
        # tree_width_in_forward_plan (headland_planner_y_type_park_combined, headland_path_planning.py:55-121;
        # 0.4 in R/test/obca.ipynb) -- otherwise the reference plans a Y-park + hybrid A* turn instead
        if turn == "dubins":
            env_fwd = orchard_environment_OBCA(tree_rows, [], tree_width=0.4, headland_width=6.0)
            if not env_fwd.check_path_feasibility(empty, path[:, :3], boundary_check=False):
                continue
        Lp = float(np.sum(np.hypot(np.diff(path[:, 0]), np.diff(path[:, 1]))))
        ds = Lp / (N - 1)
        desired_v = min(ds / dT, 0.9)
        try:
            # spline spacing half the resampled spacing, Lp / (2 N - 2): a single-gear turn's sample count
            # len(np.arange(0, S + ds, ds)) then sits on an exact integer tie (S = Lp up to summation order), which
            # the last bit of the libm decides -- the device and host builds share one correctly rounded libm
            # (csrc/htp_libm.h), so they decide it alike (tests/test_gpu_e2e.py)
            ref = get_init_ref_path(car, path[:, 0], path[:, 1], path[:, 2], path[:, 3], path[:, 4],
                                    desired_v=desired_v, ds=Lp / (2.0 * N - 2.0))
        except ValueError:
            continue
        traj = _resample_rows(ref, N)
        poses = np.stack([traj[:, 0], traj[:, 1], traj[:, 3]], axis=1)
        dense = np.stack([ref[:, 0], ref[:, 1], ref[:, 3]], axis=1)
        foot = [_polys_at(p, np.vstack([poses, dense])) for p in polys]
        pts = np.concatenate([f.reshape(-1, 2) for f in foot])
        hw = max(6.0, _needed_headland(tree_rows, pts, env.get_headland_angle(env.NEAR_SIDE)) + margin)
        env = orchard_environment_OBCA(tree_rows, [], tree_width=tree_w, headland_width=hw)
        try:   # the reference raises IndexError when no boundary piece lies beside the turn: redraw
            with _legacy_random(seed + 1):
                boundary = env.create_boundary_polygons()
            row_polys = env.get_obstacle_tree_rows(start, end)
            obs = env.get_obstacles_for_OBCA(boundary, row_polys, start, end, side=env.NEAR_SIDE)
        except (IndexError, ValueError):
            continue
        pool = [q for o in obs for q in _split_quads(o)]
        if len(pool) < M:   # the rest of the orchard: other tree rows (nearest first), the other bound quad
            a, c = _tree_row_range(tree_rows, start, end)
            mid = 0.5 * (start[1] + end[1])
            extra = sorted((abs(r[0, 1] - mid), i) for i, r in enumerate(tree_rows) if not a <= i < c)
            pool += [env._row_rect(tree_rows[i], False) for _, i in extra]
            pool += [p for p in (boundary[3] if start[1] > end[1] else boundary[2])]
        gaps = np.array([min(_min_sat_gap(f, q) for f in foot) for q in pool])
        if np.any(gaps <= -SAFETY_BOUND):   # deeper than the rows' SAFETY_BOUND margin (OGE_OBCA.py:411-475)
            continue
        if len(pool) > M:
            keep = sorted(np.argsort(gaps, kind="stable")[:M])
            pool = [pool[k] for k in keep]
        cand = pool
        break
    if cand is None:
        raise RuntimeError("[synth] problem %d: no collision-free warm start in 64 attempts" % pid)
    k = 0
    while len(cand) < M:  # far dummy quads (only when the orchard has no obstacle left)
        cx = start[0] + 60.0 + 5.0 * k
        cand.append(_rect(cx, cx + 1.0, start[1] + 60.0, start[1] + 61.0))
        k += 1
    obs_A, obs_b = zip(*[geometry.polytope_halfspaces(o) for o in cand])
    body_G, body_g = zip(*[geometry.polytope_halfspaces(p) for p in polys])
    inst = dict(
        init_traj=traj, obs_A=list(obs_A), obs_b=list(obs_b), body_G=list(body_G), body_g=list(body_g),
        obstacles=cand, dT=dT, Q=DEFAULT_WEIGHTS["Q"].copy(), R=DEFAULT_WEIGHTS["R"].copy(),
        W=DEFAULT_WEIGHTS["W"].copy(), wheelbase=veh["wheelbase"], max_steer=veh["max_steer"],
        max_velocity=1.0, max_accel=1.0, max_steer_rate=0.7, min_dist=0.1,
        x_bound=[-np.inf, np.inf], y_bound=[-np.inf, np.inf],
        meta=dict(pid=pid, turn=turn, length=Lp, start=tuple(start), goal=tuple(end), s_row=s_row, e_row=e_row,
                  headland_width=hw, n_producer=len(obs), n_dummy=k, l_std=l_std, nrows=rows_n, row_width=row_w,
                  row_length=row_len, slope=slope, tree_width=tree_w, seed=seed, exit_off=exit_off,
                  enter_off=enter_off, margin=margin, implement=implement),
    )
    for kk, vv in over.items():
        inst[kk] = vv
    return inst


def orchard_scene(meta):
    """The scene of a make_orchard_instance problem as the device producer takes it (htp_oge_obstacles_batch,
    _native.OgePacked): geometry plus the reference's np.random draws, regenerated from the problem's MT19937
    seeds (create_tree_rows: one uniform(-l_std, l_std) per row under `seed`; create_headland_countour_lines:
    uniform(-0.5, 0.5, size=rows) under `seed + 1`)."""
    n = int(meta["nrows"])
    with _legacy_random(meta["seed"]):
        row_draws = np.array([np.random.uniform(-meta["l_std"], meta["l_std"]) for _ in range(n)])
    with _legacy_random(meta["seed"] + 1):
        eps_draws = np.random.uniform(-0.5, 0.5, size=(n,))
    return dict(nrows=n, row_width=meta["row_width"], row_length=meta["row_length"], slope=meta["slope"],
                tree_width=meta["tree_width"], headland_width=meta["headland_width"], start=meta["start"],
                end=meta["goal"], side=1, row_draws=row_draws, eps_draws=eps_draws)


def orchard_obstacles_host(meta):
    """The reference producer's obstacle list for the same scene, through the Python restatement
    (orchard_environment_OBCA); the device producer is pinned against it."""
    from .path_planner import map_utils
    from .path_planner.OGE_OBCA import orchard_environment_OBCA
    with _legacy_random(meta["seed"]):
        rows = map_utils.create_tree_rows(int(meta["nrows"]), meta["row_width"], meta["row_length"],
                                          slope_angle=meta["slope"], l_std=meta["l_std"])
    env = orchard_environment_OBCA(rows, [], tree_width=meta["tree_width"], headland_width=meta["headland_width"])
    with _legacy_random(meta["seed"] + 1):
        boundary = env.create_boundary_polygons()
    row_polys = env.get_obstacle_tree_rows(meta["start"], meta["goal"])
    return env.get_obstacles_for_OBCA(boundary, row_polys, meta["start"], meta["goal"], side=env.NEAR_SIDE)


def _orchard_env(meta):
    from .path_planner import map_utils
    from .path_planner.OGE_OBCA import orchard_environment_OBCA
    with _legacy_random(meta["seed"]):
        rows = map_utils.create_tree_rows(int(meta["nrows"]), meta["row_width"], meta["row_length"],
                                          slope_angle=meta["slope"], l_std=meta["l_std"])
    return rows, orchard_environment_OBCA(rows, [], tree_width=meta["tree_width"], headland_width=6.0)


def classic_turn(meta):
    """The warm-start planner call of a make_orchard_instance problem as the device planner takes it
    (htp_classic_turn_batch, _native.ClassicPacked): turn type, row poses, car, and the blocker polygons
    (env.obs_poly_list) the fish-tail's footprint checks use."""
    from .path_planner.geom import ring_of
    _, env = _orchard_env(meta)
    veh = VEHICLE
    body = geometry.body_rectangle(veh["axle_to_front"], veh["axle_to_back"], veh["width"])
    r = 1.0 / (math.tan(veh["max_steer"]) / veh["wheelbase"])
    return dict(type=meta["turn"], side=1, start=meta["start"], end=meta["goal"], wheel_base=veh["wheelbase"],
                max_steer=veh["max_steer"], radius=r, step=0.1, body=body,
                blockers=[ring_of(q) for q in env.obs_poly_list])


def classic_turn_host(meta, implement="none"):
    """The same call through the host planners (path_planner/, the restated reference) -> rows [x, y, yaw, k, dir]."""
    from .path_planner.car_model import CarModel
    rows, env = _orchard_env(meta)
    veh = VEHICLE
    feat = IMPLEMENTS[implement]
    car = CarModel(max_steer=veh["max_steer"], wheel_base=veh["wheelbase"], axle_to_front=veh["axle_to_front"],
                   axle_to_back=veh["axle_to_back"], width=veh["width"],
                   aux_poly_features=[feat] if feat is not None else [], with_aux=feat is not None)
    empty = CarModel(max_steer=veh["max_steer"], wheel_base=veh["wheelbase"], axle_to_front=veh["axle_to_front"],
                     axle_to_back=veh["axle_to_back"], width=veh["width"], with_aux=False)
    return _warm_start_path(meta["turn"], rows, meta["s_row"], meta["e_row"], car, empty, env,
                            np.asarray(meta["start"]), np.asarray(meta["goal"]), meta["exit_off"], meta["enter_off"])


# turn types of the BASELINE configs: A fish-tail, B Omega/circle-back, C mixed, D/E the Dubins turn
TURNS = {"A": "fishtail", "B": "circleback", "C": "mixed", "D": "dubins", "E": "dubins"}


def config_instance(cfg, pid, **over):
    """Problem `pid` of BASELINE config `cfg` (shape, implement and turn type), scene and warm start from
    the reference's producers (make_orchard_instance)."""
    _, N, M, imp = CONFIGS[cfg]
    return make_orchard_instance(pid, N=N, M=M, implement=imp, turn=TURNS[cfg], **over)


CONFIGS = {
    # name: (batch, N, M, implement)  -- BASELINE.json configs[0..4]
    "A": (1, 40, 2, "none"),
    "B": (256, 80, 6, "none"),
    "C": (4096, 80, 6, "mower"),
    "D": (32768, 80, 6, "none"),
    "E": (4096, 160, 12, "pruner"),
}
