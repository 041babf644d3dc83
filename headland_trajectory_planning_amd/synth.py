"""Deterministic synthetic headland-turn workload.

Problem `pid` is drawn from Philox(key=[20251015, pid]) so a problem is
identical for any batch composition and any GPU count.

Geometry follows the reference's orchard model:
* tree rows  ........... R/path_planner/utils/map_utils.py:45-61 (create_tree_rows)
* exit / enter poses ... map_utils.py:228-271 (get_base_pose, NEAR_SIDE)
* obstacles ............ R/path_planner/OGE_OBCA.py:306-373,477-677: a headland
  boundary quad, the up/low bound quad and tree-row rectangles (SAFETY_BOUND 0.2),
  trimmed / padded to exactly M convex quads (padding: far dummy quads, >= 50 m away)
* warm start ........... one of the reference's turn types (`turn=`):
  - "dubins": the Dubins fallback (R/path_planner/OBCA_warm_start.py:166-174,
    pydubins shortest path);
  - "circleback": the circle-back / Omega turn of
    R/path_planner/safety_forward_path_plan.py:395-454 (forward arc R_f by
    theta, reverse arc R_b by pi - theta, Dubins lead-in; radii grow 5 % until
    the reverse arc ends short of the row; rows wider than 2R fall back to Dubins);
  - "fishtail": a three-arc C|C|C K-turn (forward, reverse, forward at the
    minimum radius, symmetric outer arcs) joined to the row poses by straights --
    the Reeds-Shepp C|C|C family the fish-tail planner
    (safety_forward_path_plan.py:300-392) picks between offset poses of one x;
    rows wider than 2R fall back to Dubins;
  - "mixed": one of the three per problem (its own Philox stream, key + 1).
  The path is sampled to exactly N poses and turned into [x, y, v, theta, steer]
  as R/obca_py/util.py:62-113 does (v = dir*desired_v, steer = atan(L*kappa)
  with kappa the steering curvature, v[0]=v[-1]=steer[0]=0, heading wrapped +
  unwrapped).

The headland boundary is placed behind the warm start's swept footprint with a
random margin, so every instance starts collision-free and the boundary is
close to active -- the regime the reference notebooks exercise.
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


# turn types of the BASELINE configs: A fish-tail, B Omega/circle-back, C mixed, D/E the Dubins turn
TURNS = {"A": "fishtail", "B": "circleback", "C": "mixed", "D": "dubins", "E": "dubins"}


def config_instance(cfg, pid, **over):
    """Problem `pid` of BASELINE config `cfg` (shape, implement and turn type)."""
    _, N, M, imp = CONFIGS[cfg]
    return make_instance(pid, N=N, M=M, implement=imp, turn=TURNS[cfg], **over)


CONFIGS = {
    # name: (batch, N, M, implement)  -- BASELINE.json configs[0..4]
    "A": (1, 40, 2, "none"),
    "B": (256, 80, 6, "none"),
    "C": (4096, 80, 6, "mower"),
    "D": (32768, 80, 6, "none"),
    "E": (4096, 160, 12, "pruner"),
}
