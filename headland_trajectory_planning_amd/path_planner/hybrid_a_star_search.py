"""HybridAStarSearch of R/path_planner/hybrid_a_star_search.py, searched on the GPU.

Drop-in surface: `HybridAStarSearch(start_pose, goal_pose, config_environment,
car_model, search_heuristic, motion_type, yaw_resolution, plan_resolution)`
(:38-74) and `.hybrid_a_star_search(plt=None, max_nodes=2000) -> (xs, ys,
yaws, dirs, ks, counter)` (:497-607), plus the batched
`hybrid_a_star_search_batch(searches, max_nodes)` for many start/goal pairs at
once.  The environment and heuristic are lowered to polygons
(`lower_problem`) and every search runs as one wavefront of the
htp_hastar_search_batch kernel (libhtp.so, csrc/hastar_core.h).  There is no
CPU fallback: the HIP library must be built.

Duck types read by the lowering (the reference's own objects work too):
  car_model           .car_poly, .WHEEL_BASE, .MAX_STEER (curvature = tan(MAX_STEER)/WHEEL_BASE, car_model.py:34)
  config_environment  .tree_polys, .obstacle_polys, .field_range_poly (check_path_feasibility :423-437)
  search_heuristic    .segment_lanes, .search_lengths, .guided_path, .default_search_length
Motion type "Pawn" takes Dubins goal shots (pydubins restated in
csrc/dubins_core.h, re-splined like get_dubins_path :289-304); "King" takes
Reeds-Shepp shots.
"""
import math
import time

import numpy as np

from .. import _native
from .geom import ring_of

STATUS_FOUND, STATUS_NO_PATH, STATUS_MAX_NODES, STATUS_BLOCKED = 0, 1, 2, 3


def motion_steers(max_steer, yaw_resolution, motion_type):
    """_get_motion_steers_dubins :331-341 / _get_motion_steers_reeds_shepp :343-354."""
    if motion_type == "King":
        s = np.arange(max_steer, -(max_steer + yaw_resolution / 2.0), -yaw_resolution / 2.0)
        d = np.ones_like(s)
        d[1:len(d):2] = -1
    else:
        s = np.arange(max_steer, -(max_steer + yaw_resolution), -yaw_resolution)
        d = np.ones_like(s)
    return np.vstack((s, d)).T


def lower_problem(start_pose, goal_pose, config_environment, car_model, search_heuristic, motion_type="King",
                  yaw_resolution=math.radians(10), plan_resolution=0.1, max_nodes=2000):
    """Flat polygon description of one search (input of _native.HastarPacked)."""
    env, heur = config_environment, search_heuristic
    return dict(
        start=np.asarray(start_pose, dtype=np.float64)[:3], goal=np.asarray(goal_pose, dtype=np.float64)[:3],
        body=ring_of(car_model.car_poly),
        blockers=[ring_of(p) for p in list(env.obstacle_polys) + list(env.tree_polys)],
        field=ring_of(env.field_range_poly),
        lanes=[ring_of(p) for p in heur.segment_lanes],
        search_lengths=np.asarray(heur.search_lengths, dtype=np.float64),
        guide=np.asarray(heur.guided_path, dtype=np.float64)[:, :4],
        king=(motion_type == "King"), res=float(plan_resolution), yaw_res=float(yaw_resolution),
        max_nodes=int(max_nodes), wheel_base=float(car_model.WHEEL_BASE), max_steer=float(car_model.MAX_STEER),
        curvature=math.tan(car_model.MAX_STEER) / car_model.WHEEL_BASE,
        default_search_length=float(heur.default_search_length),
        motions=motion_steers(car_model.MAX_STEER, yaw_resolution, motion_type))


# Per-search limits of the device search (include/htp.h HTP_HA_MAX_*, hastar_core.h valid_search).  The reference
# has none; its planners' settings stay far inside them (King: 14 motions x 16 poses of 512).
MAX_BODY, MAX_LANES, MAX_MOTIONS, MAX_POSES, TRAJ_CAP = 8, 32, 16, 64, 512


def check_limits(p):
    """Raise ValueError, naming the limit, for a lowered search the device would reject (HTP_HA_BAD_INPUT): every
    search length L (the default and each lane's) needs n = rint(L / res) >= 1 with n + 1 <= MAX_POSES poses per
    motion primitive and nmotions * (n + 1) <= TRAJ_CAP (one expansion's rollouts are held in LDS)."""
    nmot = len(p["motions"])
    if not 1 <= nmot <= MAX_MOTIONS:
        raise ValueError(f"[HA*] {nmot} motion primitives; the device search takes 1..{MAX_MOTIONS}")
    nb = len(_native._clean_ring(p["body"]))
    if not 3 <= nb <= MAX_BODY:
        raise ValueError(f"[HA*] body polygon with {nb} vertices; the device search takes 3..{MAX_BODY}")
    if not 1 <= len(p["lanes"]) <= MAX_LANES:
        raise ValueError(f"[HA*] {len(p['lanes'])} lane polygons; the device search takes 1..{MAX_LANES}")
    for L in [p["default_search_length"]] + [float(v) for v in p["search_lengths"]]:
        n = int(np.rint(L / p["res"]))
        if n < 1 or n + 1 > MAX_POSES or nmot * (n + 1) > TRAJ_CAP:
            raise ValueError(f"[HA*] search length {L} at resolution {p['res']} gives {n + 1} poses per motion "
                             f"primitive x {nmot} primitives; the device search holds at most {MAX_POSES} per "
                             f"primitive and {TRAJ_CAP} per expansion (include/htp.h HTP_HA_TRAJ_CAP)")


_CTX = None


def _context():
    global _CTX
    if _CTX is None:
        _CTX = _native.Context(0)
    return _CTX


def search_lowered(problems, ctx=None, cap_path=4096):
    """Run lowered problems on the GPU -> list of dicts (xs, ys, yaws, dirs, ks, counter, status, expanded)."""
    ctx = ctx or _context()
    for p in problems:
        check_limits(p)
    packed = _native.HastarPacked(problems, cap_path=cap_path)
    res = ctx.hastar(packed)
    if np.any(res.n_path > cap_path):
        return search_lowered(problems, ctx, cap_path=int(res.n_path.max()))
    out = []
    for b in range(len(problems)):
        xs, ys, yaws, dirs, ks = res.path(b)
        out.append(dict(xs=xs, ys=ys, yaws=yaws, dirs=dirs, ks=ks, counter=int(res.counter[b]),
                        status=int(res.status[b]), expanded=res.expansions(b), n_pose=int(res.n_pose[b])))
    return out


class HybridAStarSearch(object):
    STEER_COST = 1
    DELTA_STEER_COST = 5
    DEVIATION_COST = 1
    DISTANCE_COST = 1
    DIRECTION_CHANGE_COST = 1000
    REVERSE_COST = 5000
    HYBRID_COST = 50
    MIN_LENGTH_TO_GOAL = 1000

    def __init__(self, start_pose, goal_pose, config_environment, car_model, search_heuristic, motion_type="Pawn",
                 yaw_resolution=math.radians(10), plan_resolution=0.1):
        self.plan_resolution = plan_resolution
        self.yaw_resolution = yaw_resolution
        self.config_env = config_environment
        self.car_model = car_model
        self.search_heuristic = search_heuristic
        self.motion_type = motion_type
        self.motion_steers = motion_steers(car_model.MAX_STEER, yaw_resolution, motion_type)
        self.start_pose = list(start_pose)[:3]
        self.goal_pose = list(goal_pose)[:3]
        self.status = None
        self.expanded = []

    def calculate_node_index(self, x, y, yaw):
        return (round(x / self.plan_resolution), round(y / self.plan_resolution), round(yaw / self.yaw_resolution))

    def lower(self, max_nodes=2000):
        return lower_problem(self.start_pose, self.goal_pose, self.config_env, self.car_model,
                             self.search_heuristic, self.motion_type, self.yaw_resolution, self.plan_resolution,
                             max_nodes)

    def _report(self, r, dt):
        if r["status"] == STATUS_BLOCKED:
            print("start or goal position is interfere with obstacles!!")
            return
        if r["status"] == STATUS_MAX_NODES:
            print("drop the planner")
        elif r["status"] == STATUS_NO_PATH:
            print("No solution is available")
        elif r["status"] not in (STATUS_FOUND,):
            raise RuntimeError(f"[HA*] search failed: {_native.HA_STATUS.get(r['status'], r['status'])}")
        print("hybrid search time: ", dt)
        print("counter of nodes: ", r["counter"])

    def hybrid_a_star_search(self, plt=None, max_nodes=2000):
        t0 = time.time()
        r = search_lowered([self.lower(max_nodes)])[0]
        self.status, self.expanded = r["status"], r["expanded"]
        self._report(r, time.time() - t0)
        if r["status"] == STATUS_BLOCKED:
            return [], [], [], [], [], 0
        if plt is not None and len(r["xs"]):
            plt.plot(r["xs"], r["ys"], linewidth=0.3, color="g")
        return r["xs"], r["ys"], r["yaws"], r["dirs"], r["ks"], r["counter"]


def hybrid_a_star_search_batch(searches, max_nodes=2000, ctx=None):
    """Many HybridAStarSearch objects in one GPU launch -> list of
    (xs, ys, yaws, dirs, ks, counter) tuples, in order."""
    res = search_lowered([s.lower(max_nodes) for s in searches], ctx)
    out = []
    for s, r in zip(searches, res):
        s.status, s.expanded = r["status"], r["expanded"]
        if r["status"] not in (STATUS_FOUND, STATUS_NO_PATH, STATUS_MAX_NODES, STATUS_BLOCKED):
            raise RuntimeError(f"[HA*] search failed: {_native.HA_STATUS.get(r['status'], r['status'])}")
        out.append((r["xs"], r["ys"], r["yaws"], r["dirs"], r["ks"], r["counter"]))
    return out
