"""TEST-ONLY helpers for the hybrid A* parity tests: seeded headland search
scenarios built with the product's host shims (orchard environment, reference
line heuristic, car model) and lowered for the kernel, the oracle run on the
same lowered problem, and comparison of results."""
import math

import numpy as np

from headland_trajectory_planning_amd.path_planner import map_utils
from headland_trajectory_planning_amd.path_planner.car_model import CarModel
from headland_trajectory_planning_amd.path_planner.hybrid_a_star_search import lower_problem
from headland_trajectory_planning_amd.path_planner.orchard_geometry_environment import OrchardGeometryEnvironment
from headland_trajectory_planning_amd.path_planner.reference_line_heuristic import ReferenceLineHeuristic
from oracle import hastar as oha


def scenario(seed, n_obs=None, res=0.2, max_nodes=150, return_objects=False):
    """Start = LEAVE pose of row s (near side), goal = ENTER-like pose of row e
    pulled into the headland; a few point obstacles in the headland."""
    rng = np.random.default_rng(seed)
    np.random.seed(seed)
    row_w = rng.uniform(2.4, 3.2)
    rows = map_utils.create_tree_rows(8, row_w, 20.0, slope_angle=math.radians(rng.uniform(-10, 10)),
                                      l_std=[0.0, 0.5][seed % 2])
    s_row = int(rng.integers(0, 3))
    e_row = s_row + int(rng.integers(1, 4))
    n_obs = int(rng.integers(0, 4)) if n_obs is None else n_obs
    start = map_utils.get_base_pose(s_row, rows, rng.uniform(0.0, 1.5), pose_type=map_utils.LEAVE_POSE)
    goal = map_utils.get_base_pose(e_row, rows, rng.uniform(-1.5, -0.5), pose_type=map_utils.ENTER_POSE)
    goal[2] = goal[2] + rng.uniform(-0.3, 0.3)
    lo, hi = min(start[1], goal[1]), max(start[1], goal[1])
    obs = [[rng.uniform(rows[:, 0, 0].min() - 5.0, rows[:, 0, 0].min() - 1.0), rng.uniform(lo, hi)]
           for _ in range(n_obs)]
    env = OrchardGeometryEnvironment(rows, obs, tree_width=0.3, headland_width=6.0)
    car = CarModel(max_steer=0.55, axle_to_front=3.0, axle_to_back=0.55, width=1.48)
    wp = env.get_topology_waypoints(start, goal, drive_row_offset=4.5)
    heur = ReferenceLineHeuristic(wp, goal, car)
    prob = lower_problem(start, goal, env, car, heur, "King", math.radians(10), res, max_nodes)
    if return_objects:
        return prob, (env, car, heur, start, goal)
    return prob


def scenario_pawn(seed, max_nodes=60, res=0.2, n_obs=0):
    """Pawn (Dubins goal shots): the goal sits in the headland, headed along it,
    so forward Dubins turns can reach it."""
    from headland_trajectory_planning_amd.path_planner.hybrid_a_star_search import motion_steers
    rng = np.random.default_rng(500 + seed)
    np.random.seed(seed)
    row_w = rng.uniform(2.4, 3.2)
    rows = map_utils.create_tree_rows(8, row_w, 20.0, slope_angle=math.radians(rng.uniform(-5, 5)), l_std=0.0)
    s_row = int(rng.integers(0, 3))
    e_row = s_row + int(rng.integers(2, 4))
    start = map_utils.get_base_pose(s_row, rows, rng.uniform(0.5, 1.5), pose_type=map_utils.LEAVE_POSE)
    goal = map_utils.get_base_pose(e_row, rows, rng.uniform(3.5, 4.5), pose_type=map_utils.ENTER_POSE)
    goal[2] = math.pi / 2 + rng.uniform(-0.2, 0.2)
    obs = [[(start[0] + goal[0]) / 2 + rng.uniform(-1.5, 1.5), rng.uniform(start[1], goal[1])] for _ in range(n_obs)]
    env = OrchardGeometryEnvironment(rows, obs, tree_width=0.3, headland_width=rng.uniform(7.0, 9.0))
    car = CarModel(max_steer=0.55, axle_to_front=3.0, axle_to_back=0.55, width=1.48)
    wp = env.get_topology_waypoints(start, goal, drive_row_offset=4.5)
    heur = ReferenceLineHeuristic(wp, goal, car)
    return lower_problem(start, goal, env, car, heur, "Pawn", math.radians(10), res, max_nodes)


def oracle_problem(p):
    return oha.hastar_problem(p["start"], p["goal"], p["body"], p["blockers"], p["field"], p["lanes"],
                              p["search_lengths"], p["guide"], king=p["king"], res=p["res"], yaw_res=p["yaw_res"],
                              max_nodes=p["max_nodes"], wheel_base=p["wheel_base"], max_steer=p["max_steer"],
                              default_search_length=p["default_search_length"])


def run_oracle(p):
    return oha.HybridAStar(oracle_problem(p)).search()


def compare(o, r, exact=True, tol=1e-9):
    """Differences between an oracle result and a kernel result (dicts)."""
    bad = []
    for k in ("status", "counter"):
        if o[k] != r[k]:
            bad.append((k, o[k], r[k]))
    if [tuple(e) for e in o["expanded"]] != [tuple(e) for e in r["expanded"]]:
        bad.append(("expanded", len(o["expanded"]), len(r["expanded"])))
    for k in ("xs", "ys", "yaws", "dirs", "ks"):
        a, b = np.asarray(o[k], dtype=np.float64), np.asarray(r[k], dtype=np.float64)
        if a.shape != b.shape:
            bad.append((k, "len", a.shape, b.shape))
        elif exact and not np.array_equal(a, b):
            bad.append((k, float(np.max(np.abs(a - b)))))
        elif not exact and a.size and np.max(np.abs(a - b)) > tol:
            bad.append((k, float(np.max(np.abs(a - b)))))
    return bad
