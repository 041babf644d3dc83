"""TEST-ONLY helpers for the Y-park grid-search parity tests: seeded row-enter
scenarios lowered with the product's shim, the oracle on the same problem, and
comparison."""
import math

import numpy as np

from headland_trajectory_planning_amd.path_planner import map_utils
from headland_trajectory_planning_amd.path_planner.car_model import CarModel
from headland_trajectory_planning_amd.path_planner.headland_path_planning import (
    get_backward_steer_dir_for_y_type_parking, lower_ypark)
from headland_trajectory_planning_amd.path_planner.orchard_geometry_environment import OrchardGeometryEnvironment
from oracle import ypark as oyp


def scenario(seed, small=False):
    rng = np.random.default_rng(1000 + seed)
    np.random.seed(seed)
    row_w = rng.uniform(2.3, 3.2)
    rows = map_utils.create_tree_rows(8, row_w, 20.0, slope_angle=math.radians(rng.uniform(-10, 10)),
                                      l_std=[0.0, 0.5][seed % 2])
    s_row = int(rng.integers(0, 3))
    e_row = s_row + int(rng.integers(1, 4))
    start = map_utils.get_base_pose(s_row, rows, rng.uniform(-1.0, 1.0), pose_type=map_utils.LEAVE_POSE)
    end = map_utils.get_base_pose(e_row, rows, rng.uniform(0.0, 3.66), pose_type=map_utils.ENTER_POSE)
    env = OrchardGeometryEnvironment(rows, [], tree_width=0.3, headland_width=rng.uniform(4.5, 7.0))
    car = CarModel(max_steer=0.55, axle_to_front=3.0, axle_to_back=0.55, width=1.48)
    bdir = get_backward_steer_dir_for_y_type_parking(start, end)
    kw = dict(max_steer_backward=0.15, max_steer_forward=0.55, max_backward_distance=3.0 if not small else 2.0,
              max_forward_distance=2.0, min_forward_distance=1.0, min_backward_distance=1.0,
              min_steer_backward=0.0, min_steer_forward=0.5, step_size=0.2 if seed % 3 else 0.1)
    return lower_ypark(car, env, end, bdir, -bdir, **kw)


def oracle_problem(p):
    return dict(end_pose=p["end_pose"], bdir=p["backward_steer_dir"], fdir=p["forward_steer_dir"],
                wheel_base=p["wheel_base"], step=p["step"],
                axes=(list(p["backward_lengths"]), list(p["forward_lengths"]), list(p["backward_steers"]),
                      list(p["forward_steers"])),
                body=p["body"], blockers=p["blockers"], field=p["field"])


def run_oracle(p):
    return oyp.search(oracle_problem(p))


def compare(o, r, tol=1e-12):
    bad = []
    for k in ("status", "cand"):
        if o[k] != r[k]:
            bad.append((k, o[k], r[k]))
    if not np.allclose(o["params"], r["params"], rtol=0, atol=0):
        bad.append(("params", o["params"], r["params"]))
    a, b = np.asarray(o["path"]), np.asarray(r["path"])
    if a.shape != b.shape:
        bad.append(("path shape", a.shape, b.shape))
    elif a.size and np.max(np.abs(a - b)) > tol:
        bad.append(("path", float(np.max(np.abs(a - b)))))
    return bad
