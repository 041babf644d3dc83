"""TEST-ONLY: the data flow of R/test/classic_planner.ipynb (cells 3-15) rebuilt on the
product's drop-in modules, with the notebook's printed values as pins.
`rs` swaps the Reeds-Shepp module (CPU tests pass the oracle restatement)."""
import contextlib
import io
import math

import numpy as np

from headland_trajectory_planning_amd.obca_py.util import get_init_ref_path
from headland_trajectory_planning_amd.path_planner import map_utils
from headland_trajectory_planning_amd.path_planner import safety_forward_path_plan as sfp
from headland_trajectory_planning_amd.path_planner.car_model import CarModel
from headland_trajectory_planning_amd.path_planner.OGE_OBCA import orchard_environment_OBCA

# R/test/classic_planner.ipynb outputs (cells 11-12)
PIN_START_EXIT = np.array([0.38166505, 3.75, 3.14159265])
PIN_SAFE_START = np.array([-1.30805046, 3.75, 3.14159265])
PIN_WORD = ["R", "L", "R"]
PIN_REF0 = np.array([0.38166505, 3.75, 0.0, -3.14159265, 0.0])


@contextlib.contextmanager
def rs_module(rs):
    saved = sfp.rs_curves
    if rs is not None:
        sfp.rs_curves = rs
    try:
        yield
    finally:
        sfp.rs_curves = saved


def run(rs=None, with_circle_back=True):
    out = io.StringIO()
    res = {}
    with rs_module(rs), contextlib.redirect_stdout(out):
        np.random.seed(1)
        tree_rows = map_utils.create_tree_rows(8, 2.5, 20, slope_angle=math.radians(10), l_std=1.0)
        env = orchard_environment_OBCA(tree_rows, [], tree_width=0.3, headland_width=6.0)
        car_op = CarModel(max_steer=0.55, axle_to_back=0.55, width=1.48,
                          aux_poly_features=[[[-1.84, 0.5], 1.0, 1.1]], with_aux=True)
        empty = CarModel(max_steer=0.55, axle_to_back=0.55, width=1.48, with_aux=False)
        side = map_utils.NEAR_SIDE
        start = map_utils.get_base_pose(1, tree_rows, -0.0, side=side, pose_type=map_utils.LEAVE_POSE)
        end = map_utils.get_base_pose(3, tree_rows, 0, side=side, pose_type=map_utils.ENTER_POSE)
        # cell 8: Dubins warm start
        ds_start, ds_end, d_leave, d_enter = sfp.get_start_end_pose_for_dubins(tree_rows, 1, 3, car_op, env,
                                                                               max_steer_angle=0.55, side=side)
        # cells 10-11: Reeds-Shepp warm start
        safe_start, safe_end, leave_offset, enter_offset = sfp.get_start_end_pose_for_reeds_shepp(
            tree_rows, 1, 3, car_op, env, max_steer_angle=0.55, side=side)
        paths = sfp.rs_curves.calc_all_paths(safe_start[0], safe_start[1], safe_start[2], safe_end[0], safe_end[1],
                                             safe_end[2], car_op.curvature, 0.1)
        feasible, optimal, best = [], None, 99999
        for p in paths:
            traj = np.array([p.x, p.y, p.yaw]).T
            if env.check_path_feasibility(empty, traj, boundary_check=False):
                print("path type: ", p.ctypes)
                feasible.append(list(p.ctypes))
                lengths = np.array(p.lengths)
                cost = np.abs(lengths[lengths < 0].sum())
                if cost < best:
                    optimal, best = p, cost
        path = np.array([optimal.x, optimal.y, optimal.yaw, optimal.cs, optimal.directions]).T
        print("start_exit_pose: ", start)
        print("safe_start_pose: ", safe_start)
        if leave_offset > 0.1:
            leave = sfp.get_dubins_path_full(start, safe_start, 1.0 / car_op.curvature)
            path = np.vstack([leave[:-1], path])
        if enter_offset > 0.1:
            enter = sfp.get_dubins_path_full(safe_end, end, 1.0 / car_op.curvature)
            path = np.vstack([path, enter[1:]])
        # cell 12: init guess
        ref = get_init_ref_path(empty, path[:, 0], path[:, 1], path[:, 2], path[:, 3], path[:, 4],
                                desired_v=0.5, ds=0.5 * 0.2)
        res.update(env=env, empty=empty, car_op=car_op, start=start, end=end, tree_rows=tree_rows,
                   dubins=(ds_start, ds_end, d_leave, d_enter), safe=(safe_start, safe_end, leave_offset, enter_offset),
                   n_paths=len(paths), feasible=feasible, word=list(optimal.ctypes), path=path, ref=ref)
        # cell 15: classic circle-back turn
        if with_circle_back:
            res["circle_back"] = sfp.classic_circle_back_turning_path(start, end, env, empty, step_size=0.3)
    res["prints"] = out.getvalue()
    return res
