"""Headland turn planners of R/path_planner/headland_path_planning.py:
forward Dubins turn if feasible, else a Y-type parking manoeuvre found by the
lexicographic parameter grid search (:382-451) plus a hybrid A* drive to its
first pose (searched on the GPU through hybrid_a_star_search)."""
import copy
import math

import numpy as np

from .. import _native
from ..obca_py.util import calc_spline_course
from . import transformation as trans
from .geom import angle_wrap, ring_of
from .hybrid_a_star_search import HybridAStarSearch
from .navigation_utils import convert_2d_xys_to_target_frame
from .reference_line_heuristic import ReferenceLineHeuristic
from .safety_forward_path_plan import get_dubins_path_full, get_offset_poses_for_row_traversing

ERROR_CODE_FOR_NONE = -1
ERROR_CODE_FOR_Y_PARKING = 0
ERROR_CODE_FOR_HYBRID_A_STAR = 1


def headland_planner_y_type_park_combined(config_env, car_model, start_pose, end_pose, motion_type="Pawn",
                                          drive_row_offset=4.5, max_steer_backward=0.35, min_steer_backward=0.22,
                                          max_steer_forward=0.55, min_steer_forward=0.50, max_backward_distance=2.0,
                                          min_forward_distance=1.4, max_forward_distance=2.5,
                                          min_backward_distance=0.7, step_size=0.1, tree_width_in_forward_plan=0.2,
                                          max_steer_for_offset_plan=0.5):
    """:55-121."""
    env_plan = copy.deepcopy(config_env)
    env_plan.update_tree_width(tree_width_in_forward_plan)
    start_exit, end_enter = get_offset_poses_for_row_traversing(start_pose, end_pose, car_model, env_plan,
                                                                max_steer_angle=max_steer_for_offset_plan)
    path = get_dubins_path_full(start_exit, end_enter, car_model.get_turn_radius(max_steer_angle=None),
                                step_size=step_size)
    if env_plan.check_path_feasibility(car_model, path, boundary_check=True):
        print("got a path forward driving")
        return ERROR_CODE_FOR_NONE, path[:, 0], path[:, 1], path[:, 2], path[:, 3], path[:, 4]
    return headland_planner_y_type_park(
        config_env=config_env, car_model=car_model, start_pose=start_pose, end_pose=end_pose,
        motion_type=motion_type, drive_row_offset=drive_row_offset, max_steer_backward=max_steer_backward,
        min_steer_backward=min_steer_backward, max_steer_forward=max_steer_forward,
        min_steer_forward=min_steer_forward, max_backward_distance=max_backward_distance,
        min_forward_distance=min_forward_distance, max_forward_distance=max_forward_distance,
        min_backward_distance=min_backward_distance, step_size=step_size, debug=False)


def headland_planner_y_type_park(config_env, car_model, start_pose, end_pose, motion_type="Pawn",
                                 drive_row_offset=4.5, max_steer_backward=0.35, min_steer_backward=0.22,
                                 max_steer_forward=0.55, min_steer_forward=0.50, max_backward_distance=2.0,
                                 min_forward_distance=1.4, max_forward_distance=2.5, min_backward_distance=0.7,
                                 step_size=0.1, debug=True):
    """:124-255."""
    error_code = ERROR_CODE_FOR_NONE
    backward_steer_dir = get_backward_steer_dir_for_y_type_parking(start_pose, end_pose)
    forward_steer_dir = -backward_steer_dir
    print("start Y park searching")
    res = search_y_type_parking_path(car_model, config_env, end_pose, backward_steer_dir, forward_steer_dir,
                                     max_steer_backward, max_steer_forward, max_backward_distance,
                                     max_forward_distance, min_forward_distance, min_backward_distance,
                                     min_steer_backward, min_steer_forward, step_size=step_size, debug=debug)
    y_path, parameters = res if debug else (res, [])
    if len(y_path) == 0:
        error_code = ERROR_CODE_FOR_Y_PARKING
        print("No enough space on headland for the tractor to enter the row!!")
        return (error_code, parameters, 0, [], [], [], [], []) if debug else (error_code, [], [], [], [], [])
    intermediate_pose = y_path[0][:3]
    way_points = config_env.get_topology_waypoints(start_pose, intermediate_pose, drive_row_offset=drive_row_offset)
    heuristic = ReferenceLineHeuristic(way_points, intermediate_pose, car_model)
    planner = HybridAStarSearch(start_pose, intermediate_pose, config_env, car_model, heuristic,
                                motion_type=motion_type, plan_resolution=step_size)
    xs, ys, yaws, dirs, ks, count = planner.hybrid_a_star_search(max_nodes=400)
    if len(xs) == 0:
        print("cannot search a path to parking start pose!!")
        error_code = ERROR_CODE_FOR_HYBRID_A_STAR
        return (error_code, parameters, count, [], [], [], [], []) if debug else (error_code, [], [], [], [], [])
    path_xs = np.concatenate([xs, y_path[:, 0]])
    path_ys = np.concatenate([ys, y_path[:, 1]])
    path_yaws = np.concatenate([yaws, y_path[:, 2]])
    path_ks = np.concatenate([ks, y_path[:, 3]])
    dirs = np.concatenate([dirs, y_path[:, 4]])
    if debug:
        return error_code, parameters, count, path_xs, path_ys, path_yaws, path_ks, dirs
    return error_code, path_xs, path_ys, path_yaws, path_ks, dirs


def get_backward_steer_dir_for_y_type_parking(start_pose, end_pose):
    """:370-378."""
    if end_pose[1] - start_pose[1] > 0:
        return np.sign(1 * math.cos(start_pose[2]))
    return np.sign(-1 * math.cos(start_pose[2]))


def y_park_grid(max_steer_backward, max_steer_forward, max_backward_distance, max_forward_distance,
                min_forward_distance, min_backward_distance, min_steer_backward, min_steer_forward):
    """The four parameter axes of :404-414 in their loop order."""
    sb = list(np.arange(min_steer_backward, max_steer_backward + 0.1, 0.1))
    if np.max(sb) < max_steer_backward:
        sb.append(max_steer_backward)
    sf = list(np.arange(min_steer_forward, max_steer_forward + 0.1, 0.1))
    if np.max(sf) < max_steer_forward:
        sf.append(max_steer_forward)
    bl = list(np.arange(max_backward_distance, min_backward_distance, -0.1))
    fl = list(np.arange(max_forward_distance, min_forward_distance, -0.1))
    return bl, fl, sb, sf


def lower_ypark(car_model, config_env, end_pose, backward_steer_dir, forward_steer_dir, max_steer_backward=0.4,
                max_steer_forward=0.45, max_backward_distance=3.5, max_forward_distance=2.0,
                min_forward_distance=1.4, min_backward_distance=0.7, min_steer_backward=0.3,
                min_steer_forward=0.3, step_size=0.1):
    """Flat description of one search_y_type_parking_path call (input of _native.YparkPacked)."""
    bl, fl, sb, sf = y_park_grid(max_steer_backward, max_steer_forward, max_backward_distance, max_forward_distance,
                                 min_forward_distance, min_backward_distance, min_steer_backward, min_steer_forward)
    T = trans.states2SE3([end_pose[0], end_pose[1], 0, 0, 0, end_pose[2]])
    return dict(end_pose=np.asarray(end_pose, dtype=np.float64)[:3], backward_steer_dir=float(backward_steer_dir),
                forward_steer_dir=float(forward_steer_dir), wheel_base=float(car_model.WHEEL_BASE),
                step=float(step_size), T=T, yaw_odom=float(trans.SE32states(T)[-1]),
                backward_lengths=np.asarray(bl, dtype=np.float64), forward_lengths=np.asarray(fl, dtype=np.float64),
                backward_steers=np.asarray(sb, dtype=np.float64), forward_steers=np.asarray(sf, dtype=np.float64),
                body=ring_of(car_model.car_poly), blockers=[ring_of(q) for q in config_env.obs_poly_list],
                field=ring_of(config_env.field_range_poly))


_CTX = None


def search_y_lowered(problems, ctx=None):
    """Run lowered Y-park searches on the GPU -> list of dicts (status, params, path)."""
    global _CTX
    if ctx is None:
        if _CTX is None:
            _CTX = _native.Context(0)
        ctx = _CTX
    res = ctx.ypark(_native.YparkPacked(problems))
    out = []
    for b in range(len(problems)):
        n = int(res.n_path[b])
        out.append(dict(status=int(res.status[b]), cand=int(res.cand[b]), params=res.params[b].tolist(),
                        path=res.path[b, :n].copy(), n_pose=int(res.n_pose[b])))
    return out


def _report_ypark(r, debug):
    if r["status"] == _native.YP_STATUS_BY_NAME["end_blocked"]:
        print(" [Y-type Planner] The end pose is interfered with the environment!")
        return [], []
    if r["status"] == _native.YP_STATUS_BY_NAME["bad_input"]:
        raise ValueError("[Y-type Planner] grid outside the kernel's limits (<= 63 poses per arc)")
    if r["status"] != _native.YP_STATUS_BY_NAME["found"]:
        return ([], []) if debug else []
    bl, fl, sb, sf = r["params"]
    print("backward distance:%.2f, forward distance:%.2f, backward steer:%.2f, forward steer:%.2f,  "
          % (bl, fl, sb, sf))
    return (r["path"], [bl, fl, sb, sf]) if debug else r["path"]


def search_y_type_parking_path(car_model, config_env, end_pose, backward_steer_dir, forward_steer_dir,
                               max_steer_backward=0.4, max_steer_forward=0.45, max_backward_distance=3.5,
                               max_forward_distance=2.0, min_forward_distance=1.4, min_backward_distance=0.7,
                               min_steer_backward=0.3, min_steer_forward=0.3, step_size=0.1, debug=False):
    """:382-451: first feasible (backward length, forward length, backward steer,
    forward steer) in lexicographic loop order, searched on the GPU
    (htp_ypark_search_batch)."""
    prob = lower_ypark(car_model, config_env, end_pose, backward_steer_dir, forward_steer_dir, max_steer_backward,
                       max_steer_forward, max_backward_distance, max_forward_distance, min_forward_distance,
                       min_backward_distance, min_steer_backward, min_steer_forward, step_size)
    # an interfering end pose gives ([], []) regardless of debug, like the reference (:400-402)
    return _report_ypark(search_y_lowered([prob])[0], debug)


def search_y_type_parking_path_batch(searches, ctx=None):
    """Many searches in one launch: `searches` are keyword dicts of
    search_y_type_parking_path's arguments; returns [(path, [bl, fl, sb, sf])]
    with ([], []) where none is feasible."""
    probs = [lower_ypark(**{k: v for k, v in s.items() if k != "debug"}) for s in searches]
    out = []
    for r in search_y_lowered(probs, ctx):
        ok = r["status"] == _native.YP_STATUS_BY_NAME["found"]
        out.append((r["path"], list(r["params"])) if ok else ([], []))
    return out


def calculate_motion_path(init_pose, motion_command, search_length, wheel_base, step):
    """:455-484."""
    steer_angle, speed_direction = motion_command[0], motion_command[1]
    num_steps = round(search_length / step)
    yaw_step = speed_direction * step / wheel_base * math.tan(steer_angle)
    init_yaw = angle_wrap(init_pose[-1] + yaw_step)
    yaws = angle_wrap(np.linspace(init_yaw, init_yaw + yaw_step * (num_steps), num_steps + 1))
    xs = init_pose[0] + np.cumsum(step * np.cos(yaws[:-1]) * speed_direction)
    ys = init_pose[1] + np.cumsum(step * np.sin(yaws[:-1]) * speed_direction)
    path = np.vstack([init_pose, np.vstack([xs, ys, yaws[1:]]).T])
    curvature = 0
    if abs(motion_command[0]) > 0.00001:
        curvature = math.tan(motion_command[0]) / wheel_base
    ks = np.ones((len(path), 1)) * curvature
    dirs = np.ones((len(path), 1)) * motion_command[1]
    return np.hstack((path, ks, dirs))


def get_y_type_parking_path(car_model, backward_length, backward_steer, forward_length, forward_steer, step):
    """:487-516: backward arc then forward arc from the row-entry pose, both reversed."""
    back = calculate_motion_path([0, 0, 0], [backward_steer, -1], backward_length, car_model.WHEEL_BASE, step)
    fwd = calculate_motion_path(back[-1, :3], [forward_steer, 1], forward_length, car_model.WHEEL_BASE, step)
    back[:, -1] = 1
    back = back[::-1]
    fwd[:, -1] = -1
    fwd = fwd[::-1]
    return np.vstack([fwd, back])


def get_path_in_odom(odom_T_baselink, path, plt=None):
    """:519-527."""
    pose = trans.SE32states(odom_T_baselink)
    out = np.copy(path)
    out[:, 2] += pose[-1]
    out[:, 0], out[:, 1] = convert_2d_xys_to_target_frame(out[:, 0], out[:, 1], odom_T_baselink)
    return out


def get_y_type_parking_path_in_odom(car, start_pose, end_pose, backward_distance=5.0, forward_distance=2.5,
                                    backward_steer=0.1, forward_steer=0.5, step_size=0.1):
    """:258-281."""
    bdir = get_backward_steer_dir_for_y_type_parking(start_pose, end_pose)
    p = get_y_type_parking_path(car, backward_distance, backward_steer * bdir, forward_distance,
                                forward_steer * -bdir, step_size)
    return get_path_in_odom(trans.states2SE3([end_pose[0], end_pose[1], 0, 0, 0, end_pose[2]]), p)


def get_row_enter_path(config_env, car_model, start_pose, end_pose, drive_row_offset=4.5, steer_backward=0.35,
                       steer_forward=0.55, backward_distance=2.0, forward_distance=2.5, step_size=0.1):
    """:284-367 (motion_type "Pawn" in the reference: raises NotImplementedError until Dubins shots land)."""
    error_code = ERROR_CODE_FOR_NONE
    y_path = get_y_type_parking_path_in_odom(car_model, start_pose, end_pose, backward_distance, forward_distance,
                                             steer_backward, steer_forward, step_size)
    if not config_env.check_path_feasibility(car_model, y_path):
        print("not enough space for row entering")
        error_code = ERROR_CODE_FOR_Y_PARKING
    intermediate_pose = y_path[0][:3]
    way_points = config_env.get_topology_waypoints(start_pose, intermediate_pose, drive_row_offset=drive_row_offset)
    heuristic = ReferenceLineHeuristic(way_points, intermediate_pose, car_model)
    planner = HybridAStarSearch(start_pose, intermediate_pose, config_env, car_model, heuristic, motion_type="Pawn",
                                plan_resolution=step_size)
    xs, ys, yaws, dirs, _, count = planner.hybrid_a_star_search(max_nodes=400)
    if len(xs) == 0:
        print("cannot search a path to parking start pose!!")
        return (ERROR_CODE_FOR_HYBRID_A_STAR, count, y_path[:, 0], y_path[:, 1], y_path[:, 2], y_path[:, 3],
                y_path[:, 4])
    xs, ys, yaws, ks, _ = calc_spline_course(xs, ys, ds=step_size)
    dirs = np.ones_like(xs)
    return (error_code, count, np.concatenate([xs, y_path[:, 0]]), np.concatenate([ys, y_path[:, 1]]),
            np.concatenate([yaws, y_path[:, 2]]), np.concatenate([ks, y_path[:, 3]]),
            np.concatenate([dirs, y_path[:, 4]]))
