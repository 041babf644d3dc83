"""Row-exit / row-enter offsets and Dubins forward turns of
R/path_planner/safety_forward_path_plan.py (host side; the footprint checks
are the reference's env.check_path_feasibility)."""
import math

import numpy as np

from ..obca_py.util import calc_spline_course
from . import dubins
from .map_utils import ENTER_POSE, FAR_SIDE, LEAVE_POSE, NEAR_SIDE, get_base_pose  # noqa: F401
from .navigation_utils import get_dubins_path


def get_dubins_turn_dirs(start_pose, end_pose, turning_radius):
    """:25-34."""
    configs, _ = dubins.shortest_path(start_pose, end_pose, turning_radius).sample_many(0.1)
    start_turn_dir = -1 if configs[0][2] > start_pose[2] else 1
    end_turn_dir = -1 if configs[-1][2] > end_pose[2] else 1
    return start_turn_dir, end_turn_dir


def get_steer_dir_for_enter_calculation(start_pose, end_pose):
    """:37-45."""
    if end_pose[1] - start_pose[1] > 0:
        return np.sign(1 * math.cos(start_pose[2]))
    return np.sign(-1 * math.cos(start_pose[2]))


def get_offset_pose(init_pose, pose_type, turn_out_dir, car, config_env, steer_angle=0.55,
                    delta_yaw=math.radians(45), max_offset=5, accuracy=0.1):
    """:248-283: first offset (0, 0.1, ...) whose 45-degree turn-out arc is collision free."""
    init_x, init_y, init_yaw = init_pose[0], init_pose[1], init_pose[2]
    motion_dir = -1 if pose_type == ENTER_POSE else 1
    offset_dir = -1 if pose_type == ENTER_POSE else 1
    for dist in np.arange(0, max_offset + accuracy, accuracy):
        x = init_x + dist * np.cos(init_yaw) * offset_dir
        y = init_y + dist * np.sin(init_yaw) * offset_dir
        pose = np.array([x, y, init_yaw])
        path = car.calculate_motion_path(pose, [steer_angle * turn_out_dir, motion_dir], delta_yaw, accuracy)
        if config_env.check_path_feasibility(car, path, boundary_check=False):
            break
    if dist >= max_offset:
        print("no solution is available!! dist: %.2f, x: %.2f" % (dist, x))
    return dist, pose, path


def get_offset_poses_for_row_traversing(start_leave_pose_base, end_enter_pose_base, car, config_env,
                                        max_steer_angle=0.55, plt=None):
    """:48-84."""
    turn_dir = get_steer_dir_for_enter_calculation(start_leave_pose_base, end_enter_pose_base)
    leave_dist, start_off, leave_path = get_offset_pose(start_leave_pose_base, LEAVE_POSE, turn_dir, car, config_env,
                                                        steer_angle=max_steer_angle)
    print("backward distance for leaving is %.2f" % (leave_dist))
    enter_dist, end_off, enter_path = get_offset_pose(end_enter_pose_base, ENTER_POSE, turn_dir, car, config_env,
                                                      steer_angle=max_steer_angle)
    print("backward distance for entering is %.2f" % (enter_dist))
    if plt is not None:
        plt.plot(leave_path[:, 0], leave_path[:, 1])
        plt.plot(enter_path[:, 0], enter_path[:, 1])
    return start_off, end_off


def get_dubins_path_full(pose_start, pose_end, turning_radius, step_size=0.1):
    """:286-297 (re-splined at the default ds = 0.1, as the reference does)."""
    cfg = get_dubins_path(pose_start, pose_end, turning_radius, step_size=step_size)
    rx, ry, ryaw, rk, _ = calc_spline_course(cfg[:, 0], cfg[:, 1])
    return np.vstack([rx, ry, ryaw, rk, np.ones_like(rx)]).T


# ---------------------------------------------------------------- classic turns
# Reeds-Shepp words come from the HIP drop-in (libhtp.so htp_rs_all_paths_batch);
# there is no host fallback.  Tests may swap `rs_curves` for the CPU restatement.
from .. import reeds_shepp as rs_curves  # noqa: E402
from .geom import polyline_buffer_intersects, ring_of  # noqa: E402


def filter_consecutive_duplicate(array):
    """:19-22 (element 0 is compared with the last one, as in the reference)."""
    return np.array([elem for i, elem in enumerate(array) if (elem - array[i - 1]).any()])


def get_car_outmost_pose(tree_rows, row_id, base_yaw, car, side=NEAR_SIDE, pose_type=ENTER_POSE):
    """:87-129: the pose whose footprint (body + implements on the near side) just clears the row ends."""
    lower, upper = tree_rows[row_id, :, :], tree_rows[row_id + 1, :, :]
    if side == NEAR_SIDE:
        lo_end, up_end = lower[0, :], upper[0, :]
        outmost_x = min(lo_end[0], up_end[0])
        min_x, max_x = car.car_poly.bounds[0], car.car_poly.bounds[2]
        for aux in car.aux_polys:
            min_x = min(min_x, aux.bounds[0])
            max_x = max(max_x, aux.bounds[2])
        off = abs(min_x) if pose_type == LEAVE_POSE else abs(max_x)
        return np.array([outmost_x - off, (lo_end[1] + up_end[1]) / 2, base_yaw])
    lo_end, up_end = lower[1, :], upper[1, :]
    outmost_x = max(lo_end[0], up_end[0])
    off = car.AXLE_TO_BACK if pose_type == LEAVE_POSE else car.AXLE_TO_FRONT
    return np.array([outmost_x + off, (lo_end[1] + up_end[1]) / 2, base_yaw])


def get_start_end_pose_for_dubins(map_tree_rows, start_row_id, end_row_id, car, config_env, max_steer_angle=0.55,
                                  plt=None, side=NEAR_SIDE, extra_offset_enter_dist=0.0, extra_offset_leave_dist=0.0):
    """:132-198: offset poses whose 45-degree turn-out arcs clear the rows, re-run until the
    Dubins word's first/last turn directions agree with the arcs' directions."""
    start_base = get_base_pose(start_row_id, map_tree_rows, extra_offset_leave_dist, side=side, pose_type=LEAVE_POSE)
    end_base = get_base_pose(end_row_id, map_tree_rows, extra_offset_enter_dist, side=side, pose_type=ENTER_POSE)
    turn_dir = get_steer_dir_for_enter_calculation(start_base, end_base)
    leave_dir = enter_dir = turn_dir
    while True:
        leave_offset, start_off, leave_path = get_offset_pose(start_base, LEAVE_POSE, leave_dir, car, config_env,
                                                              steer_angle=max_steer_angle)
        enter_offset, end_off, enter_path = get_offset_pose(end_base, ENTER_POSE, enter_dir, car, config_env,
                                                            steer_angle=max_steer_angle)
        s_dir, e_dir = get_dubins_turn_dirs(start_off, end_off, 1.0 / car.curvature)
        if s_dir == leave_dir and e_dir == enter_dir:
            break
        leave_dir, enter_dir = s_dir, e_dir
    if plt is not None:
        plt.plot(leave_path[:, 0], leave_path[:, 1])
        plt.plot(enter_path[:, 0], enter_path[:, 1])
    return start_off, end_off, leave_offset, enter_offset


def get_start_end_pose_for_reeds_shepp(map_tree_rows, start_row_id, end_row_id, car, config_env,
                                       max_steer_angle=0.55, plt=None, side=NEAR_SIDE, extra_offset_enter_dist=0.0,
                                       extra_offset_leave_dist=0.0):
    """:300-364: both offset poses moved to one outmost x.  As in the reference, that x is taken
    from the start BASE pose and the end OFFSET pose."""
    start_base = get_base_pose(start_row_id, map_tree_rows, extra_offset_leave_dist, side=side, pose_type=LEAVE_POSE)
    end_base = get_base_pose(end_row_id, map_tree_rows, extra_offset_enter_dist, side=side, pose_type=ENTER_POSE)
    turn_dir = get_steer_dir_for_enter_calculation(start_base, end_base)
    _, start_off, leave_path = get_offset_pose(start_base, LEAVE_POSE, turn_dir, car, config_env,
                                               steer_angle=max_steer_angle)
    _, end_off, enter_path = get_offset_pose(end_base, ENTER_POSE, turn_dir, car, config_env,
                                             steer_angle=max_steer_angle)
    if side == NEAR_SIDE:
        outmost_x = np.min([start_base[0], end_off[0]])
    else:
        outmost_x = np.max([start_base[0], end_off[0]])
    start_off[0] = outmost_x
    end_off[0] = outmost_x
    leave_offset = abs(outmost_x - start_base[0])
    enter_offset = abs(outmost_x - end_base[0])
    if plt is not None:
        plt.plot(leave_path[:, 0], leave_path[:, 1])
        plt.plot(enter_path[:, 0], enter_path[:, 1])
    return start_off, end_off, leave_offset, enter_offset


def _rs_rows(p):
    return np.array([p.x, p.y, p.yaw, p.cs, p.directions], dtype=np.float64).T


def get_all_reeds_shepp_paths_full(pose_start, pose_end, turning_radius, step_size=0.1):
    """:367-392: every Reeds-Shepp word as rows [x, y, yaw, curvature, direction]."""
    paths = rs_curves.calc_all_paths(pose_start[0], pose_start[1], pose_start[2], pose_end[0], pose_end[1],
                                     pose_end[2], 1.0 / turning_radius, step_size)
    return [_rs_rows(p) for p in paths]


def get_circle_back_path_full(pose_start, pose_end, turning_radius, car, side=NEAR_SIDE, step_size=0.1):
    """:395-454: forward arc (radius Rf, angle theta), backward arc (Rb, pi - theta), Dubins lead-in;
    both radii grow by 5 % until the backward arc stays clear of the end pose's x.  Rows wider
    than 2R fall back to the plain Dubins turn."""
    w = abs(pose_start[1] - pose_end[1])
    turning_radius = max(turning_radius, 1.0 / car.curvature)
    if w >= turning_radius * 2:
        return get_dubins_path_full(pose_start, pose_end, turning_radius, step_size)
    Rf = Rb = turning_radius
    while True:
        theta = np.pi / 2 + np.arcsin((Rb + w - Rf) / (Rf + Rb))
        if side == NEAR_SIDE and pose_start[0] - (Rf + Rb) * np.cos(theta - np.pi / 2) < pose_end[0] - step_size:
            break
        if side == FAR_SIDE and pose_start[0] + (Rf + Rb) * np.cos(theta - np.pi / 2) > pose_end[0] + step_size:
            break
        Rf *= 1.05
        Rb *= 1.05
    turn_dir = get_steer_dir_for_enter_calculation(pose_start, pose_end)
    forward = car.calculate_motion_path_new(init_pose=pose_start, motion_dir=1, steer_dir=turn_dir,
                                            turning_radius=Rf, delta_yaw=theta, step_size=step_size)
    back = car.calculate_motion_path_new(init_pose=forward[-1, :3], motion_dir=-1, steer_dir=-turn_dir,
                                         turning_radius=Rb, delta_yaw=np.pi - theta, step_size=step_size)
    straight = get_dubins_path_full(back[-1, :3], pose_end, turning_radius, step_size)
    return np.vstack([forward, back, straight])


def classic_circle_back_turning_path(start_exit_pose, end_enter_pose, map_env, car_model, step_size=0.1, plt=None):
    """:793-882: the Reeds-Shepp word with the least backward length among those whose 0.3 m
    flat-capped corridor misses every row/obstacle polygon, then shifted along the exit heading
    until the footprints clear the rows (boundary_check=False), with Dubins lead-in/out when moved.

    Reference behaviour kept: the shift loop tests the path BEFORE moving it, so the returned path
    sits one step past the first feasible one; with no clear word it raises IndexError
    (`feasible_paths[0]` on an empty list)."""
    to_goal = rs_curves.calc_all_paths(start_exit_pose[0], start_exit_pose[1], start_exit_pose[2],
                                       end_enter_pose[0], end_enter_pose[1], end_enter_pose[2],
                                       car_model.curvature, step_size)
    rings = [ring_of(p) for p in map_env.obs_poly_list]
    feasible = []
    for p in to_goal:
        xy = np.array([p.x, p.y], dtype=np.float64).T
        if not any(polyline_buffer_intersects(xy, 0.3, Q) for Q in rings):
            feasible.append(p)
    if len(feasible) == 0:
        raise IndexError("list index out of range")
    optimal, best = None, 99999
    for p in feasible:
        lengths = np.array(p.lengths)
        cost = np.abs(lengths[lengths < 0].sum())
        if cost < best:
            optimal, best = p, cost
    turning_path = _rs_rows(optimal)
    ok = map_env.check_path_feasibility(car_model, turning_path[:, :3], boundary_check=False)
    offset = 0
    shift = np.array([[step_size * np.cos(start_exit_pose[2]), step_size * np.sin(start_exit_pose[2])]])
    while not ok:
        ok = map_env.check_path_feasibility(car_model, turning_path[:, :3], boundary_check=False)
        if plt is not None:
            plt.plot(turning_path[:, 0], turning_path[:, 1], "--", c="black", alpha=0.5)
        offset += step_size
        turning_path[:, :2] += shift
    if offset > step_size:
        radius = 1.0 / car_model.curvature
        leave = get_dubins_path_full(start_exit_pose, turning_path[0, :3], radius)
        turning_path = np.vstack([leave[:-1], turning_path])
        enter = get_dubins_path_full(turning_path[-1, :3], end_enter_pose, radius)
        turning_path = np.vstack([turning_path, enter])
    return turning_path
