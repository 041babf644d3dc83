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
