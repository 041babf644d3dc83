"""Warm starts of R/path_planner/OBCA_warm_start.py:11-174."""
import numpy as np

from .headland_path_planning import (get_backward_steer_dir_for_y_type_parking, get_path_in_odom,  # noqa: F401
                                     get_y_type_parking_path, get_y_type_parking_path_in_odom)
from .safety_forward_path_plan import get_dubins_path_full


def get_warm_start_path_y_type(car, start_pose, end_pose, steer_backward, forward_distance, backward_distance,
                               steer_forward, step_size):
    """:124-163: Dubins lead-in to the Y-park's first pose, then the Y-park."""
    y = get_y_type_parking_path_in_odom(car, start_pose, end_pose, backward_distance=backward_distance,
                                        forward_distance=forward_distance, backward_steer=steer_backward,
                                        forward_steer=steer_forward, step_size=step_size)
    lead = get_dubins_path_full(start_pose, y[0][:3], turning_radius=1.0 / car.curvature, step_size=step_size)
    path = np.vstack([lead, y])
    return path[:, 0], path[:, 1], path[:, 2], path[:, 3], path[:, 4]


def get_warm_start_path_dubins(car, start_pose, end_pose, step_size):
    """:166-174."""
    path = get_dubins_path_full(start_pose, end_pose, turning_radius=1.0 / car.curvature, step_size=step_size)
    return path[:, 0], path[:, 1], path[:, 2], path[:, 3], path[:, 4]
