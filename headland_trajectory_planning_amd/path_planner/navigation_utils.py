"""Helpers of R/path_planner/utils/navigation_utils.py used by the warm starts."""
import math

import numpy as np

from . import dubins, transformation


def angle_wrap(angles):
    return (angles + math.pi) % (2 * math.pi) - math.pi


def convert_2d_xys_to_target_frame(xs_source, ys_source, target_T_source):
    """navigation_utils.py:196-203."""
    pts = np.vstack((xs_source, ys_source, np.zeros_like(ys_source))).T
    homo = transformation.xyz2homo(pts).T
    p2 = target_T_source.dot(homo)[:2, :].T
    return p2[:, 0], p2[:, 1]


def get_dubins_path(pose_start, pose_end, turning_radius, step_size):
    """navigation_utils.py:206-215."""
    q0 = (pose_start[0], pose_start[1], pose_start[2])
    q1 = (pose_end[0], pose_end[1], pose_end[2])
    path, _ = dubins.shortest_path(q0, q1, turning_radius).sample_many(step_size)
    return np.asarray(path)
