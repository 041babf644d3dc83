"""Small path helpers of R/path_planner/utils/path_utils.py (:5-29), used by
the flat-import drop-in (`from utils.path_utils import angle_wrap`)."""
import math

import numpy as np


def calculate_path_length(xs, ys):
    """Arc length of a polyline (path_utils.py:5-12)."""
    return np.cumsum(np.hypot(np.diff(xs), np.diff(ys)))[-1]


def get_projection_point(x_m, y_m, yaw_m, k_m, x, y):
    """Projection of (x, y) on the tangent at (x_m, y_m, yaw_m) (path_utils.py:15-23)."""
    tau = np.array([math.cos(yaw_m), math.sin(yaw_m)])
    along = np.array([x - x_m, y - y_m]).dot(tau)
    return np.array([x_m, y_m]) + along * tau, yaw_m + k_m * along


def angle_wrap(angles):
    """Wrap to [-pi, pi) with Python's floored modulo (path_utils.py:26-29)."""
    return (angles + math.pi) % (2 * math.pi) - math.pi
