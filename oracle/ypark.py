"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's Y-type
parking grid search, the checker for csrc/ypark_core.h.  Never imported by the
product.

Follows R/path_planner/headland_path_planning.py:
  search_y_type_parking_path :382-451 (grid axes :404-411 by np.arange, the
  loop order, first feasible wins, end-pose check :400-402),
  calculate_motion_path :455-484, get_y_type_parking_path :487-516,
  get_path_in_odom :519-527 with R/path_planner/utils/transformation.py
  states2SE3 / SE32states and navigation_utils.convert_2d_xys_to_target_frame,
and orchard_geometry_environment.check_path_feasibility :423-458
(boundary_check=True, aux_check=False) through the footprint predicates of
oracle/hastar.py.  Parity: pinned end to end by the notebook's printed
parameters (1.70, 2.00, 0.00, 0.50), R/test/obca.ipynb:253."""
import math

import numpy as np

from . import hastar as oha


def grid(max_steer_backward, max_steer_forward, max_backward_distance, max_forward_distance, min_forward_distance,
         min_backward_distance, min_steer_backward, min_steer_forward):
    sb = list(np.arange(min_steer_backward, max_steer_backward + 0.1, 0.1))
    if np.max(sb) < max_steer_backward:
        sb.append(max_steer_backward)
    sf = list(np.arange(min_steer_forward, max_steer_forward + 0.1, 0.1))
    if np.max(sf) < max_steer_forward:
        sf.append(max_steer_forward)
    return (list(np.arange(max_backward_distance, min_backward_distance, -0.1)),
            list(np.arange(max_forward_distance, min_forward_distance, -0.1)), sb, sf)


def motion_path(init_pose, steer, direction, length, wheel_base, step):
    n = round(length / step)
    yaw_step = direction * step / wheel_base * math.tan(steer)
    init_yaw = oha.angle_wrap(init_pose[-1] + yaw_step)
    yaws = oha.angle_wrap(np.linspace(init_yaw, init_yaw + yaw_step * n, n + 1))
    xs = init_pose[0] + np.cumsum(step * np.cos(yaws[:-1]) * direction)
    ys = init_pose[1] + np.cumsum(step * np.sin(yaws[:-1]) * direction)
    path = np.vstack([init_pose, np.vstack([xs, ys, yaws[1:]]).T])
    k = math.tan(steer) / wheel_base if abs(steer) > 0.00001 else 0
    return np.hstack((path, np.ones((len(path), 1)) * k, np.ones((len(path), 1)) * direction))


def se3(x, y, yaw):
    c, s = math.cos(yaw), math.sin(yaw)
    T = np.diag([1.0, 1.0, 1.0, 1.0])
    T[:3, :3] = np.dot(np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]]), np.eye(3))
    T[:3, 3] = [x, y, 0]
    return T


def y_path(prob, bl, fl, sb, sf):
    back = motion_path([0, 0, 0], sb * prob["bdir"], -1, bl, prob["wheel_base"], prob["step"])
    fwd = motion_path(back[-1, :3], sf * prob["fdir"], 1, fl, prob["wheel_base"], prob["step"])
    back[:, -1] = 1
    fwd[:, -1] = -1
    path = np.vstack([fwd[::-1], back[::-1]])
    e = prob["end_pose"]
    T = se3(e[0], e[1], e[2])
    yaw_odom = math.atan2(T[1, 0], T[0, 0])
    out = np.copy(path)
    out[:, 2] += yaw_odom
    homo = np.vstack([out[:, 0], out[:, 1], np.zeros(len(out)), np.ones(len(out))])
    xy = T.dot(homo)[:2, :].T
    out[:, 0], out[:, 1] = xy[:, 0], xy[:, 1]
    return out


def feasible(prob, path):
    F = oha.place(prob["body"], np.asarray(path)[:, :3])
    for Q in prob["blockers"]:
        if oha.sat_intersects(F, Q).any():
            return False
    if prob["field"] is not None and not oha.field_contains(F, prob["field"]).all():
        return False
    return True


def search(prob):
    """-> dict(status 0 found / 1 none / 2 end blocked, cand, params, path)."""
    e = np.asarray(prob["end_pose"], dtype=np.float64)
    if not feasible(prob, e[None, :3]):
        return dict(status=2, cand=-1, params=[0.0] * 4, path=np.zeros((0, 5)))
    bl, fl, sb, sf = prob["axes"]
    k = 0
    for b in bl:
        for f in fl:
            for s1 in sb:
                for s2 in sf:
                    p = y_path(prob, b, f, s1, s2)
                    if feasible(prob, p):
                        return dict(status=0, cand=k, params=[b, f, s1, s2], path=p)
                    k += 1
    return dict(status=1, cand=-1, params=[0.0] * 4, path=np.zeros((0, 5)))
