"""Warm-start -> OBCA initial guess glue (R/obca_py/util.py:7-113) and the
arc-length cubic spline it uses (R/obca_py/cubic_spline.py:19-112)."""
import math

import numpy as np
from scipy.interpolate import CubicSpline


def wrap_angle(angle):
    """util.py:7-13 (floored modulo)."""
    return (angle + math.pi) % (2 * math.pi) - math.pi


def convert_angle_to_monotonic(raw_angles):
    """util.py:29-43."""
    if len(raw_angles) <= 1:
        return np.copy(raw_angles)
    out = np.zeros(len(raw_angles))
    out[0] = raw_angles[0]
    for i in range(1, len(raw_angles)):
        out[i] = out[i - 1] + wrap_angle(raw_angles[i] - raw_angles[i - 1])
    return out


def process_angle(raw_angles):
    """util.py:16-26."""
    adj = np.array([wrap_angle(a) for a in raw_angles], dtype=np.float64)
    return convert_angle_to_monotonic(adj)


class Spline2D:
    """cubic_spline.py:19-89: x(s), y(s) not-a-knot cubic splines over arc length."""

    def __init__(self, x, y):
        dx, dy = np.diff(x), np.diff(y)
        self.ds = np.hypot(dx, dy)
        self.s = [0] + list(np.cumsum(self.ds))
        self.sx = CubicSpline(self.s, x)
        self.sy = CubicSpline(self.s, y)

    def calc_position(self, s):
        return self.sx(s), self.sy(s)

    def calc_curvature(self, s):
        dx, dy = np.asarray(self.sx(s, 1)), np.asarray(self.sy(s, 1))
        ddx, ddy = np.asarray(self.sx(s, 2)), np.asarray(self.sy(s, 2))
        return (ddy * dx - ddx * dy) / ((dx ** 2 + dy ** 2) ** (3.0 / 2.0))

    def calc_yaw(self, s):
        return np.arctan2(self.sy(s, 1), self.sx(s, 1))


def calc_spline_course(x, y, ds=0.1):
    """cubic_spline.py:92-112 (vectorised sampling; same values).  Note the
    reference's singular-point filter deletes index *tuples* from np.where, i.e.
    consecutive duplicate points."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    singular = np.where((np.diff(x) == 0) & (np.diff(y) == 0))
    if len(singular) > 0:
        x = np.delete(x, singular, axis=0)
        y = np.delete(y, singular, axis=0)
    sp = Spline2D(x, y)
    s = list(np.arange(0, sp.s[-1] + ds, ds))
    sa = np.asarray(s)
    rx, ry = sp.calc_position(sa)
    return list(rx), list(ry), list(sp.calc_yaw(sa)), list(sp.calc_curvature(sa)), s


def get_init_ref_path_coarse(car, path_xs, path_ys, path_yaws, path_ks, dirs, desired_v=0.5, ds=0.1):
    """util.py:46-59."""
    ref = np.vstack([path_xs, path_ys, dirs, path_yaws, path_ks]).T.astype(np.float64)
    ref[:, 2] = np.asarray(dirs) * desired_v
    ref[:, -1] = np.arctan(car.WHEEL_BASE * np.array(path_ks))
    ref[:, 3] = process_angle(ref[:, 3])
    ref[0, 2] = 0
    ref[-1, 2] = 0
    return ref


def get_init_ref_path(car, path_xs, path_ys, path_yaws, path_ks, dirs, desired_v=0.5, ds=0.1):
    """util.py:62-113: split at gear changes, re-spline each segment at ds,
    v = dir*desired_v, steer = atan(L*kappa) (sign-flipped in reverse), heading
    wrapped + unwrapped, v[0] = v[-1] = 0."""
    ref_path = np.vstack([path_xs, path_ys, path_yaws, path_ks, dirs]).T.astype(np.float64)
    dividers = np.where(np.diff(ref_path[:, -1]) != 0)[0]
    segs = []
    if len(dividers) > 0:
        for i, idx in enumerate(dividers):
            segs.append(ref_path[: idx + 1] if i == 0 else ref_path[dividers[i - 1] + 1: idx + 1])
        segs.append(ref_path[idx + 1:])
    else:
        segs.append(ref_path)
    ref = None
    for path in segs:
        xs, ys, yaws, ks, _ = calc_spline_course(path[:, 0], path[:, 1], ds=ds)
        if path[-1, -1] < 0:
            yaws = wrap_angle(np.array(yaws) + np.pi)
            steer_dir = -1
        else:
            steer_dir = 1
        steers = np.arctan(car.WHEEL_BASE * np.array(ks)) * steer_dir
        vs = np.ones_like(xs) * path[0, -1] * desired_v
        vs[0] = 0
        steers[0] = 0
        traj = np.vstack([xs, ys, vs, yaws, steers]).T
        ref = traj if ref is None else np.vstack([ref, traj])
    ref[:, 3] = process_angle(ref[:, 3])
    ref[0, 2] = 0
    ref[-1, 2] = 0
    return ref


def get_init_ref_path_batch(car, paths, desired_v=0.5, ds=0.1, device=0):
    """get_init_ref_path (util.py:62-113) for many warm-start paths in one HIP launch
    (include/htp.h htp_init_ref_path_batch; one path per wavefront, no CPU fallback).
    paths: list of (xs, ys, yaws, ks, dirs) as returned by the planners; returns a list of
    (rows, 5) arrays [x, y, v, theta, steer].  Raises ValueError where scipy's CubicSpline
    would (a gear segment with fewer than two distinct points)."""
    from .. import _native
    from .optimizer import _context
    packed = _native.RefPathPacked([(p[0], p[1], p[4]) for p in paths],
                                   [(car.WHEEL_BASE, desired_v, ds)] * len(paths))
    res = _context(device).init_ref_path(packed)
    out = []
    for b in range(len(paths)):
        st = int(res.status[b])
        if st == 2:
            raise ValueError(f"[init_ref_path] path {b}: a gear segment has fewer than two distinct points")
        if st != 0:
            raise RuntimeError(f"[init_ref_path] path {b}: {_native.RP_STATUS.get(st, st)}")
        out.append(res.path(b))
    return out


def get_init_ref_path_gpu(car, path_xs, path_ys, path_yaws, path_ks, dirs, desired_v=0.5, ds=0.1):
    """Single-path form of get_init_ref_path_batch (same signature as get_init_ref_path)."""
    return get_init_ref_path_batch(car, [(path_xs, path_ys, path_yaws, path_ks, dirs)], desired_v, ds)[0]
