"""TEST INFRASTRUCTURE ONLY -- restatements used by oracle/hastar.py for the
Pawn goal shot (hybrid_a_star_search.py:184-230, :289-304):

* pydubins (AndrewWalker/pydubins, unpinned git dependency, R/requirements.txt:13;
  its dubins.c: intermediate results, words LSL LSR RSL RSR RLR LRL in that
  order, strictly cheaper word wins, dubins_path_sample / sample_many with
  x += step while x < length).  Not installed here: "parity unpinned".
* calc_spline_course of R/path_planner/utils/cubic_spline.py:92-112 with
  scipy.interpolate.CubicSpline (not-a-knot), which is importable here."""
import math

import numpy as np
from scipy.interpolate import CubicSpline

TWO_PI = 2 * math.pi
_TYPES = ["LSL", "LSR", "RSL", "RSR", "RLR", "LRL"]


def mod2pi(t):
    return t - TWO_PI * math.floor(t / TWO_PI)


def _words(a, b, d):
    sa, sb, ca, cb = math.sin(a), math.sin(b), math.cos(a), math.cos(b)
    cab = math.cos(a - b)
    dd = d * d
    w = {}
    p2 = 2 + dd - (2 * cab) + (2 * d * (sa - sb))
    if p2 >= 0:
        t1 = math.atan2(cb - ca, d + sa - sb)
        w["LSL"] = (mod2pi(t1 - a), math.sqrt(p2), mod2pi(b - t1))
    p2 = -2 + dd + (2 * cab) + (2 * d * (sa + sb))
    if p2 >= 0:
        p = math.sqrt(p2)
        t0 = math.atan2(-ca - cb, d + sa + sb) - math.atan2(-2.0, p)
        w["LSR"] = (mod2pi(t0 - a), p, mod2pi(t0 - mod2pi(b)))
    p2 = -2 + dd + (2 * cab) - (2 * d * (sa + sb))
    if p2 >= 0:
        p = math.sqrt(p2)
        t0 = math.atan2(ca + cb, d - sa - sb) - math.atan2(2.0, p)
        w["RSL"] = (mod2pi(a - t0), p, mod2pi(b - t0))
    p2 = 2 + dd - (2 * cab) + (2 * d * (sb - sa))
    if p2 >= 0:
        t1 = math.atan2(ca - cb, d - sa + sb)
        w["RSR"] = (mod2pi(a - t1), math.sqrt(p2), mod2pi(t1 - b))
    t0 = (6. - dd + 2 * cab + 2 * d * (sa - sb)) / 8.
    phi = math.atan2(ca - cb, d - sa + sb)
    if abs(t0) <= 1:
        p = mod2pi(TWO_PI - math.acos(t0))
        t = mod2pi(a - phi + mod2pi(p / 2.))
        w["RLR"] = (t, p, mod2pi(a - b - t + mod2pi(p)))
    t0 = (6. - dd + 2 * cab + 2 * d * (sb - sa)) / 8.
    phi = math.atan2(ca - cb, d + sa - sb)
    if abs(t0) <= 1:
        p = mod2pi(TWO_PI - math.acos(t0))
        t = mod2pi(-a - phi + p / 2.)
        w["LRL"] = (t, p, mod2pi(mod2pi(b) - a - t + mod2pi(p)))
    return w


def _seg(t, qi, typ):
    st, ct = math.sin(qi[2]), math.cos(qi[2])
    if typ == "L":
        q = (math.sin(qi[2] + t) - st, -math.cos(qi[2] + t) + ct, t)
    elif typ == "R":
        q = (-math.sin(qi[2] - t) + st, math.cos(qi[2] - t) - ct, -t)
    else:
        q = (ct * t, st * t, 0.0)
    return (q[0] + qi[0], q[1] + qi[1], q[2] + qi[2])


def dubins_samples(q0, q1, rho, step):
    """dubins.shortest_path(q0, q1, rho).sample_many(step)[0]."""
    dx, dy = q1[0] - q0[0], q1[1] - q0[1]
    d = math.sqrt(dx * dx + dy * dy) / rho
    th = mod2pi(math.atan2(dy, dx)) if d > 0 else 0
    a, b = mod2pi(q0[2] - th), mod2pi(q1[2] - th)
    words = _words(a, b, d)
    best, bc = None, math.inf
    for name in _TYPES:
        if name in words:
            c = words[name][0] + words[name][1] + words[name][2]
            if c < bc:
                best, bc = name, c
    prm = words[best]
    length = ((0. + prm[0]) + prm[1] + prm[2]) * rho
    out = []
    x = 0.0
    while x < length:
        tp = x / rho
        qi = (0.0, 0.0, q0[2])
        q1s = _seg(prm[0], qi, best[0])
        q2s = _seg(prm[1], q1s, best[1])
        if tp < prm[0]:
            q = _seg(tp, qi, best[0])
        elif tp < prm[0] + prm[1]:
            q = _seg(tp - prm[0], q1s, best[1])
        else:
            q = _seg(tp - prm[0] - prm[1], q2s, best[2])
        out.append((q[0] * rho + q0[0], q[1] * rho + q0[1], mod2pi(q[2])))
        x += step
    return out


def calc_spline_course(x, y, ds=0.1):
    """cubic_spline.py:92-112 (Spline2D :19-89)."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    sing = np.where((np.diff(x) == 0) & (np.diff(y) == 0))
    if len(sing) > 0:
        x = np.delete(x, sing, axis=0)
        y = np.delete(y, sing, axis=0)
    ss = [0]
    ss.extend(np.cumsum(np.hypot(np.diff(x), np.diff(y))))
    sx, sy = CubicSpline(ss, x), CubicSpline(ss, y)
    s = np.arange(0, ss[-1] + ds, ds)
    dx, dy, ddx, ddy = sx(s, 1), sy(s, 1), sx(s, 2), sy(s, 2)
    k = (ddy * dx - ddx * dy) / ((dx ** 2 + dy ** 2) ** (3.0 / 2.0))
    return sx(s), sy(s), np.arctan2(dy, dx), k, s
