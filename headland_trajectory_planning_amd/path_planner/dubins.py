"""Dubins shortest paths: restatement of pydubins (AndrewWalker/pydubins,
unpinned git dependency of R/requirements.txt:13; its dubins.c:
dubins_intermediate_results, the six words LSL LSR RSL RSR RLR LRL,
dubins_shortest_path (strictly cheaper word wins, in that order),
dubins_path_sample / dubins_segment, dubins_path_sample_many (x = 0, step,
... while x < length)).  pydubins is not installed here, so its outputs are
"parity unpinned" beyond the notebook's end-to-end pins."""
import math

LSL, LSR, RSL, RSR, RLR, LRL = range(6)
_L, _S, _R = 0, 1, 2
_DIRDATA = {LSL: (_L, _S, _L), LSR: (_L, _S, _R), RSL: (_R, _S, _L), RSR: (_R, _S, _R), RLR: (_R, _L, _R),
            LRL: (_L, _R, _L)}
TWO_PI = 2 * math.pi


def _mod2pi(t):
    return t - TWO_PI * math.floor(t / TWO_PI)


def _words(alpha, beta, d):
    sa, sb, ca, cb = math.sin(alpha), math.sin(beta), math.cos(alpha), math.cos(beta)
    c_ab = math.cos(alpha - beta)
    d_sq = d * d
    out = {}
    p_sq = 2 + d_sq - (2 * c_ab) + (2 * d * (sa - sb))
    if p_sq >= 0:
        t1 = math.atan2(cb - ca, d + sa - sb)
        out[LSL] = (_mod2pi(t1 - alpha), math.sqrt(p_sq), _mod2pi(beta - t1))
    p_sq = -2 + d_sq + (2 * c_ab) + (2 * d * (sa + sb))
    if p_sq >= 0:
        p = math.sqrt(p_sq)
        t0 = math.atan2(-ca - cb, d + sa + sb) - math.atan2(-2.0, p)
        out[LSR] = (_mod2pi(t0 - alpha), p, _mod2pi(t0 - _mod2pi(beta)))
    p_sq = -2 + d_sq + (2 * c_ab) - (2 * d * (sa + sb))
    if p_sq >= 0:
        p = math.sqrt(p_sq)
        t0 = math.atan2(ca + cb, d - sa - sb) - math.atan2(2.0, p)
        out[RSL] = (_mod2pi(alpha - t0), p, _mod2pi(beta - t0))
    p_sq = 2 + d_sq - (2 * c_ab) + (2 * d * (sb - sa))
    if p_sq >= 0:
        t1 = math.atan2(ca - cb, d - sa + sb)
        out[RSR] = (_mod2pi(alpha - t1), math.sqrt(p_sq), _mod2pi(t1 - beta))
    t0 = (6. - d_sq + 2 * c_ab + 2 * d * (sa - sb)) / 8.
    phi = math.atan2(ca - cb, d - sa + sb)
    if abs(t0) <= 1:
        p = _mod2pi(TWO_PI - math.acos(t0))
        t = _mod2pi(alpha - phi + _mod2pi(p / 2.))
        out[RLR] = (t, p, _mod2pi(alpha - beta - t + _mod2pi(p)))
    t0 = (6. - d_sq + 2 * c_ab + 2 * d * (sb - sa)) / 8.
    phi = math.atan2(ca - cb, d + sa - sb)
    if abs(t0) <= 1:
        p = _mod2pi(TWO_PI - math.acos(t0))
        t = _mod2pi(-alpha - phi + p / 2.)
        out[LRL] = (t, p, _mod2pi(_mod2pi(beta) - alpha - t + _mod2pi(p)))
    return out


def _segment(t, qi, typ):
    st, ct = math.sin(qi[2]), math.cos(qi[2])
    if typ == _L:
        q = [math.sin(qi[2] + t) - st, -math.cos(qi[2] + t) + ct, t]
    elif typ == _R:
        q = [-math.sin(qi[2] - t) + st, math.cos(qi[2] - t) - ct, -t]
    else:
        q = [ct * t, st * t, 0.0]
    return [q[0] + qi[0], q[1] + qi[1], q[2] + qi[2]]


class DubinsPath:
    def __init__(self, q0, params, rho, ptype):
        self.qi = [float(q0[0]), float(q0[1]), float(q0[2])]
        self.param = list(params)
        self.rho = rho
        self.type = ptype

    def path_length(self):
        length = 0.
        for p in self.param:
            length += p
        return length * self.rho

    def path_type(self):
        return self.type

    def segment_length(self, i):
        return self.param[i] * self.rho

    def sample(self, t):
        tprime = t / self.rho
        qi = [0.0, 0.0, self.qi[2]]
        types = _DIRDATA[self.type]
        p1, p2 = self.param[0], self.param[1]
        q1 = _segment(p1, qi, types[0])
        q2 = _segment(p2, q1, types[1])
        if tprime < p1:
            q = _segment(tprime, qi, types[0])
        elif tprime < (p1 + p2):
            q = _segment(tprime - p1, q1, types[1])
        else:
            q = _segment(tprime - p1 - p2, q2, types[2])
        return (q[0] * self.rho + self.qi[0], q[1] * self.rho + self.qi[1], _mod2pi(q[2]))

    def sample_many(self, step_size):
        qs, ts = [], []
        x = 0.0
        length = self.path_length()
        while x < length:
            qs.append(self.sample(x))
            ts.append(x)
            x += step_size
        return qs, ts


def shortest_path(q0, q1, rho):
    if rho <= 0.0:
        raise RuntimeError("dubins: bad rho")
    dx, dy = q1[0] - q0[0], q1[1] - q0[1]
    D = math.sqrt(dx * dx + dy * dy)
    d = D / rho
    theta = _mod2pi(math.atan2(dy, dx)) if d > 0 else 0
    alpha = _mod2pi(q0[2] - theta)
    beta = _mod2pi(q1[2] - theta)
    best, best_cost = None, math.inf
    words = _words(alpha, beta, d)
    for w in range(6):
        if w in words:
            prm = words[w]
            cost = prm[0] + prm[1] + prm[2]
            if cost < best_cost:
                best, best_cost = w, cost
    if best is None:
        raise RuntimeError("dubins: no path")
    return DubinsPath(q0, words[best], rho, best)
