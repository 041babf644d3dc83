"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's Reeds-Shepp
path set (R/path_planner/utils/reeds_shepp.py), used as the checker for the
HIP kernels in headland_trajectory_planning_amd/csrc/htp_rs.hip.  Never
imported by the product.

Pinned against golden vectors produced by the reference itself
(tests/golden/rs_calc_all_paths.npz, tests/golden/make_golden.py): identical
path lists, ctypes, lengths, sample counts and sample values (bit-for-bit on
this host's libm).

The candidate list is generated from the Reeds-Shepp symmetry group instead of
being spelled out: every base word is evaluated under
    identity   (x,  y,  phi)           lengths as is
    time-flip  (-x, y, -phi)           lengths negated
    reflect    (x, -y, -phi)           L <-> R
    both       (-x, -y, phi)           negated, L <-> R
and, for CCC and CCSC, on the "backwards" pose (reeds_shepp.py:221-223) with
the word read in reverse.  The enumeration order reproduces generate_path
(:565-582), which matters because de-duplication (set_path, :68-86) keeps the
first of two near-equal words.
"""
import math

PI = math.pi
MAX_LENGTH = 1000.0  # reeds_shepp.py:6
HALF = 0.5 * PI


def pymod_2pi(theta):
    return theta % (2.0 * PI)


def wrap_pm_pi(theta):
    """M() (:620-632): Python modulo into [0, 2pi) then shift."""
    phi = pymod_2pi(theta)
    if phi < -PI:
        phi += 2.0 * PI
    if phi > PI:
        phi -= 2.0 * PI
    return phi


def pi_2_pi(theta):
    """pi_2_pi (:597-604)."""
    while theta > PI:
        theta -= 2.0 * PI
    while theta < -PI:
        theta += 2.0 * PI
    return theta


def polar(x, y):
    return math.hypot(x, y), math.atan2(y, x)


# ---------------------------------------------------------------- base words
# Each returns (t, u, v) or None (formulas of Reeds & Shepp 1990 as the
# reference evaluates them, :144-160, :88-128, :285-323, :326-351, :406-421).

def word_SLS(x, y, phi):
    phi = wrap_pm_pi(phi)
    if not (0.0 < phi < PI * 0.99) or y == 0.0:
        return None
    xd = -y / math.tan(phi) + x
    tan_half = math.tan(phi / 2.0)
    dist = math.sqrt((x - xd) ** 2 + y ** 2)
    if y < 0.0:
        dist = -dist
    return xd - tan_half, phi, dist - tan_half


def word_LSL(x, y, phi):
    u, t = polar(x - math.sin(phi), y - 1.0 + math.cos(phi))
    if t < 0.0:
        return None
    v = wrap_pm_pi(phi - t)
    return (t, u, v) if v >= 0.0 else None


def word_LSR(x, y, phi):
    r, t1 = polar(x + math.sin(phi), y - 1.0 - math.cos(phi))
    r2 = r ** 2
    if r2 < 4.0:
        return None
    u = math.sqrt(r2 - 4.0)
    t = wrap_pm_pi(t1 + math.atan2(2.0, u))
    v = wrap_pm_pi(t - phi)
    return (t, u, v) if (t >= 0.0 and v >= 0.0) else None


def word_LRL(x, y, phi):
    r, t1 = polar(x - math.sin(phi), y - 1.0 + math.cos(phi))
    if r > 4.0:
        return None
    u = -2.0 * math.asin(0.25 * r)
    t = wrap_pm_pi(t1 + 0.5 * u + PI)
    v = wrap_pm_pi(phi - t + u)
    return (t, u, v) if (t >= 0.0 and u <= 0.0) else None


def _tau_omega(u, v, xi, eta, phi):
    delta = wrap_pm_pi(u - v)
    a = math.sin(u) - math.sin(delta)
    b = math.cos(u) - math.cos(delta) - 1.0
    t1 = math.atan2(eta * a - xi * b, xi * a + eta * b)
    t2 = 2.0 * (math.cos(delta) - math.cos(v) - math.cos(u)) + 3.0
    tau = wrap_pm_pi(t1 + PI) if t2 < 0 else wrap_pm_pi(t1)
    return tau, wrap_pm_pi(tau - u + v - phi)


def word_LRLRn(x, y, phi):
    xi, eta = x + math.sin(phi), y - 1.0 - math.cos(phi)
    rho = 0.25 * (2.0 + math.sqrt(xi * xi + eta * eta))
    if rho > 1.0:
        return None
    u = math.acos(rho)
    t, v = _tau_omega(u, -u, xi, eta, phi)
    return (t, u, v) if (t >= 0.0 and v <= 0.0) else None


def word_LRLRp(x, y, phi):
    xi, eta = x + math.sin(phi), y - 1.0 - math.cos(phi)
    rho = (20.0 - xi * xi - eta * eta) / 16.0
    if not (0.0 <= rho <= 1.0):
        return None
    u = -math.acos(rho)
    if u < -0.5 * PI:
        return None
    t, v = _tau_omega(u, u, xi, eta, phi)
    return (t, u, v) if (t >= 0.0 and v >= 0.0) else None


def word_LRSR(x, y, phi):
    xi, eta = x + math.sin(phi), y - 1.0 - math.cos(phi)
    rho, theta = polar(-eta, xi)
    if rho < 2.0:
        return None
    t, u = theta, 2.0 - rho
    v = wrap_pm_pi(t + 0.5 * PI - phi)
    return (t, u, v) if (t >= 0.0 and u <= 0.0 and v <= 0.0) else None


def word_LRSL(x, y, phi):
    xi, eta = x - math.sin(phi), y - 1.0 + math.cos(phi)
    rho, theta = polar(xi, eta)
    if rho < 2.0:
        return None
    r = math.sqrt(rho * rho - 4.0)
    u = 2.0 - r
    t = wrap_pm_pi(theta + math.atan2(r, -2.0))
    v = wrap_pm_pi(phi - 0.5 * PI - t)
    return (t, u, v) if (t >= 0.0 and u <= 0.0 and v <= 0.0) else None


def word_LRSLR(x, y, phi):
    xi, eta = x + math.sin(phi), y - 1.0 - math.cos(phi)
    rho, _ = polar(xi, eta)
    if rho < 2.0:
        return None
    u = 4.0 - math.sqrt(rho * rho - 4.0)
    if u > 0.0:
        return None
    t = wrap_pm_pi(math.atan2((4.0 - u) * xi - 2.0 * eta, -2.0 * xi + (u - 4.0) * eta))
    v = wrap_pm_pi(t - phi)
    return (t, u, v) if (t >= 0.0 and v >= 0.0) else None


# base word -> (evaluator, segment letters, (t,u,v) -> segment lengths)
BASE = {
    "SLS": (word_SLS, "SLS", lambda t, u, v: [t, u, v]),
    "LSL": (word_LSL, "LSL", lambda t, u, v: [t, u, v]),
    "LSR": (word_LSR, "LSR", lambda t, u, v: [t, u, v]),
    "LRL": (word_LRL, "LRL", lambda t, u, v: [t, u, v]),
    "LRLRn": (word_LRLRn, "LRLR", lambda t, u, v: [t, u, -u, v]),
    "LRLRp": (word_LRLRp, "LRLR", lambda t, u, v: [t, u, u, v]),
    "LRSL": (word_LRSL, "LRSL", lambda t, u, v: [t, -0.5 * PI, u, v]),
    "LRSR": (word_LRSR, "LRSR", lambda t, u, v: [t, -0.5 * PI, u, v]),
    "LRSLR": (word_LRSLR, "LRSLR", lambda t, u, v: [t, -0.5 * PI, u, -0.5 * PI, v]),
}

# symmetry name -> (sign x, sign y, sign phi, negate lengths, swap L/R)
SYM = {"id": (1, 1, 1, False, False), "flip": (-1, 1, -1, True, False),
       "refl": (1, -1, -1, False, True), "both": (-1, -1, 1, True, True)}
ALL4 = ("id", "flip", "refl", "both")

# generate_path order: (base word, symmetries, backwards?)
ORDER = [("SLS", ("id", "refl"), False),
         ("LSL", ALL4, False), ("LSR", ALL4, False),
         ("LRL", ALL4, False), ("LRL", ALL4, True),
         ("LRLRn", ALL4, False), ("LRLRp", ALL4, False),
         ("LRSL", ALL4, False), ("LRSR", ALL4, False), ("LRSL", ALL4, True), ("LRSR", ALL4, True),
         ("LRSLR", ALL4, False)]

_SWAP = str.maketrans("LR", "RL")


def candidates():
    """The 46 (word, symmetry, backwards) triples in reference order."""
    return [(w, s, b) for w, syms, b in ORDER for s in syms]


class Path:
    """Mirror of reeds_shepp.PATH (:12-25)."""

    def __init__(self, lengths, ctypes):
        self.lengths = lengths
        self.ctypes = ctypes
        self.L = 0.0
        self.x, self.y, self.yaw, self.cs, self.directions = [], [], [], [], []


def admissible_words(x, y, phi):
    """generate_path after the pose change: list of Path (normalised lengths)."""
    xb = x * math.cos(phi) + y * math.sin(phi)
    yb = x * math.sin(phi) - y * math.cos(phi)
    out = []
    for w, s, back in candidates():
        fn, letters, lens_of = BASE[w]
        sx, sy, sp, neg, swap = SYM[s]
        px, py = (xb, yb) if back else (x, y)
        r = fn(sx * px if sx < 0 else px, sy * py if sy < 0 else py, -phi if sp < 0 else phi)
        if r is None:
            continue
        lens = lens_of(*r)
        if neg:
            lens = [-a for a in lens]
        segs = letters.translate(_SWAP) if swap else letters
        if back:
            lens, segs = lens[::-1], segs[::-1]
        _insert(out, lens, list(segs))
    return out


def _insert(paths, lengths, ctypes):
    """set_path (:68-86): skip near-duplicates, MAX_LENGTH filter, assert."""
    for p in paths:
        if p.ctypes == ctypes and sum([a - b for a, b in zip(p.lengths, lengths)]) <= 0.01:
            return
    total = sum([abs(a) for a in lengths])
    if total >= MAX_LENGTH:
        return
    if not total >= 0.01:
        raise AssertionError("path shorter than 0.01")
    p = Path(lengths, ctypes)
    p.L = total
    paths.append(p)


def _sample(ind, l, seg, maxc, origin, buf):
    """interpolate (:533-562)."""
    ox, oy, oyaw = origin
    px, py, pyaw, cs, dirs = buf
    if seg == "S":
        px[ind] = ox + l / maxc * math.cos(oyaw)
        py[ind] = oy + l / maxc * math.sin(oyaw)
        pyaw[ind] = oyaw
        cs[ind] = 0
    else:
        ldx = math.sin(l) / maxc
        if seg == "L":
            ldy = (1.0 - math.cos(l)) / maxc
            cs[ind] = maxc
        else:
            ldy = (1.0 - math.cos(l)) / (-maxc)
            cs[ind] = -maxc
        px[ind] = ox + (math.cos(-oyaw) * ldx + math.sin(-oyaw) * ldy)
        py[ind] = oy + (-math.sin(-oyaw) * ldx + math.cos(-oyaw) * ldy)
    if seg == "L":
        pyaw[ind] = oyaw + l
    elif seg == "R":
        pyaw[ind] = oyaw - l
    dirs[ind] = 1 if l > 0.0 else -1


def local_course(L, lengths, segs, maxc, step):
    """generate_local_course (:471-530) with its list semantics (index rewind
    at segment starts, trailing exact-0.0 pop)."""
    n = int(L / step) + len(lengths) + 3
    buf = ([0.0] * n, [0.0] * n, [0.0] * n, [0] * n, [0] * n)
    buf[4][0] = 1 if lengths[0] > 0.0 else -1
    ind = 1
    pd = step if lengths[0] > 0.0 else -step
    rem = 0.0
    for i, (seg, l) in enumerate(zip(segs, lengths)):
        d = step if l > 0.0 else -step
        origin = (buf[0][ind], buf[1][ind], buf[2][ind])
        ind -= 1
        same_dir = i >= 1 and (lengths[i - 1] * lengths[i]) > 0
        pd = (-d - rem) if same_dir else (d - rem)
        while abs(pd) <= abs(l):
            ind += 1
            _sample(ind, pd, seg, maxc, origin, buf)
            pd += d
        rem = l - pd - d
        ind += 1
        _sample(ind, l, seg, maxc, origin, buf)
    px = buf[0]
    keep = len(px)
    while keep > 0 and px[keep - 1] == 0.0:
        keep -= 1
    if keep == 0:  # the reference's `while px[-1] == 0.0: pop()` empties the list
        raise IndexError("pop from empty list")
    return tuple(b[:keep] for b in buf)


def calc_all_paths(sx, sy, syaw, gx, gy, gyaw, maxc, step_size=0.2):
    """calc_all_paths (:39-65)."""
    dx, dy, dth = gx - sx, gy - sy, gyaw - syaw
    c, s = math.cos(syaw), math.sin(syaw)
    x = (c * dx + s * dy) * maxc
    y = (-s * dx + c * dy) * maxc
    paths = admissible_words(x, y, dth)
    cq, sq = math.cos(-syaw), math.sin(-syaw)
    for p in paths:
        lx, ly, lyaw, cs, dirs = local_course(p.L, p.lengths, p.ctypes, maxc, step_size * maxc)
        p.x = [cq * a + sq * b + sx for a, b in zip(lx, ly)]
        p.y = [-sq * a + cq * b + sy for a, b in zip(lx, ly)]
        p.yaw = [pi_2_pi(a + syaw) for a in lyaw]
        p.cs, p.directions = cs, dirs
        p.lengths = [a / maxc for a in p.lengths]
        p.L = p.L / maxc
    return paths
