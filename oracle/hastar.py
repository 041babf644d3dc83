"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's hybrid A*
warm-start search, the checker for the HIP search
kernel in headland_trajectory_planning_amd/csrc/hastar_core.h.  Never imported
by the product.

Follows, line by line:
  R/path_planner/hybrid_a_star_search.py
      calculate_node_index :82-89, init_node :110-127,
      calculate_reeds_shepp_path_cost :129-160 (incl. the `len(np.where(..))`
      quirk that always counts 1, and the "WB" left-steer that never matches),
      _get_goal_extension_with_reeds_shepp_path :232-287 (heapdict over paths),
      simulated_path_cost :306-329, motion steers :331-354,
      kinematic_simulation_node :357-410, check_collision :412-427,
      get_path_from_expanded_nodes :429-454, check_the_arrival :464-495,
      hybrid_a_star_search :497-607 (open/closed dicts, heapdict priority
      max(g, 50 h), strict-improvement replacement :590).
  R/path_planner/reference_line_heuristic.py
      check_path_feasibility :105-118, get_search_length :120-129,
      calculate_state_cost :131-158.
  R/path_planner/orchard_geometry_environment.py
      check_path_feasibility :423-458 with boundary_check=True, aux_check=False
      (nearest-then-intersects == any-intersects; field polygon containment).
  R/path_planner/car_model.py get_path_poly :39-73 (body at every pose).
  heapdict 1.0.1 (third-party, `heapdict.heapdict`): restated below.

shapely/GEOS is absent here, so the geometric predicates are restated on the
lowered geometry (htp_hastar problem format, see hastar_problem()):
  * union-of-footprints intersects a blocker  <=>  some footprint intersects it
    (closed convex polygons, separating-axis test);
  * field.contains(union)  <=>  every footprint inside the (simple) field
    polygon: all corners inside (crossing number) and no proper edge crossing;
  * guided_lane.contains(union)  <=>  every footprint edge covered by the
    union of its clip intervals against the convex lane polygons (valid while
    the lane union has no hole smaller than a footprint);
  * segment_lane.contains(point): strictly inside the convex lane polygon.
These agree with GEOS's exact predicates except on measure-zero boundary
contacts.  Parity status: pinned end-to-end by the notebook (HA* counter = 1,
R/test/obca.ipynb:253-255) through tests/test_hastar_cpu.py; otherwise
"restated, shapely unavailable" (SURVEY.md §8c).
"""
import math

import numpy as np

from . import dubins_spline as ods
from . import reeds_shepp as ors

# hybrid_a_star_search.py:28-36
STEER_COST = 1
DELTA_STEER_COST = 5
DIRECTION_CHANGE_COST = 1000
REVERSE_COST = 5000
HYBRID_COST = 50
MIN_LENGTH_TO_GOAL = 1000
# reference_line_heuristic.py:14
ACCEPT_PATH_DEVIATION = 2

ST_FOUND, ST_NO_PATH, ST_MAX_NODES, ST_START_GOAL_BLOCKED, ST_RS_ERROR = 0, 1, 2, 3, 4


class HeapDict:
    """heapdict 1.0.1 semantics: __setitem__ on an existing key deletes it
    (bubble to the root unconditionally, then popitem) and re-appends;
    _decrease_key moves up while parent >= child; _min_heapify uses strict <."""

    def __init__(self):
        self.heap = []  # [value, key, pos]
        self.d = {}

    def __len__(self):
        return len(self.d)

    def __contains__(self, k):
        return k in self.d

    def _swap(self, i, j):
        h = self.heap
        h[i], h[j] = h[j], h[i]
        h[i][2] = i
        h[j][2] = j

    def _decrease_key(self, i):
        while i:
            parent = (i - 1) >> 1
            if self.heap[parent][0] < self.heap[i][0]:
                break
            self._swap(i, parent)
            i = parent

    def _min_heapify(self, i):
        h = self.heap
        n = len(h)
        while True:
            l, r = 2 * i + 1, 2 * i + 2
            low = l if (l < n and h[l][0] < h[i][0]) else i
            if r < n and h[r][0] < h[low][0]:
                low = r
            if low == i:
                break
            self._swap(i, low)
            i = low

    def popitem(self):
        w = self.heap[0]
        if len(self.heap) == 1:
            self.heap.pop()
        else:
            self.heap[0] = self.heap.pop()
            self.heap[0][2] = 0
            self._min_heapify(0)
        del self.d[w[1]]
        return w[1], w[0]

    def _delete(self, key):
        w = self.d[key]
        while w[2]:
            parent = self.heap[(w[2] - 1) >> 1]
            self._swap(w[2], parent[2])
        self.popitem()

    def __setitem__(self, key, value):
        if key in self.d:
            self._delete(key)
        w = [value, key, len(self)]
        self.d[key] = w
        self.heap.append(w)
        self._decrease_key(len(self.heap) - 1)


def angle_wrap(a):
    """path_utils.angle_wrap (Python / numpy floored modulo)."""
    return (a + math.pi) % (2 * math.pi) - math.pi


# ---------------------------------------------------------------- geometry
def place(poly, poses):
    """car_model.get_path_poly :42-51: R(yaw) @ poly + (x, y) -> (P, k, 2)."""
    poses = np.asarray(poses, dtype=np.float64).reshape(-1, 3)
    c = np.cos(poses[:, 2])[:, None]
    s = np.sin(poses[:, 2])[:, None]
    vx, vy = poly[None, :, 0], poly[None, :, 1]
    px = c * vx + (-s) * vy + poses[:, 0:1]
    py = s * vx + c * vy + poses[:, 1:2]
    return np.stack([px, py], axis=2)


def _edges(poly):
    return np.roll(poly, -1, axis=-2) - poly


def sat_intersects(F, Q):
    """Closed convex polygons F[p] (P,k,2) vs Q (m,2): True where they touch or overlap."""
    sep = np.zeros(F.shape[0], dtype=bool)
    for ax in (_edges(F), np.broadcast_to(_edges(Q), (F.shape[0],) + Q.shape)):
        n = np.stack([ax[..., 1], -ax[..., 0]], axis=-1)  # (P,e,2)
        pa = np.einsum("pkd,ped->pke", F, n)
        pb = np.einsum("md,ped->pme", Q, n)
        s = (pa.max(1) < pb.min(1)) | (pb.max(1) < pa.min(1))  # (P,e)
        sep |= s.any(1)
    return ~sep


def ccw(poly):
    a = np.sum(poly[:, 0] * np.roll(poly[:, 1], -1) - np.roll(poly[:, 0], -1) * poly[:, 1])
    return poly if a > 0 else poly[::-1].copy()


def convex_contains_point(C, px, py):
    """Point strictly inside the convex polygon C (CCW)."""
    a, b = C, np.roll(C, -1, axis=0)
    cr = (b[:, 0] - a[:, 0]) * (py - a[:, 1]) - (b[:, 1] - a[:, 1]) * (px - a[:, 0])
    return bool(np.all(cr > 0))


def clip_interval(C, A, B):
    """Parameter interval of segments A[i] + t (B[i] - A[i]) inside the closed
    convex polygon C (CCW): (lo, hi) arrays, empty where lo > hi."""
    lo = np.zeros(A.shape[0])
    hi = np.ones(A.shape[0])
    for i in range(C.shape[0]):
        v, w = C[i], C[(i + 1) % C.shape[0]]
        ex, ey = w[0] - v[0], w[1] - v[1]
        c0 = ex * (A[:, 1] - v[1]) - ey * (A[:, 0] - v[0])
        c1 = ex * (B[:, 1] - A[:, 1]) - ey * (B[:, 0] - A[:, 0])
        with np.errstate(divide="ignore", invalid="ignore"):
            t = -c0 / c1
        lo = np.where(c1 > 0, np.maximum(lo, t), lo)
        hi = np.where(c1 < 0, np.minimum(hi, t), hi)
        dead = (c1 == 0) & (c0 < 0)
        lo = np.where(dead, 2.0, lo)
    return lo, hi


def lane_covers(F, lanes):
    """Every edge of every footprint F[p] covered by the union of the lanes."""
    P, k = F.shape[0], F.shape[1]
    A = F.reshape(-1, 2)
    B = np.roll(F, -1, axis=1).reshape(-1, 2)
    ivs = [clip_interval(C, A, B) for C in lanes]
    ok = np.zeros(A.shape[0], dtype=bool)
    for e in range(A.shape[0]):
        iv = sorted((lo[e], hi[e]) for lo, hi in ivs if lo[e] <= hi[e])
        reach = 0.0
        good = bool(iv)
        for lo, hi in iv:
            if lo > reach:
                good = False
                break
            reach = max(reach, hi)
        ok[e] = good and reach >= 1.0
    return ok.reshape(P, k).all(1)


def _orient(ax, ay, bx, by, cx, cy):
    return (bx - ax) * (cy - ay) - (by - ay) * (cx - ax)


def field_contains(F, field):
    """Every footprint F[p] inside the simple polygon `field` (V,2)."""
    P, k = F.shape[0], F.shape[1]
    X, Y = F[..., 0], F[..., 1]
    V = field.shape[0]
    inside = np.zeros((P, k), dtype=bool)
    for i in range(V):
        xi, yi = field[i]
        xj, yj = field[(i + 1) % V]
        cond = (yi > Y) != (yj > Y)
        with np.errstate(divide="ignore", invalid="ignore"):
            xc = (xj - xi) * (Y - yi) / (yj - yi) + xi
        inside ^= cond & (X < xc)
    ok = inside.all(1)
    A = F
    B = np.roll(F, -1, axis=1)
    for i in range(V):
        cx, cy = field[i]
        dx, dy = field[(i + 1) % V]
        o1 = _orient(A[..., 0], A[..., 1], B[..., 0], B[..., 1], cx, cy)
        o2 = _orient(A[..., 0], A[..., 1], B[..., 0], B[..., 1], dx, dy)
        o3 = _orient(cx, cy, dx, dy, A[..., 0], A[..., 1])
        o4 = _orient(cx, cy, dx, dy, B[..., 0], B[..., 1])
        cross = (o1 * o2 < 0) & (o3 * o4 < 0)
        ok &= ~cross.any(1)
    return ok


# ---------------------------------------------------------------- problem
def hastar_problem(start, goal, body, blockers, field, lanes, search_lengths, guide, *, king=True,
                   res=0.1, yaw_res=math.radians(10), max_nodes=2000, wheel_base=1.9, max_steer=0.55,
                   default_search_length=1.5):
    """Flat description of one HybridAStarSearch(...).hybrid_a_star_search(max_nodes) call."""
    return dict(start=np.asarray(start, np.float64)[:3], goal=np.asarray(goal, np.float64)[:3],
                body=np.asarray(body, np.float64), blockers=[np.asarray(b, np.float64) for b in blockers],
                field=None if field is None else np.asarray(field, np.float64),
                lanes=[ccw(np.asarray(c, np.float64)) for c in lanes],
                search_lengths=np.asarray(search_lengths, np.float64), guide=np.asarray(guide, np.float64),
                king=bool(king), res=float(res), yaw_res=float(yaw_res), max_nodes=int(max_nodes),
                wheel_base=float(wheel_base), max_steer=float(max_steer),
                default_search_length=float(default_search_length))


def motion_steers(max_steer, yaw_res, king):
    """_get_motion_steers_dubins :331-341 / _reeds_shepp :343-354."""
    if king:
        s = np.arange(max_steer, -(max_steer + yaw_res / 2.0), -yaw_res / 2.0)
        d = np.ones_like(s)
        d[1:len(d):2] = -1
    else:
        s = np.arange(max_steer, -(max_steer + yaw_res), -yaw_res)
        d = np.ones_like(s)
    return np.vstack((s, d)).T


class _Node:
    __slots__ = ("grid", "traj", "curv", "cost", "dirs", "parent")

    def __init__(self, grid, traj, curv, cost, dirs, parent):
        self.grid, self.traj, self.curv, self.cost, self.dirs, self.parent = grid, traj, curv, cost, dirs, parent


class HybridAStar:
    def __init__(self, prob):
        self.p = prob
        self.curvature = math.tan(prob["max_steer"]) / prob["wheel_base"]   # car_model.py:34
        self.steers = motion_steers(prob["max_steer"], prob["yaw_res"], prob["king"])
        self.n_collision_checks = 0
        self.n_pose_checks = 0

    # ------------------------------------------------------------ predicates
    def collides(self, traj):
        """check_collision :412-427."""
        p = self.p
        traj = np.asarray(traj, dtype=np.float64).reshape(-1, 3)
        self.n_collision_checks += 1
        self.n_pose_checks += traj.shape[0]
        F = place(p["body"], traj)
        for Q in p["blockers"]:
            if sat_intersects(F, Q).any():
                return True
        if p["field"] is not None and not field_contains(F, p["field"]).all():
            return True
        if not lane_covers(F, p["lanes"]).all():
            return True
        return False

    def search_length(self, pose):
        """get_search_length :120-129 (the last containing segment wins)."""
        out = self.p["default_search_length"]
        for j, C in enumerate(self.p["lanes"]):
            if convex_contains_point(C, pose[0], pose[1]):
                out = self.p["search_lengths"][j]
        return out

    def heuristic(self, pose):
        """calculate_state_cost :131-158."""
        g = self.p["guide"]
        dists = np.hypot(g[:, 0] - pose[0], g[:, 1] - pose[1])
        m = int(np.argmin(dists))
        dtp = dists[m] * 100
        yaw_diff = abs(angle_wrap(g[m, 2] - pose[2]))
        if dtp > ACCEPT_PATH_DEVIATION:
            dtp = 100
        dist_to_goal = g[-1, -1] - g[m, -1]
        return dtp + yaw_diff * 0.2 + dist_to_goal * 5

    def index(self, x, y, yaw):
        """calculate_node_index :82-89 (Python round: half to even)."""
        return (round(x / self.p["res"]), round(y / self.p["res"]), round(yaw / self.p["yaw_res"]))

    # ------------------------------------------------------------ expansion
    def simulate(self, node, cmd):
        """kinematic_simulation_node :357-410 -> (child or None)."""
        p = self.p
        steer, direction = cmd[0], cmd[1]
        res = p["res"]
        L = self.search_length(node.traj[-1])
        n = round(L / res)
        yaw_step = direction * res / p["wheel_base"] * math.tan(steer)
        init_yaw = angle_wrap(node.traj[-1][2] + yaw_step)
        yaws = np.linspace(init_yaw, init_yaw + yaw_step * (n + 1), n + 2)
        yaws = angle_wrap(yaws)
        xs = node.traj[-1][0] + np.cumsum(res * np.cos(yaws[:-1]) * direction)
        ys = node.traj[-1][1] + np.cumsum(res * np.sin(yaws[:-1]) * direction)
        traj = np.vstack([xs, ys, yaws[1:]]).T
        grid = self.index(traj[-1][0], traj[-1][1], traj[-1][2])
        if self.collides(traj):
            return None
        # simulated_path_cost :306-329
        cost = node.cost
        cost += np.cumsum(np.hypot(np.diff(traj[:, 0]), np.diff(traj[:, 1])))[-1]
        if direction == -1:
            cost += REVERSE_COST
        cost += steer * STEER_COST
        cost += abs(steer - math.atan(node.curv[0] * p["wheel_base"])) * DELTA_STEER_COST
        if node.dirs[0] != direction:
            cost += DIRECTION_CHANGE_COST
        curv = np.tan(steer) / p["wheel_base"]
        return _Node(grid, traj, [curv] * len(traj), cost, [direction] * len(traj), node.grid)

    def rs_cost(self, node, path):
        """calculate_reeds_shepp_path_cost :129-160."""
        cost = node.cost
        lens = np.array(path.lengths)
        nneg = int(np.sum(lens < 0))
        cost += REVERSE_COST * nneg + (len(lens) - nneg)
        cost += 1 * DIRECTION_CHANGE_COST
        cost += self.p["max_steer"] * STEER_COST * 1
        types = np.array(path.ctypes)
        steers = np.zeros(len(types))
        steers[np.where(types == "R")[0]] = -self.p["max_steer"]
        cost += np.sum(np.abs(np.diff(steers)))
        return cost

    def goal_extension(self, node):
        """_get_goal_extension_with_reeds_shepp_path :232-287."""
        s, g = node.traj[-1], self.goal.traj[-1]
        paths = ors.calc_all_paths(s[0], s[1], s[2], g[0], g[1], g[2], self.curvature, self.p["res"])
        if not paths:
            return None
        q = HeapDict()
        for i, path in enumerate(paths):
            q[i] = self.rs_cost(node, path)
        while len(q):
            i, c = q.popitem()
            path = paths[i]
            traj = np.array([path.x, path.y, path.yaw]).T
            if not self.collides(traj) and path.L < MIN_LENGTH_TO_GOAL:
                return _Node(self.goal.grid, traj, path.cs, c, path.directions, node.grid)
        return None

    def goal_extension_dubins(self, node):
        """_get_goal_extension_with_dubins_path :184-230 (get_dubins_path :289-304,
        calculate_dubins_path_cost :162-182; the cost is a (cost, length) tuple there)."""
        s, g = node.traj[-1], self.goal.traj[-1]
        res = self.p["res"]
        smp = ods.dubins_samples([s[0], s[1], s[2]], [g[0], g[1], g[2]], 1.0 / self.curvature, res)
        pts = np.vstack([np.array(smp), np.array([[g[0], g[1], g[2]]])])
        xs, ys, yaws, ks, _ = ods.calc_spline_course(pts[:, 0], pts[:, 1], ds=res)
        path = np.array([xs, ys, yaws, ks]).T
        cost = node.cost + np.cumsum(np.hypot(np.diff(path[:, 0]), np.diff(path[:, 1])))[-1] * 1
        cost += angle_wrap(np.max(path[:, -1]) - np.min(path[:, -1])) * 1
        traj = np.copy(path[:, :3])
        traj[:, -1] = angle_wrap(traj[:, -1])
        length = np.cumsum(np.hypot(np.diff(path[:, 0]), np.diff(path[:, 1])))[-1]
        ks = list(path[:, 3])
        if not self.collides(traj) and length < MIN_LENGTH_TO_GOAL:
            return _Node(self.goal.grid, traj, ks, cost, np.ones_like(ks).tolist(), node.grid)
        return None

    def arrival(self, ext, node):
        """check_the_arrival :464-495."""
        goal_node = ext
        g0 = self.goal.traj[0]
        c = node.traj[-1]
        if (abs(c[0] - g0[0]) < self.p["res"] and abs(c[1] - g0[1]) < self.p["res"]
                and abs(angle_wrap(c[2] - g0[2])) < self.p["yaw_res"]):
            goal_node = node
            goal_node.grid = self.goal.grid
        return goal_node

    def init_node(self, pose):
        g = self.index(pose[0], pose[1], pose[2])
        return _Node(g, [list(map(float, pose[:3]))], [0], 0, [1], g)

    # ------------------------------------------------------------ search
    def search(self):
        """hybrid_a_star_search :497-607 -> dict(xs, ys, yaws, dirs, ks, counter, status, expanded)."""
        p = self.p
        self.start = self.init_node(p["start"])
        self.goal = self.init_node(p["goal"])
        open_set = {self.start.grid: self.start}
        closed = {}
        q = HeapDict()
        q[self.start.grid] = max(self.start.cost, HYBRID_COST * self.heuristic(self.start.traj[-1]))
        counter = 0
        expanded = []
        out = dict(xs=[], ys=[], yaws=[], dirs=[], ks=[], counter=0, expanded=expanded)
        if self.collides(self.start.traj) or self.collides(self.goal.traj):
            out["status"] = ST_START_GOAL_BLOCKED
            return out
        status = ST_NO_PATH
        try:
            while True:
                if counter > p["max_nodes"]:
                    status = ST_MAX_NODES
                    break
                counter += 1
                if not open_set:
                    status = ST_NO_PATH
                    break
                idx, _ = q.popitem()
                cur = open_set.pop(idx)
                closed[idx] = cur
                expanded.append(idx)
                ext = self.goal_extension(cur) if p["king"] else self.goal_extension_dubins(cur)
                gn = self.arrival(ext, cur)
                if gn is not None:
                    closed[gn.grid] = gn
                    status = ST_FOUND
                    break
                for cmd in self.steers:
                    ch = self.simulate(cur, cmd)
                    if ch is None:
                        continue
                    k = ch.grid
                    if k in closed:
                        continue
                    if k not in open_set or ch.cost < open_set[k].cost:
                        open_set[k] = ch
                        q[k] = max(ch.cost, HYBRID_COST * self.heuristic(ch.traj[-1]))
        except (AssertionError, IndexError):
            out["status"] = ST_RS_ERROR
            out["counter"] = counter
            return out
        out["status"] = status
        out["counter"] = counter
        # get_path_from_expanded_nodes :429-454
        k = self.goal.parent
        if k in closed:
            xs, ys, yaws, dirs, ks = [], [], [], [], []
            node = closed[k]
            while k != self.start.grid:
                a, b, c = zip(*node.traj)
                xs += a[::-1]
                ys += b[::-1]
                yaws += c[::-1]
                dirs += list(node.dirs)[::-1]
                ks += list(node.curv)[::-1]
                k = node.parent
                node = closed[k]
            out.update(xs=[float(v) for v in xs[::-1]], ys=[float(v) for v in ys[::-1]],
                       yaws=[float(v) for v in yaws[::-1]], dirs=[float(v) for v in dirs[::-1]],
                       ks=[float(v) for v in ks[::-1]])
        return out
