"""Drop-in replacement for R/obca_py/optimizer_points.py (point-formulation OBCAOptimizer).

Same class constants, constructor, call sequence and solution attributes as the
reference (optimizer_points.py:8-327):

    opt = OBCAOptimizer(car, dT=0.2)            # prints the hull vertices (:33)
    opt.initialize_manual(init_guess_path, obs, min_x=..., init_control=...)
    opt.build_model(); opt.generate_object(r, q); opt.generate_variable(); opt.generate_constrain()
    opt.solve()
    opt.x_opt, opt.y_opt, opt.v_opt, opt.theta_opt, opt.steer_opt, opt.a_opt, opt.steerate_opt

The NLP (hull-vertex distance rows, lambda-only duals, hard start/end states,
objective sum du^2 + 20 (v dT)^2) is packed into flat arrays and solved by the
batched HIP interior-point solver (include/htp.h htp_obca_points_solve_batch),
the IPOPT algorithm restated in oracle/ipm.py.  No CPU fallback.  Like the
reference, `solution_found` only says that a solution vector came back; the
solver status is in `status` / `status_str`.  `solve_batch([...])` solves many
prepared optimizers in one launch (shared N, obstacle edge and vertex counts).
"""
from typing import List

import numpy as np

from .. import _native, geometry
from .car_model_obca import CarModel
from .optimizer import _context


class DM(np.ndarray):
    """Column vector with the two casadi.DM accessors the reference's callers use."""

    def elements(self):
        return [float(v) for v in np.asarray(self).reshape(-1)]

    def full(self):
        return np.asarray(self).reshape(-1, 1).copy()


def _dm(v):
    return np.asarray(v, dtype=np.float64).reshape(-1, 1).view(DM)


class OBCAOptimizer:
    MAX_VELOCITY = 1
    MAX_ACCEL = 1
    MAX_STEER_RATE = 0.7
    MIN_DISTANCE_TO_OBS = 0.1

    def __init__(self, car: CarModel = None, dT=0.2) -> None:
        self.v_car = car if car is not None else CarModel()
        self.dT = dT
        self.n_controls = 2
        self.n_states = 5
        self.constrains = []
        self.lbg = []
        self.ubg = []
        self.lbx = []
        self.ubx = []
        self.variable = []
        self.N = 0
        self.x0 = []
        self.obstacles = []
        self.vertices = self.get_vehicle_vertices(self.v_car)
        print(self.vertices)

    def get_vehicle_vertices(self, car, convex_hull=True):
        """:35-50: origin + body + implement vertices, convex hull (shapely/GEOS order)."""
        polys = [car.car_poly] + list(car.aux_polys)
        if convex_hull:
            return geometry.vehicle_hull_vertices(polys)
        pts = [np.zeros((1, 2))] + [geometry.polygon_exterior_vertices(p) for p in polys]
        return np.vstack(pts)[:-1]

    def initialize_manual(self, init_guess_path, obs, min_x=-9999999, min_y=-9999999, max_x=9999999,
                          max_y=9999999, init_control=None, init_dual_var=None):
        path = np.asarray(init_guess_path, dtype=np.float64)
        self.init_state = path[0, :5].copy()
        self.end_state = path[-1, :5].copy()
        self.N = len(path)
        self.obstacles = obs
        self.ref_state = path
        self.init_guess = path[:, :5].copy()
        self.init_control = None if init_control is None else np.asarray(init_control, dtype=np.float64)
        self.x0 = list(path[:, :5].reshape(-1))
        self.x0 += list(np.zeros(self.n_controls * (self.N - 1)) if init_control is None
                        else self.init_control.reshape(-1))
        self.obs_dual_ns = self.get_dual_variable_ns()
        self.obs_dual_n_all = int(np.sum(self.obs_dual_ns))
        dual_variable_num = self.obs_dual_n_all * self.N
        self.x0 += [0.1] * dual_variable_num
        self.min_x, self.min_y, self.max_x, self.max_y = min_x, min_y, max_x, max_y
        self.solution_found = False
        print("number of constraints for obstacle free: ", self.N * len(self.obstacles) * 2,
              "number of variables: ", (self.n_states + self.N + dual_variable_num))

    def get_dual_variable_ns(self):
        return [len(o) for o in self.obstacles]

    def build_model(self) -> bool:
        if self.N < 1:
            print("empty init guess")
            return False
        self.obj = 0
        return True

    def generate_object(self, r, q):
        """:193-227 (r, q are unused by the reference as well)."""
        self._r, self._q = r, q

    def generate_variable(self):
        """:229-255 bounds, in the reference's variable order."""
        for _ in range(self.N):
            self.lbx += [self.min_x, self.min_y, -self.MAX_VELOCITY, -2 * np.pi, -self.v_car.MAX_STEER]
            self.ubx += [self.max_x, self.max_y, self.MAX_VELOCITY, 2 * np.pi, self.v_car.MAX_STEER]
        for _ in range(self.N - 1):
            self.lbx += [-self.MAX_ACCEL, -self.MAX_STEER_RATE]
            self.ubx += [self.MAX_ACCEL, self.MAX_STEER_RATE]
        self.lbx += [0.0] * (self.obs_dual_n_all * self.N)
        self.ubx += [100000] * (self.obs_dual_n_all * self.N)

    def generate_constrain(self):
        """:257-327 bounds (start, Euler dynamics, hard end, per obstacle/step/vertex rows);
        the obstacle halfspaces replace pypoman's compute_polytope_halfspaces."""
        self.lbg += [0] * 5 * (self.N + 1)
        self.ubg += [0] * 5 * (self.N + 1)
        self._A, self._b = [], []
        for obstacle in self.obstacles:
            A, b = geometry.polytope_halfspaces(obstacle)
            if A.shape[0] != len(obstacle):
                raise ValueError("[OBCA points] obstacle must list its vertices once, without the closing vertex "
                                 f"({len(obstacle)} vertices but {A.shape[0]} halfspaces)")
            self._A.append(A)
            self._b.append(b)
            for _ in range(self.N * len(self.vertices)):
                self.lbg += [0, self.MIN_DISTANCE_TO_OBS]
                self.ubg += [1, 100000]

    # ---------------------------------------------------------------- solve
    def instance(self):
        """The prepared NLP as an oracle/nlp_points.py instance dict."""
        if not hasattr(self, "_A"):
            raise RuntimeError("[OBCA points] call generate_constrain() before solve()")
        inst = dict(init_traj=self.init_guess, obs_A=self._A, obs_b=self._b, vertices=np.asarray(self.vertices),
                    dT=float(self.dT), wheelbase=float(self.v_car.WHEEL_BASE), max_steer=float(self.v_car.MAX_STEER),
                    max_velocity=float(self.MAX_VELOCITY), max_accel=float(self.MAX_ACCEL),
                    max_steer_rate=float(self.MAX_STEER_RATE), min_dist=float(self.MIN_DISTANCE_TO_OBS),
                    x_bound=[float(self.min_x), float(self.max_x)], y_bound=[float(self.min_y), float(self.max_y)])
        if self.init_control is not None:
            inst["init_control"] = self.init_control
        return inst

    def _take(self, res, k):
        N, x = self.N, res.x[k]
        self.x_opt = _dm(x[0:5 * N:5])
        self.y_opt = _dm(x[1:5 * N:5])
        self.v_opt = _dm(x[2:5 * N:5])
        self.theta_opt = _dm(x[3:5 * N:5])
        self.steer_opt = _dm(x[4:5 * N:5])
        self.a_opt = _dm(x[5 * N:5 * N + 2 * (N - 1):2])
        self.steerate_opt = _dm(x[5 * N + 1:5 * N + 2 * (N - 1):2])
        self.lambda_opt = _dm(x[5 * N + 2 * (N - 1):])
        self.status = int(res.status[k])
        self.status_str = _native.STATUS_STR.get(self.status, str(self.status))
        self.objective = float(res.objective[k])
        self.iterations = int(res.iterations[k])
        self.solution_found = len(self.x_opt.elements()) > 0

    def solve(self):
        solve_batch([self])


def solve_batch(optimizers: List[OBCAOptimizer], device=0):
    """Solve prepared point-formulation optimizers in one HIP launch."""
    if not optimizers:
        return
    packed = _native.PointsPackedBatch([o.instance() for o in optimizers])
    ctx = _context(device)
    ctx.set_option("max_cpu_time", 0.0)  # optimizer_points.py:163 sets no CPU-time limit
    res = ctx.solve_points(packed)
    for k, o in enumerate(optimizers):
        o._take(res, k)
