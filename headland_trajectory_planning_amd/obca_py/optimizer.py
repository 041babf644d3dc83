"""Drop-in replacement for R/obca_py/optimizer.py (OBCAOptimizer).

Same constructor signature, attributes, `solve()` return value and solution
dict as the reference (R/obca_py/optimizer.py:77-138, :475-571), same
"[OBCA] ..." prints and the same exceptions on invalid input.  The NLP is not
built symbolically: it is packed into flat arrays and solved by the batched
HIP interior-point solver in libhtp.so (include/htp.h) -- the IPOPT algorithm
restated in oracle/ipm.py.  There is no CPU fallback: if the HIP library is
missing, construction of the solver context raises.

Batched use: `solve_batch([OBCAOptimizer, ...])` solves many problems in one
launch (they must share N, obstacle/body edge counts and time-opt).
"""
from typing import Any, Dict, List, Tuple

import numpy as np

from .. import _native, geometry

INF = float("inf")


class PolySet(object):
    """Polygon list + edge counts (optimizer.py:39-64)."""

    def __init__(self, poly_list: List) -> None:
        if not isinstance(poly_list, list):
            raise Exception("[OBCA] The input to PolySet should be a list!")
        if len(poly_list) < 1:
            print("[OBCA] The input to PolySet is empty.")
        self.poly_list = poly_list
        self.edge_counts = np.array([len(p) for p in poly_list], dtype=int)
        self.total_edges = int(self.edge_counts.sum()) if len(poly_list) else 0

    def __len__(self) -> int:
        return len(self.poly_list)

    def __getitem__(self, idx: int) -> Any:
        return self.poly_list[idx]


def kinematic_model(wheel_base: float):
    """Numpy form of the bicycle model of optimizer.py:9-36:
    f(state=[x, y, v, theta, steer], control=[accel, steer_rate])."""
    def f(state, control):
        x, y, v, th, de = state
        return np.array([v * np.cos(th), v * np.sin(th), control[0], v * np.tan(de) / wheel_base, control[1]])
    return f


_CTX = {}


def _context(device=0):
    if device not in _CTX:
        _CTX[device] = _native.Context(device)
    return _CTX[device]


class OBCAOptimizer(object):
    """The OBCA Optimizer (optimizer.py:67) on the MI355X solver."""

    DEFAULT_MAX_VELOCITY = 1.0  # m/s
    DEFAULT_MAX_ACCEL = 1.0  # m/s^2
    DEFAULT_MAX_STEER_RATE = 0.7  # rad/s
    DEFAULT_MIN_DISTANCE_TO_OBS = 0.1  # m

    def __init__(
        self,
        car,
        obstacles: List,
        init_traj: np.ndarray,
        enable_aux: bool = True,
        init_control: np.ndarray = None,
        init_dual_var: List = None,
        dT: float = 0.2,
        Q: np.ndarray = np.diag([1, 1]),
        R: np.ndarray = np.diag([0.1, 0.1]),
        W: np.ndarray = np.diag([5, 0]),
        x_bound: List = [-INF, INF],
        y_bound: List = [-INF, INF],
        max_velocity: float = DEFAULT_MAX_VELOCITY,
        max_accel: float = DEFAULT_MAX_ACCEL,
        max_steer_rate: float = DEFAULT_MAX_STEER_RATE,
        min_dist_to_obs: float = DEFAULT_MIN_DISTANCE_TO_OBS,
        device: int = 0,
    ) -> None:
        self.n_controls = 2
        self.n_states = 5
        self.dT = dT
        self.device = device
        W = np.asarray(W)
        self.enable_time_opt = False if W[1, 1] == 0 else True
        self.MIN_DISTANCE_TO_OBS = self.DEFAULT_MIN_DISTANCE_TO_OBS
        if min_dist_to_obs is not None:
            if min_dist_to_obs < 0:
                print("[OBCA] Minimum distance to obstacles cannot be negative! Use default value.")
            else:
                self.MIN_DISTANCE_TO_OBS = min_dist_to_obs
        self.set_vehicle_param(car, max_velocity, max_accel, max_steer_rate)
        self.set_x_y_boundary(x_bound, y_bound)
        self.generate_control_objects(car, enable_aux)
        self.generate_obstacles(obstacles)
        self.set_initial_guess(np.asarray(init_traj, dtype=np.float64), init_control, init_dual_var)
        self.generate_objective(np.asarray(Q, dtype=np.float64), np.asarray(R, dtype=np.float64), W.astype(np.float64))
        print("[OBCA] The solver has been successfully initialized!")

    # ----------------------------------------------------- setup (ref :140-290)
    def set_vehicle_param(self, car, max_velocity, max_accel, max_steer_rate) -> None:
        if car.WHEEL_BASE < 0:
            raise Exception("[OBCA] Wheelbase length should be a positive number!")
        self.WHEEL_BASE = car.WHEEL_BASE
        self.MAX_STEER = abs(car.MAX_STEER)
        self.MAX_VELOCITY = abs(max_velocity)
        self.MAX_ACCEL = abs(max_accel)
        self.MAX_STEER_RATE = abs(max_steer_rate)

    def generate_control_objects(self, car, enable_aux: bool) -> None:
        self.Gs, self.gs = self.get_polytopes_for_control_objects(car, enable_aux)

    def get_polytopes_for_control_objects(self, car, enable_aux: bool) -> Tuple[List, List]:
        control_objects = [car.car_poly]
        if enable_aux:
            if len(car.aux_polys) != 0:
                control_objects += list(car.aux_polys)
            else:
                print("[OBCA] Implements not found! Use empty car model by default.")
        verts = [geometry.polygon_exterior_vertices(p) for p in control_objects]
        self.control_objects = PolySet(verts)
        Gs, gs = [], []
        for v in verts:
            G, g = geometry.polytope_halfspaces(v)
            Gs.append(G)
            gs.append(g)
        return Gs, gs

    def generate_obstacles(self, obstacles: List) -> None:
        self.obstacles = PolySet(obstacles)
        self.As, self.bs = [], []
        for poly in obstacles:
            A, b = geometry.polytope_halfspaces(np.asarray(poly, dtype=np.float64))
            self.As.append(A)
            self.bs.append(b)

    def set_init_state(self, init_state) -> None:
        if init_state is None:
            raise Exception("[OBCA] Init state can not be Empty!")
        self.init_state = np.asarray(init_state)
        print("[OBCA] Init State = ", init_state)

    def set_end_state(self, end_state) -> None:
        if end_state is None:
            raise Exception("[OBCA] End state can not be Empty!")
        self.end_state = np.asarray(end_state)
        print("[OBCA] End State = ", end_state)

    def set_x_y_boundary(self, x_bound: List, y_bound: List) -> None:
        if x_bound[1] < x_bound[0]:
            raise Exception("[OBCA] The x_bound is infeasible!")
        if y_bound[1] < y_bound[0]:
            raise Exception("[OBCA] The y_bound is infeasible!")
        self.x_bound = x_bound
        self.y_bound = y_bound

    def set_initial_guess(self, init_traj, init_control, init_dual_var) -> None:
        self.N = len(init_traj)
        if self.N < 1:
            raise Exception("[OBCA] Initial guess is empty!")
        print("[OBCA] Prediction steps: ", self.N)
        if not self.enable_time_opt:
            self.horizon = (self.N - 1) * self.dT
            print("[OBCA] Prediction horizon: ", self.horizon)
        self.set_init_state(init_traj[0, :])
        self.set_end_state(init_traj[-1, :])
        self.init_traj = init_traj
        self.init_control = None
        if init_control is not None:
            init_control = np.asarray(init_control, dtype=np.float64)
            if init_control.shape[0] != self.N - 1 or init_control.shape[1] != self.n_controls:
                raise Exception("[OBCA] The control input dimension does not match!")
            self.init_control = init_control
        mu_count = self.control_objects.total_edges * len(self.obstacles)
        lambda_count = self.obstacles.total_edges * len(self.control_objects)
        self.init_mu = self.init_lambda = None
        if init_dual_var is not None:
            init_mu, init_lambda = np.asarray(init_dual_var[0]), np.asarray(init_dual_var[1])
            if (init_mu.shape[0] != self.N or init_mu.shape[1] != mu_count
                    or init_lambda.shape[0] != self.N or init_lambda.shape[1] != lambda_count):
                raise Exception("[OBCA] The dual variable dimension does not match!")
            self.init_mu, self.init_lambda = init_mu, init_lambda

    def generate_objective(self, Q, R, W) -> None:
        if len(Q) != self.n_controls:
            raise Exception("[OBCA] Weight_Q dimension does not match!")
        if len(R) != self.n_controls:
            raise Exception("[OBCA] Weight_R dimension does not match!")
        if len(W) != 2:
            raise Exception("[OBCA] Weight_W dimension does not match!")
        self.weight = {"Q": Q, "R": R, "W": W}

    # --------------------------------------------------------- batch packing
    def instance(self) -> Dict:
        return dict(
            init_traj=self.init_traj, obs_A=self.As, obs_b=self.bs, body_G=self.Gs, body_g=self.gs,
            dT=self.dT, Q=self.weight["Q"], R=self.weight["R"], W=self.weight["W"], wheelbase=self.WHEEL_BASE,
            max_steer=self.MAX_STEER, max_velocity=self.MAX_VELOCITY, max_accel=self.MAX_ACCEL,
            max_steer_rate=self.MAX_STEER_RATE, min_dist=self.MIN_DISTANCE_TO_OBS,
            x_bound=list(self.x_bound), y_bound=list(self.y_bound), init_control=self.init_control,
            init_mu=self.init_mu, init_lambda=self.init_lambda)

    def counts(self) -> Tuple[int, int, int]:
        eo = [len(p) for p in self.obstacles.poly_list]
        eb = [int(e) for e in self.control_objects.edge_counts]
        topt = int(self.enable_time_opt)
        N, M, K = self.N, len(eo), len(eb)
        n = 5 * N + 2 * (N - 1) + N * (sum(eb) * M + sum(eo) * K) + (N - 1) * topt + 5
        P = N * M * K
        return n, 5 * (N + 1) + 2 * P, 2 * P

    def _solution(self, x: np.ndarray, objective: float) -> Dict:
        N, ns, nc = self.N, self.n_states, self.n_controls
        mu_count = self.control_objects.total_edges * len(self.obstacles)
        lambda_count = self.obstacles.total_edges * len(self.control_objects)
        o_u = ns * N
        o_mu = o_u + nc * (N - 1)
        o_la = o_mu + mu_count * N
        o_t = o_la + lambda_count * N
        return {
            "dT": self.dT, "weight": self.weight,
            "x_opt": x[0:ns * N:ns].copy(), "y_opt": x[1:ns * N:ns].copy(), "v_opt": x[2:ns * N:ns].copy(),
            "theta_opt": x[3:ns * N:ns].copy(), "steer_angle_opt": x[4:ns * N:ns].copy(),
            "accel_opt": x[o_u:o_mu:nc].copy(), "steer_rate_opt": x[o_u + 1:o_mu:nc].copy(),
            "mu_opt": x[o_mu:o_la].reshape(N, mu_count).copy(),
            "lambda_opt": x[o_la:o_t].reshape(N, lambda_count).copy(),
            "time_scale_opt": (x[-5 - (N - 1):-5].copy() if self.enable_time_opt else np.ones(N - 1)),
            "slack_opt": x[-5:].copy(), "objective": float(objective),
        }

    # ------------------------------------------------------------- solve
    def solve(self, max_cpu_time=20, verbose: bool = False) -> Tuple[bool, Dict]:
        """optimizer.py:475-571.  max_cpu_time (IPOPT option, optimizer.py:486) limits
        the solve's time on the device clock; a solve that exceeds it stops with
        "Maximum_CpuTime_Exceeded" (success False)."""
        (success, solution), = solve_batch([self], verbose=verbose, max_cpu_time=max_cpu_time)
        return success, solution

    @staticmethod
    def show_slack(solution: Dict) -> None:
        s = solution["slack_opt"]
        print("x_slack = ", s[0])
        print("y_slack = ", s[1])
        print("v_slack = ", s[2])
        print("yaw_slack = ", s[3])
        print("steer_slack = ", s[4])

    @staticmethod
    def show_cost(solution: Dict) -> None:
        """optimizer.py:582-621 (slack printed x1000 exactly as the reference)."""
        objective = solution["objective"]
        dT = solution["dT"]
        v_opt, a, w = solution["v_opt"], solution["accel_opt"], solution["steer_rate_opt"]
        ts, s = solution["time_scale_opt"], solution["slack_opt"]
        Q, R, W = solution["weight"]["Q"], solution["weight"]["R"], solution["weight"]["W"]
        control_effort_cost = (a ** 2).sum() * Q[0, 0] + (w ** 2).sum() * Q[1, 1]
        jerk_cost = ((np.diff(a) / (dT * ts[:-1])) ** 2 * R[0, 0]).sum() + \
            ((np.diff(w) / (dT * ts[:-1])) ** 2 * R[1, 1]).sum()
        dist_cost = ((np.abs(v_opt[:-1]) * (dT * ts)) ** 2).sum() * W[0, 0]
        total_time_cost = (ts * dT).sum() * W[1, 1]
        slack_cost = (s ** 2 * 1000).sum()
        print("Total cost: ", objective)
        print("control effort cost: ", control_effort_cost)
        print("jerk cost: ", jerk_cost)
        print("path length cost: ", dist_cost)
        print("total time cost: ", total_time_cost)
        print("slack cost: ", slack_cost)


def solve_batch(optimizers: List[OBCAOptimizer], verbose: bool = False, device: int = None, max_cpu_time=None):
    """Solve many OBCAOptimizer problems in one HIP launch -> [(success, solution)].
    max_cpu_time (seconds, per problem, device clock; None/<= 0: no limit)."""
    if not optimizers:
        return []
    dev = optimizers[0].device if device is None else device
    ctx = _context(dev)
    ctx.set_option("max_cpu_time", float(max_cpu_time) if max_cpu_time else 0.0)
    pk = _native.PackedBatch([o.instance() for o in optimizers])
    res = ctx.solve(pk)
    out = []
    for k, o in enumerate(optimizers):
        n, neq, nin = o.counts()
        print("[OBCA] Number of decision variables: ", n)
        print("[OBCA] Number of equality constraints: ", neq)
        print("[OBCA] Number of inequality constraints: ", nin)
        print("[OBCA] EXIT: ", _native.STATUS_STR.get(int(res.status[k]), str(res.status[k])))
        if verbose:
            print(f"[OBCA] iterations {res.iterations[k]}, factorizations {res.n_factor[k]}, "
                  f"nlp error {res.nlp_error[k]:.3e}")
        out.append((bool(res.status[k] in (0, 1)), o._solution(res.x[k], res.objective[k])))
    return out
