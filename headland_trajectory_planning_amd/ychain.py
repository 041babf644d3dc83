"""The notebook planner chain as a batch on the device (htp_ypark_hastar_chain_device, csrc/htp_ychain.hip):
headland_planner_y_type_park of R/path_planner/headland_path_planning.py:124-255 -- Y-type parking search, the
ReferenceLineHeuristic lowering, the hybrid A* search to the parking start, get_init_ref_path -- for a batch of
row pairs, then the OBCA solve of the resampled init guess from the same device buffers.

Scenes: R/test/obca.ipynb cells 3-9 with randomised geometry (row spacing, slope, start row, offsets), the
notebook's car (empty_car) and planner arguments, kept when the forward Dubins turn of
headland_planner_y_type_park_combined (:55-121) is infeasible (the case the Y-park + hybrid A* chain exists for).
The scene data (rows, the side check's np.random draws, the lowered Y-park search, the search's static polygons)
is host input; everything that depends on a search result is computed on the device."""
import contextlib
import ctypes
import math

import numpy as np

from . import _native, geometry, synth

YP_ARGS = dict(max_steer_backward=0.15, max_steer_forward=0.55, max_backward_distance=3.0, max_forward_distance=2.0,
               min_forward_distance=1.0, min_backward_distance=1.0, min_steer_backward=0.0, min_steer_forward=0.5,
               step_size=0.2)          # R/test/obca.ipynb cell 9
DRIVE_ROW_OFFSET = 4.5                 # headland_planner_y_type_park's default
MAX_NODES = 400                        # hybrid_a_star_search(max_nodes=400), :213
DESIRED_V, DS = 0.5, 0.5 * 0.4         # get_init_ref_path(..., desired_v=0.5, ds=0.5 * 0.4), cell 13
POLY_STRIDE, VERT_STRIDE, MAXROWS = 10, 9 * 80, 32


class YChainBatch(ctypes.Structure):   # htp_ychain_batch
    _fields_ = [("batch", ctypes.c_int32), ("N", ctypes.c_int32),
                ("ypark", _native.YpBatch), ("ypark_out", _native.YpResult),
                ("hastar", _native.HaBatch), ("hastar_out", _native.HaResult),
                ("rows", ctypes.c_void_p), ("nrows", ctypes.c_void_p), ("eps", ctypes.c_void_p),
                ("start", ctypes.c_void_p), ("max_rows", ctypes.c_int32), ("drive_row_offset", ctypes.c_double),
                ("lane_poly0", ctypes.c_int32), ("lane_vert0", ctypes.c_int32), ("guide0", ctypes.c_int32),
                ("guide_stride", ctypes.c_int32), ("rp_params", ctypes.c_void_p), ("cap_rows", ctypes.c_int32),
                ("ref", ctypes.c_void_p), ("n_ref", ctypes.c_void_p), ("traj", ctypes.c_void_p),
                ("status", ctypes.c_void_p)]


def _declare(lib):
    if not hasattr(lib, "_yc_declared"):
        lib.htp_ypark_hastar_chain_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(YChainBatch), ctypes.c_void_p]
        lib.htp_ypark_hastar_chain_device.restype = ctypes.c_int
        lib.htp_ychain_last_ms.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.htp_ychain_last_ms.restype = ctypes.c_int
        lib._yc_declared = True
    return lib


def notebook_cars():
    from .path_planner.car_model import CarModel
    empty = CarModel(max_steer=0.55, axle_to_front=3, axle_to_back=0.55, width=1.48, with_aux=False)
    op = CarModel(max_steer=0.55, axle_to_back=0.55, width=1.48, aux_poly_features=[[[3.259, -0.175], 1.325, 0.3]],
                  with_aux=True)
    return empty, op


def make_scene(pid, key=20261017):
    """One row pair of the randomised notebook scene whose forward Dubins turn is infeasible."""
    from .path_planner import map_utils
    from .path_planner.OGE_OBCA import orchard_environment_OBCA
    from .path_planner.safety_forward_path_plan import get_dubins_path_full, get_offset_poses_for_row_traversing
    import copy
    rng = np.random.default_rng([key, pid])
    empty, _ = notebook_cars()
    for attempt in range(64):
        seed = int(rng.integers(1, 2 ** 31 - 1))
        row_w, slope = rng.uniform(2.3, 2.9), math.radians(rng.uniform(-12.0, 12.0))
        s_row = int(rng.integers(0, 4))
        leave, enter = rng.uniform(-1.5, -0.5), rng.uniform(3.0, 4.2)
        with synth._legacy_random(seed):
            rows = map_utils.create_tree_rows(8, row_w, 20, slope_angle=slope, l_std=0.0)
            env = orchard_environment_OBCA(rows, [], tree_width=0.3, headland_width=6.0)
        start = map_utils.get_base_pose(s_row, rows, leave, side=map_utils.NEAR_SIDE, pose_type=map_utils.LEAVE_POSE)
        end = map_utils.get_base_pose(s_row + 2, rows, enter, side=map_utils.NEAR_SIDE, pose_type=map_utils.ENTER_POSE)
        env_plan = copy.deepcopy(env)
        env_plan.update_tree_width(0.4)
        try:
            se, ee = get_offset_poses_for_row_traversing(start, end, empty, env_plan, max_steer_angle=0.5)
            fwd = get_dubins_path_full(se, ee, empty.get_turn_radius(max_steer_angle=None), step_size=0.2)
            if env_plan.check_path_feasibility(empty, fwd, boundary_check=True):
                continue                     # the combined planner would drive forward: not this chain's case
        except (ValueError, IndexError):
            pass
        scene = dict(pid=pid, seed=seed, rows=np.asarray(rows), env=env, start=np.asarray(start, float),
                     end=np.asarray(end, float), eps_seed=seed + 7)
        try:   # the notebook's OBCA obstacle builder raises (IndexError) when no boundary polygon flanks the turn
            obca_obstacles(scene, 6)
        except (IndexError, ValueError):
            continue
        return scene
    raise RuntimeError(f"[ychain] scene {pid}: no row pair needing the Y-park chain in 64 draws")


def eps_draws(scene):
    """check_side_of_a_point's np.random.uniform(-0.5, 0.5, rows) under the scene's seed (the host reference
    draws the same numbers: np.random.seed(eps_seed) before get_topology_waypoints)."""
    return np.random.RandomState(scene["eps_seed"]).uniform(-0.5, 0.5, size=(len(scene["rows"]),))


def lowered(scene):
    """The host-side (scene-only) inputs of one problem: the lowered Y-park search and the hybrid A* search's
    static part (body, blockers, field, motions, start, planner constants)."""
    from .path_planner import headland_path_planning as hpp
    from .path_planner import hybrid_a_star_search as has
    from .path_planner.geom import ring_of
    empty, _ = notebook_cars()
    env, start, end = scene["env"], scene["start"], scene["end"]
    bdir = hpp.get_backward_steer_dir_for_y_type_parking(start, end)
    yp = hpp.lower_ypark(empty, env, end, bdir, -bdir, **YP_ARGS)
    ha = dict(start=start[:3], goal=np.zeros(3), body=ring_of(empty.car_poly),
              blockers=[ring_of(p) for p in list(env.obstacle_polys) + list(env.tree_polys)],
              field=ring_of(env.field_range_poly), king=True, res=YP_ARGS["step_size"], yaw_res=math.radians(10),
              max_nodes=MAX_NODES, wheel_base=float(empty.WHEEL_BASE), max_steer=float(empty.MAX_STEER),
              curvature=math.tan(empty.MAX_STEER) / empty.WHEEL_BASE, default_search_length=1.5,
              motions=has.motion_steers(empty.MAX_STEER, math.radians(10), "King"))
    return yp, ha


def obca_obstacles(scene, M):
    """OBCA obstacles of the scene (the notebook's env.get_obstacles_for_OBCA, cell 14), split into quads; the M
    closest to the start and goal poses (scene data: picked before any search)."""
    env, start, end = scene["env"], scene["start"], scene["end"]
    with synth._legacy_random(scene["seed"] + 1):
        boundary = env.create_boundary_polygons()
    rows = env.get_obstacle_tree_rows(start, end)
    obs = env.get_obstacles_for_OBCA(boundary, rows, start, end, side=env.NEAR_SIDE)
    pool = [q for o in obs for q in synth._split_quads(o)]
    pts = np.array([start[:2], end[:2], 0.5 * (start[:2] + end[:2])])
    d = [float(np.min(np.hypot(q[:, None, 0] - pts[None, :, 0], q[:, None, 1] - pts[None, :, 1]))) for q in pool]
    keep = sorted(np.argsort(d, kind="stable")[:M])
    pool = [pool[k] for k in keep]
    k = 0
    while len(pool) < M:
        cx = start[0] + 60.0 + 5.0 * k
        pool.append(synth._rect(cx, cx + 1.0, start[1] + 60.0, start[1] + 61.0))
        k += 1
    return pool


def obca_instance(scene, traj, M=6):
    """One chain output as a host OBCA instance (oracle/nlp.py format): the notebook's operation car (its body and
    implement polygons, K = 2), the scene's M OBCA quads, synth's weights and limits."""
    from .path_planner.geom import ring_of
    _, op = notebook_cars()
    bodies = [ring_of(op.car_poly)] + [ring_of(p) for p in op.aux_polys]
    obs = obca_obstacles(scene, M)
    obs_A, obs_b = zip(*[geometry.polytope_halfspaces(o) for o in obs])
    body_G, body_g = zip(*[geometry.polytope_halfspaces(p) for p in bodies])
    w = synth.DEFAULT_WEIGHTS
    return dict(init_traj=np.asarray(traj, dtype=np.float64), obs_A=list(obs_A), obs_b=list(obs_b),
                body_G=list(body_G), body_g=list(body_g), obstacles=obs, dT=w["dT"], Q=w["Q"].copy(),
                R=w["R"].copy(), W=w["W"].copy(), wheelbase=float(op.WHEEL_BASE), max_steer=float(op.MAX_STEER),
                max_velocity=1.0, max_accel=1.0, max_steer_rate=0.7, min_dist=0.1,
                x_bound=[-np.inf, np.inf], y_bound=[-np.inf, np.inf])


class DeviceYChain:
    """Device buffers (torch) of one batch of the chain and of the OBCA solve of its output; build() enqueues the
    chain, obca_batch() describes the solve's inputs (the chain's traj + the scenes' obstacles, in HBM)."""

    def __init__(self, ctx, scenes, N=80, M=6, cap_rows=1024, guide_stride=2048, ha_cap_path=1024):
        import torch
        self.ctx, self.torch, self.N, self.M, self.B = ctx, torch, N, M, len(scenes)
        _declare(ctx.lib)
        dev = torch.device("cuda", ctx.device)
        self.dev = dev
        B = self.B
        lows = [lowered(s) for s in scenes]
        self.yp_pack = _native.YparkPacked([y for y, _ in lows], cap_path=256)
        # hybrid A* pools: the static polygons of every problem, then the reserved lane slots
        ha = [h for _, h in lows]
        placeholder = dict(lanes=[np.array([[0.0, 0.0], [1.0, 0.0], [0.0, 1.0]])], search_lengths=[1.5],
                           guide=np.zeros((1, 4)))
        pk = _native.HastarPacked([dict(h, **placeholder) for h in ha], cap_path=ha_cap_path, cap_log=0)
        npoly0, nvert0, nguide0 = len(pk.poly_off) - 1, pk.vertices.shape[0], pk.guide.shape[0]
        self.lane_poly0, self.lane_vert0, self.guide0 = npoly0, nvert0, nguide0
        poly_off = np.zeros(npoly0 + B * POLY_STRIDE + 1, np.int32)
        poly_off[:npoly0 + 1] = pk.poly_off
        slot_start = nvert0 + np.arange(B + 1) * VERT_STRIDE
        poly_off[npoly0 + np.arange(B + 1) * POLY_STRIDE] = slot_start
        vertices = np.zeros((nvert0 + B * VERT_STRIDE, 2))
        vertices[:nvert0] = pk.vertices
        lane_len = np.zeros(npoly0 + B * POLY_STRIDE)
        lane_len[:npoly0] = pk.lane_len
        guide = np.zeros((nguide0 + B * guide_stride, 4))
        guide[:nguide0] = pk.guide
        self.guide_stride = guide_stride
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
        self.ha_in = dict(params=t(pk.params), desc=t(pk.desc), poly_off=t(poly_off), vertices=t(vertices),
                          lane_len=t(lane_len), guide=t(guide), motions=t(pk.motions))
        self.yp_in = {k: t(getattr(self.yp_pack, k)) for k in ("params", "desc", "poly_off", "vertices", "axis")}
        rows = np.zeros((B, MAXROWS, 4))
        eps = np.zeros((B, MAXROWS))
        nrows = np.zeros(B, np.int32)
        for b, s in enumerate(scenes):
            r = np.asarray(s["rows"])
            rows[b, :len(r)] = r.reshape(len(r), 4)
            eps[b, :len(r)] = eps_draws(s)
            nrows[b] = len(r)
        _, op = notebook_cars()
        self.scene_in = dict(rows=t(rows), eps=t(eps), nrows=t(nrows), start=t(np.array([s["start"][:3] for s in scenes])),
                             rp_params=t(np.tile([op.WHEEL_BASE, DESIRED_V, DS], (B, 1))))
        z = lambda shape, dt=torch.float64: torch.zeros(shape, dtype=dt, device=dev)   # noqa: E731
        i32 = torch.int32
        self.yp_out = dict(status=z(B, i32), cand=z(B, i32), n_path=z(B, i32), params=z((B, 4)), n_pose=z(B, torch.int64),
                           path=z((B, 256, 5)))
        self.ha_out = dict(status=z(B, i32), counter=z(B, i32), n_path=z(B, i32), n_expanded=z(B, i32),
                           n_pose=z(B, torch.int64), x=z((B, ha_cap_path)), y=z((B, ha_cap_path)),
                           yaw=z((B, ha_cap_path)), dir=z((B, ha_cap_path)), k=z((B, ha_cap_path)))
        self.ref = z((B, cap_rows, 5))
        self.n_ref = z(B, i32)
        self.traj = z((B, N, 5))
        self.status = z(B, i32)
        yb = self.yp_pack.struct({k: v.data_ptr() for k, v in self.yp_in.items()})
        hb = pk.struct({k: v.data_ptr() for k, v in self.ha_in.items()})
        hb.npoly, hb.nvert, hb.nguide = len(poly_off) - 1, vertices.shape[0], guide.shape[0]
        yr = _native.YpResult()
        for k, v in self.yp_out.items():
            setattr(yr, k, v.data_ptr())
        hr = _native.HaResult()
        for k, v in self.ha_out.items():
            setattr(hr, k, v.data_ptr())
        hr.expanded = None
        cb = YChainBatch()
        cb.batch, cb.N = B, N
        cb.ypark, cb.ypark_out, cb.hastar, cb.hastar_out = yb, yr, hb, hr
        cb.rows, cb.nrows, cb.eps = (self.scene_in[k].data_ptr() for k in ("rows", "nrows", "eps"))
        cb.start, cb.rp_params = self.scene_in["start"].data_ptr(), self.scene_in["rp_params"].data_ptr()
        cb.max_rows, cb.drive_row_offset = MAXROWS, DRIVE_ROW_OFFSET
        cb.lane_poly0, cb.lane_vert0, cb.guide0, cb.guide_stride = npoly0, nvert0, nguide0, guide_stride
        cb.cap_rows = cap_rows
        cb.ref, cb.n_ref, cb.traj, cb.status = (getattr(self, k).data_ptr() for k in ("ref", "n_ref", "traj", "status"))
        self.cb = cb
        # the OBCA solve's scene inputs (obstacles picked from the scene before any search; K = 2 bodies)
        tmpl = [obca_instance(s, np.zeros((N, 5)), M) for s in scenes]
        if any(a.shape[0] != 4 for it in tmpl for a in it["obs_A"]):
            raise ValueError("[ychain] OBCA obstacles must be quads")
        self.obs_A = t(np.array([np.concatenate(it["obs_A"]) for it in tmpl]))
        self.obs_b = t(np.array([np.concatenate(it["obs_b"]) for it in tmpl]))
        self.body_G = t(np.array([np.concatenate(it["body_G"]) for it in tmpl]))
        self.body_g = t(np.array([np.concatenate(it["body_g"]) for it in tmpl]))
        self.params = t(np.array([_native.params_of(it) for it in tmpl]))
        self.K = len(tmpl[0]["body_G"])
        self.body_edges = np.array([a.shape[0] for a in tmpl[0]["body_G"]], np.int32)
        self.obs_edges = np.full(M, 4, np.int32)
        self.time_opt = int(np.asarray(tmpl[0]["W"])[1, 1] != 0)
        self.templates = tmpl

    def obca_batch(self):
        """htp_obca_batch over the chain's traj and the scenes' obstacles (device pointers)."""
        b = _native.ObcaBatch()
        b.batch, b.N, b.M, b.K, b.time_opt = self.B, self.N, self.M, self.K, self.time_opt
        b.obs_edges, b.body_edges = self.obs_edges.ctypes.data, self.body_edges.ctypes.data
        b.traj, b.obs_A, b.obs_b = self.traj.data_ptr(), self.obs_A.data_ptr(), self.obs_b.data_ptr()
        b.body_G, b.body_g, b.params = self.body_G.data_ptr(), self.body_g.data_ptr(), self.params.data_ptr()
        b.init_control = b.init_mu = b.init_lambda = None
        return b

    def struct(self, ptrs=None):
        """PackedBatch-style hook for the persistent launch (Context.solve_queue_device)."""
        return self.obca_batch()

    def build(self, stream=None):
        s = stream or self.torch.cuda.current_stream(self.dev)
        if self.ctx.lib.htp_ypark_hastar_chain_device(self.ctx.ctx, ctypes.byref(self.cb), ctypes.c_void_p(s.cuda_stream)):
            raise RuntimeError(f"[htp] htp_ypark_hastar_chain_device failed: {self.ctx.error()}")

    def stage_ms(self):
        ms = np.zeros(4)
        if self.ctx.lib.htp_ychain_last_ms(self.ctx.ctx, ms.ctypes.data) != 0:
            raise RuntimeError("[htp] htp_ychain_last_ms failed")
        return dict(zip(("ypark", "lower", "hastar", "init_guess"), ms.tolist()))

    def lanes(self, b):
        """The device-lowered heuristic of problem b: (lane rings, search lengths, guide rows)."""
        d = self.ha_in["desc"][b].cpu().numpy()
        po = self.ha_in["poly_off"].cpu().numpy()
        v = self.ha_in["vertices"].cpu().numpy()
        ll = self.ha_in["lane_len"].cpu().numpy()
        g = self.ha_in["guide"].cpu().numpy()
        rings = [v[po[p]:po[p + 1]] for p in range(d[_native.HA_D_LANE0], d[_native.HA_D_LANE1])]
        return rings, ll[d[_native.HA_D_LANE0]:d[_native.HA_D_LANE1]], g[d[_native.HA_D_GUIDE0]:d[_native.HA_D_GUIDE1]]


def host_reference(scene, ypark_runner, hastar_runner, N=80):
    """The same chain on the host: the restated reference planner steps (path_planner/) with the given search
    runners (host builds in the CPU tests, the GPU searches otherwise) -> dict(status, heuristic, path, ref, traj)."""
    from .obca_py.util import get_init_ref_path
    from .path_planner import hybrid_a_star_search as has
    from .path_planner.reference_line_heuristic import ReferenceLineHeuristic
    empty, op = notebook_cars()
    yp, ha = lowered(scene)
    y = ypark_runner([yp])[0]
    if y["status"] != 0:
        return dict(status=16 + y["status"])
    y_path = np.asarray(y["path"])
    inter = y_path[0][:3]
    env = scene["env"]
    with synth._legacy_random(scene["eps_seed"]):
        wps = env.get_topology_waypoints(scene["start"], inter, drive_row_offset=DRIVE_ROW_OFFSET)
    heur = ReferenceLineHeuristic(wps, inter, empty)
    prob = has.lower_problem(scene["start"], inter, env, empty, heur, motion_type="King",
                             plan_resolution=YP_ARGS["step_size"], max_nodes=MAX_NODES)
    h = hastar_runner([prob])[0]
    out = dict(heuristic=heur, waypoints=np.asarray(wps), prob=prob, hastar=h, ypark=y)
    if h["status"] != 0:
        out["status"] = 48 + h["status"]
        return out
    xs = np.concatenate([h["xs"], y_path[:, 0]])
    ys = np.concatenate([h["ys"], y_path[:, 1]])
    yaws = np.concatenate([h["yaws"], y_path[:, 2]])
    ks = np.concatenate([h["ks"], y_path[:, 3]])
    dirs = np.concatenate([h["dirs"], y_path[:, 4]])
    ref = get_init_ref_path(op, xs, ys, yaws, ks, dirs, desired_v=DESIRED_V, ds=DS)
    out.update(status=0, ref=ref, traj=synth._resample_rows(ref, N))
    return out


def cpu_lower(scene, goal):
    """The chain's lowering core (csrc/ychain_core.h) through its host build (libhtp_cpu.so) for one problem ->
    dict(waypoints, guide, lanes, lengths) or the core's status."""
    lib = _native.cpu_lib()
    f = lib.htp_cpu_ychain_lower
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double,
                  ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    rows = np.ascontiguousarray(np.asarray(scene["rows"], dtype=np.float64).reshape(-1, 4))
    eps = np.ascontiguousarray(eps_draws(scene))
    start = np.ascontiguousarray(scene["start"][:3], dtype=np.float64)
    goal = np.ascontiguousarray(goal[:3], dtype=np.float64)
    wp, nwp = np.zeros((10, 2)), np.zeros(1, np.int32)
    guide, ng = np.zeros((4096, 4)), np.zeros(1, np.int32)
    rings, nring, lengths = np.zeros((9, 80, 2)), np.zeros(9, np.int32), np.zeros(9)
    rc = f(rows.ctypes.data, rows.shape[0], eps.ctypes.data, start.ctypes.data, goal.ctypes.data, DRIVE_ROW_OFFSET,
           1.5, wp.ctypes.data, nwp.ctypes.data, guide.ctypes.data, guide.shape[0], ng.ctypes.data, rings.ctypes.data,
           nring.ctypes.data, lengths.ctypes.data)
    if rc != 0:
        return dict(status=rc)
    n = int(nwp[0])
    return dict(status=0, waypoints=wp[:n], guide=guide[:int(ng[0])],
                lanes=[rings[k, :nring[k]] for k in range(n - 1)], lengths=lengths[:n - 1])


def run_bench(scenes, steps, warmup, max_cpu_time=20.0, device=0):
    """Time `steps` passes of the whole chain + the OBCA solve of its output over `scenes`, one batch per step on
    one stream (the chain's four launches, then one htp_obca_solve_batch_device launch).  Per-stage times from
    the chain's own HIP events (htp_ychain_last_ms) and an event pair around the solve."""
    import time

    import torch

    from . import e2e
    ctx = _native.Context(device)
    ctx.set_option("max_cpu_time", max_cpu_time)
    ch = DeviceYChain(ctx, scenes)
    n_var = _native.PackedBatch([ch.templates[0]]).n_var
    outs = e2e.solve_outputs(torch, ch.dev, ch.B, n_var)
    stream = torch.cuda.Stream(ch.dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def step():
        ch.build(stream)
        ev[0].record(stream)
        e2e.solve_chain(ctx, ch, outs, stream)
        ev[1].record(stream)
        stream.synchronize()
        return ch.stage_ms(), ev[0].elapsed_time(ev[1])

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(ch.dev)
    stages, solve_ms = {}, 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        sm, so = step()
        for k, v in sm.items():
            stages[k] = stages.get(k, 0.0) + v / steps
        solve_ms += so / steps
    elapsed = time.perf_counter() - t0
    cst, st = ch.status.cpu().numpy(), outs["status"].cpu().numpy()
    ok = (cst == 0) & np.isin(st, [0, 1])
    hist = lambda a: {str(k): int(v) for k, v in zip(*np.unique(a, return_counts=True))}   # noqa: E731
    return dict(value=steps * ch.B / elapsed, ms_per_step=1e3 * elapsed / steps, batch=ch.B, stage_ms=stages,
                solve_ms=solve_ms, chain_status=hist(cst), solve_status=hist(st), success_rate=float(ok.mean()),
                mean_iters=float(outs["iterations"].cpu().numpy().mean()))
