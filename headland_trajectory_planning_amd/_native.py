"""ctypes binding of libhtp.so (include/htp.h) and batch packing.

The product path REQUIRES the in-tree HIP library: `load()` raises if it is
missing -- there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libhtp.so")
NPARAM = 24
(P_DT, P_Q00, P_Q01, P_Q10, P_Q11, P_R00, P_R01, P_R10, P_R11, P_W00, P_W11, P_WHEELBASE, P_MAXSTEER,
 P_MAXV, P_MAXACC, P_MAXSR, P_DMIN, P_XLO, P_XHI, P_YLO, P_YHI, P_HAS_INIT_CONTROL, P_HAS_INIT_DUAL) = range(23)

STATUS_STR = {0: "Solve_Succeeded", 1: "Solved_To_Acceptable_Level", 2: "Maximum_Iterations_Exceeded",
              3: "Restoration_Failed", 4: "Error_In_Step_Computation", 5: "Invalid_Problem_Definition",
              6: "Maximum_CpuTime_Exceeded", 7: "Infeasible_Problem_Detected", 8: "Search_Direction_Becomes_Too_Small"}

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


class ObcaBatch(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("N", ctypes.c_int32), ("M", ctypes.c_int32), ("K", ctypes.c_int32),
                ("time_opt", ctypes.c_int32), ("obs_edges", ctypes.c_void_p), ("body_edges", ctypes.c_void_p),
                ("traj", ctypes.c_void_p), ("obs_A", ctypes.c_void_p), ("obs_b", ctypes.c_void_p),
                ("body_G", ctypes.c_void_p), ("body_g", ctypes.c_void_p), ("params", ctypes.c_void_p),
                ("init_control", ctypes.c_void_p), ("init_mu", ctypes.c_void_p), ("init_lambda", ctypes.c_void_p)]


class ObcaResult(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("objective", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("iterations", ctypes.c_void_p), ("n_factor", ctypes.c_void_p), ("nlp_error", ctypes.c_void_p),
                ("n_resto", ctypes.c_void_p)]


class RsPaths(ctypes.Structure):
    _fields_ = [("cap_paths", ctypes.c_int64), ("cap_points", ctypes.c_int64), ("n_paths", ctypes.c_int64),
                ("n_points", ctypes.c_int64)] + [(n, ctypes.c_void_p) for n in (
                    "path_offsets", "status", "lengths", "ctypes", "L", "point_offsets", "x", "y", "yaw", "cs",
                    "directions")]


class HaBatch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("batch", "npoly", "nvert", "nguide", "nmotion")] + \
        [(n, ctypes.c_void_p) for n in ("params", "desc", "poly_off", "vertices", "lane_len", "guide", "motions")] + \
        [(n, ctypes.c_int32) for n in ("max_nodes_cap", "cap_path", "cap_log")]


class HaResult(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("status", "counter", "n_path", "n_expanded", "n_pose", "x", "y", "yaw",
                                               "dir", "k", "expanded")]


class YpBatch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("batch", "npoly", "nvert", "naxis")] + \
        [(n, ctypes.c_void_p) for n in ("params", "desc", "poly_off", "vertices", "axis")] + [("cap_path", ctypes.c_int32)]


class YpResult(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("status", "cand", "n_path", "params", "n_pose", "path")]


YP_NPARAM, YP_NDESC = 16, 12
(YP_P_EX, YP_P_EY, YP_P_EYAW, YP_P_BDIR, YP_P_FDIR, YP_P_WB, YP_P_STEP, YP_P_R00, YP_P_R01, YP_P_R10, YP_P_R11,
 YP_P_TX, YP_P_TY, YP_P_YAW_ODOM) = range(14)
YP_STATUS = {0: "found", 1: "none", 2: "end_blocked", 3: "bad_input"}
YP_STATUS_BY_NAME = {v: k for k, v in YP_STATUS.items()}

HA_NPARAM, HA_NDESC = 16, 12
(HA_P_SX, HA_P_SY, HA_P_SYAW, HA_P_GX, HA_P_GY, HA_P_GYAW, HA_P_RES, HA_P_YAWRES, HA_P_WB, HA_P_MAXSTEER,
 HA_P_CURV, HA_P_DEFLEN, HA_P_MAXNODES) = range(13)
(HA_D_BODY, HA_D_BLK0, HA_D_BLK1, HA_D_LANE0, HA_D_LANE1, HA_D_FIELD, HA_D_GUIDE0, HA_D_GUIDE1, HA_D_MOT0,
 HA_D_MOT1, HA_D_KING) = range(11)
HA_STATUS = {0: "found", 1: "no_path", 2: "max_nodes", 3: "start_goal_blocked", 4: "rs_error", 5: "capacity",
             6: "bad_input", 7: "backtrack_error"}

RS_OK, RS_ASSERT, RS_OVERFLOW, RS_CAPACITY = 0, 1, 2, 3
RS_SEG = "LSR"  # HTP_RS_SEG_L / _S / _R


EXPORTS = ["htp_obca_sizes", "htp_create", "htp_destroy", "htp_last_error", "htp_set_option",
           "htp_obca_solve_batch", "htp_obca_solve_batch_device", "htp_last_kernel_ms", "htp_last_cycles",
           "htp_rs_all_paths_batch", "htp_rs_all_paths_batch_device", "htp_rs_last_ms",
           "htp_hastar_search_batch", "htp_hastar_search_batch_device", "htp_hastar_last_ms",
           "htp_ypark_search_batch", "htp_ypark_search_batch_device", "htp_ypark_last_ms",
           "htp_obca_points_sizes", "htp_obca_points_solve_batch", "htp_obca_points_solve_batch_device",
           "htp_init_ref_path_batch", "htp_init_ref_path_batch_device", "htp_init_ref_path_last_ms",
           "htp_queue_create", "htp_queue_destroy", "htp_queue_publish", "htp_queue_close", "htp_queue_published",
           "htp_queue_claimed", "htp_obca_solve_queue_device", "htp_obca_resident_waves",
           "htp_oge_obstacles_batch", "htp_oge_obstacles_batch_device", "htp_oge_last_ms",
           "htp_classic_turn_batch", "htp_classic_turn_batch_device", "htp_classic_last_ms",
           "htp_orchard_chain_device", "htp_chain_last_ms"]


def _declare(lib):
    lib.htp_obca_sizes.argtypes = [ctypes.c_int32] * 4 + [ctypes.c_void_p] * 2 + [ctypes.POINTER(ctypes.c_int64)] * 4
    lib.htp_obca_sizes.restype = ctypes.c_int
    lib.htp_create.argtypes = [ctypes.c_int32]
    lib.htp_create.restype = ctypes.c_void_p
    lib.htp_destroy.argtypes = [ctypes.c_void_p]
    lib.htp_destroy.restype = None
    lib.htp_last_error.argtypes = [ctypes.c_void_p]
    lib.htp_last_error.restype = ctypes.c_char_p
    lib.htp_set_option.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_double]
    lib.htp_set_option.restype = ctypes.c_int
    lib.htp_obca_solve_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ObcaBatch), ctypes.POINTER(ObcaResult)]
    lib.htp_obca_solve_batch.restype = ctypes.c_int
    lib.htp_obca_solve_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ObcaBatch),
                                                ctypes.POINTER(ObcaResult), ctypes.c_void_p]
    lib.htp_obca_solve_batch_device.restype = ctypes.c_int
    lib.htp_init_ref_path_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(RpBatch), ctypes.POINTER(RpResult)]
    lib.htp_init_ref_path_batch.restype = ctypes.c_int
    lib.htp_init_ref_path_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(RpBatch), ctypes.POINTER(RpResult),
                                                   ctypes.c_void_p]
    lib.htp_init_ref_path_batch_device.restype = ctypes.c_int
    lib.htp_init_ref_path_last_ms.argtypes = [ctypes.c_void_p]
    lib.htp_init_ref_path_last_ms.restype = ctypes.c_double
    lib.htp_obca_points_sizes.argtypes = [ctypes.c_int32] * 3 + [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int64)] * 4
    lib.htp_obca_points_sizes.restype = ctypes.c_int
    lib.htp_obca_points_solve_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ObcaPointsBatch),
                                                ctypes.POINTER(ObcaResult)]
    lib.htp_obca_points_solve_batch.restype = ctypes.c_int
    lib.htp_obca_points_solve_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ObcaPointsBatch),
                                                       ctypes.POINTER(ObcaResult), ctypes.c_void_p]
    lib.htp_obca_points_solve_batch_device.restype = ctypes.c_int
    lib.htp_last_kernel_ms.argtypes = [ctypes.c_void_p]
    lib.htp_last_kernel_ms.restype = ctypes.c_double
    lib.htp_last_cycles.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
    lib.htp_last_cycles.restype = ctypes.c_int
    lib.htp_rs_all_paths_batch.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(RsPaths)]
    lib.htp_rs_all_paths_batch.restype = ctypes.c_int
    lib.htp_rs_all_paths_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                                  ctypes.POINTER(RsPaths), ctypes.c_void_p, ctypes.c_void_p]
    lib.htp_rs_all_paths_batch_device.restype = ctypes.c_int
    lib.htp_rs_last_ms.argtypes = [ctypes.c_void_p]
    lib.htp_rs_last_ms.restype = ctypes.c_double
    lib.htp_hastar_search_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(HaBatch), ctypes.POINTER(HaResult)]
    lib.htp_hastar_search_batch.restype = ctypes.c_int
    lib.htp_hastar_search_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(HaBatch), ctypes.POINTER(HaResult),
                                                   ctypes.c_void_p]
    lib.htp_hastar_search_batch_device.restype = ctypes.c_int
    lib.htp_hastar_last_ms.argtypes = [ctypes.c_void_p]
    lib.htp_hastar_last_ms.restype = ctypes.c_double
    lib.htp_ypark_search_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(YpBatch), ctypes.POINTER(YpResult)]
    lib.htp_ypark_search_batch.restype = ctypes.c_int
    lib.htp_ypark_search_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(YpBatch), ctypes.POINTER(YpResult),
                                                  ctypes.c_void_p]
    lib.htp_ypark_search_batch_device.restype = ctypes.c_int
    lib.htp_ypark_last_ms.argtypes = [ctypes.c_void_p]
    lib.htp_ypark_last_ms.restype = ctypes.c_double
    lib.htp_queue_create.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    lib.htp_queue_create.restype = ctypes.c_void_p
    lib.htp_queue_destroy.argtypes = [ctypes.c_void_p]
    lib.htp_queue_destroy.restype = None
    lib.htp_queue_publish.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    lib.htp_queue_publish.restype = ctypes.c_int
    lib.htp_queue_close.argtypes = [ctypes.c_void_p]
    lib.htp_queue_close.restype = ctypes.c_int
    lib.htp_queue_published.argtypes = [ctypes.c_void_p]
    lib.htp_queue_published.restype = ctypes.c_int64
    lib.htp_queue_claimed.argtypes = [ctypes.c_void_p]
    lib.htp_queue_claimed.restype = ctypes.c_int64
    lib.htp_obca_solve_queue_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ObcaBatch), ctypes.c_void_p,
                                                ctypes.POINTER(ObcaResult), ctypes.c_void_p, ctypes.c_int32,
                                                ctypes.c_double]
    lib.htp_obca_solve_queue_device.restype = ctypes.c_int
    lib.htp_obca_resident_waves.argtypes = [ctypes.c_void_p, ctypes.POINTER(ObcaBatch)]
    lib.htp_obca_resident_waves.restype = ctypes.c_int32
    lib.htp_oge_obstacles_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(OgeBatch), ctypes.POINTER(OgeResult)]
    lib.htp_oge_obstacles_batch.restype = ctypes.c_int
    lib.htp_oge_obstacles_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(OgeBatch),
                                                   ctypes.POINTER(OgeResult), ctypes.c_void_p]
    lib.htp_oge_obstacles_batch_device.restype = ctypes.c_int
    lib.htp_oge_last_ms.argtypes = [ctypes.c_void_p]
    lib.htp_oge_last_ms.restype = ctypes.c_double
    lib.htp_classic_turn_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(CtBatch), ctypes.POINTER(CtResult)]
    lib.htp_classic_turn_batch.restype = ctypes.c_int
    lib.htp_classic_turn_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(CtBatch), ctypes.POINTER(CtResult),
                                                  ctypes.c_void_p]
    lib.htp_classic_turn_batch_device.restype = ctypes.c_int
    lib.htp_classic_last_ms.argtypes = [ctypes.c_void_p]
    lib.htp_classic_last_ms.restype = ctypes.c_double
    lib.htp_orchard_chain_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ChainBatch), ctypes.c_void_p]
    lib.htp_orchard_chain_device.restype = ctypes.c_int
    lib.htp_chain_last_ms.argtypes = [ctypes.c_void_p]
    lib.htp_chain_last_ms.restype = ctypes.c_double
    lib.htp_libm_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_int32] + [ctypes.c_void_p] * 3 + \
        [ctypes.c_int64, ctypes.c_void_p]
    lib.htp_libm_batch_device.restype = ctypes.c_int
    if hasattr(lib, "htp_mfma_f64_probe"):   # absent from libraries built before it (A/B variants of old kernels)
        lib.htp_mfma_f64_probe.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_void_p]
        lib.htp_mfma_f64_probe.restype = ctypes.c_int
    return lib


# correctly rounded libm of the planner cores (csrc/htp_libm.h): function ids of htp_libm_batch_device
LIBM_FN = {"sin": 0, "cos": 1, "tan": 2, "atan": 3, "atan2": 4, "asin": 5, "acos": 6, "hypot": 7, "pow": 8, "log": 9,
           "fast_log": 10, "fast_sin": 11, "fast_cos": 12, "fast_tan": 13}
LIBM_BINARY = {"atan2", "hypot", "pow"}
CPU_LIB_PATH = os.path.join(HERE, "libhtp_cpu.so")
_CPU_LIB = None


def cpu_lib():
    """libhtp_cpu.so: the g++ build of the same cores (CPU baseline, workload generator, host twins)."""
    global _CPU_LIB
    if _CPU_LIB is None:
        if not os.path.exists(CPU_LIB_PATH):
            raise RuntimeError(f"[htp] CPU library not built: {CPU_LIB_PATH} (run __graft_entry__.build())")
        lib = ctypes.CDLL(CPU_LIB_PATH)
        lib.htp_cpu_libm_batch.argtypes = [ctypes.c_int32] + [ctypes.c_void_p] * 3 + [ctypes.c_int64]
        lib.htp_cpu_libm_batch.restype = ctypes.c_int
        _CPU_LIB = lib
    return _CPU_LIB


def cpu_libm(name, x, y=None):
    """Host build of the planner libm: name in LIBM_FN, x (and y) float64 arrays -> float64 array."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    yy = np.ascontiguousarray(np.broadcast_to(y, x.shape), dtype=np.float64) if y is not None else None
    if name in LIBM_BINARY and yy is None:
        raise ValueError(f"[htp] {name} needs two arguments")
    out = np.empty_like(x)
    rc = cpu_lib().htp_cpu_libm_batch(LIBM_FN[name], x.ctypes.data, yy.ctypes.data if yy is not None else None,
                                      out.ctypes.data, x.size)
    if rc != 0:
        raise RuntimeError("[htp] htp_cpu_libm_batch failed")
    return out


_LIB = None


def core_sha():
    """Short hash of the OBCA solver sources (ties profiles/*_traffic.json to a solver version)."""
    import hashlib
    h = hashlib.sha256()
    for f in ("obca_core.h", "htp_common.h", "htp_obca.hip", "dyn_gen.h", "wave_ctx.h", "htp_fastm.h", "htp_libm.h"):
        with open(os.path.join(HERE, "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def load(path=LIB_PATH):
    """Load the in-tree HIP library; raise loudly if it is absent."""
    global _LIB
    if _LIB is not None and path == LIB_PATH:
        return _LIB
    if not os.path.exists(path):
        raise RuntimeError(f"[htp] HIP library not built: {path} (run __graft_entry__.build())")
    # torch wheels bundle their own libamdhip64.so.7 (same SONAME as /opt/rocm's).
    # Whichever is loaded first serves the whole process; loading torch's first
    # keeps torch.cuda working when callers import torch after this library.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = _declare(ctypes.CDLL(path))
    if path == LIB_PATH:
        _LIB = lib
    return lib


def sizes(N, M, K, time_opt, obs_edges, body_edges, lib=None):
    lib = lib or load()
    eo = np.ascontiguousarray(obs_edges, dtype=np.int32)
    eb = np.ascontiguousarray(body_edges, dtype=np.int32)
    out = [ctypes.c_int64() for _ in range(4)]
    rc = lib.htp_obca_sizes(N, M, K, int(time_opt), eo.ctypes.data, eb.ctypes.data, *[ctypes.byref(v) for v in out])
    if rc != 0:
        raise ValueError("[OBCA] invalid problem shape")
    return tuple(v.value for v in out)


# ------------------------------------------------------------------ packing
def params_of(inst):
    p = np.zeros(NPARAM)
    Q, R, W = (np.asarray(inst[k], dtype=np.float64) for k in ("Q", "R", "W"))
    p[P_DT] = inst["dT"]
    p[P_Q00:P_Q11 + 1] = Q.reshape(-1)[:4]
    p[P_R00:P_R11 + 1] = R.reshape(-1)[:4]
    p[P_W00], p[P_W11] = W[0, 0], W[1, 1]
    p[P_WHEELBASE] = inst["wheelbase"]
    p[P_MAXSTEER] = inst["max_steer"]
    p[P_MAXV] = inst["max_velocity"]
    p[P_MAXACC] = inst["max_accel"]
    p[P_MAXSR] = inst["max_steer_rate"]
    dmin = inst.get("min_dist", 0.1)
    p[P_DMIN] = 0.1 if (dmin is None or dmin < 0) else dmin
    xb = inst.get("x_bound", [-np.inf, np.inf])
    yb = inst.get("y_bound", [-np.inf, np.inf])
    p[P_XLO], p[P_XHI], p[P_YLO], p[P_YHI] = xb[0], xb[1], yb[0], yb[1]
    p[P_HAS_INIT_CONTROL] = inst.get("init_control") is not None
    p[P_HAS_INIT_DUAL] = inst.get("init_mu") is not None
    return p


class PackedBatch:
    """Contiguous problem-major arrays for one batch (shared shape)."""

    def __init__(self, insts):
        i0 = insts[0]
        self.batch = len(insts)
        self.N = int(np.asarray(i0["init_traj"]).shape[0])
        self.M = len(i0["obs_A"])
        self.K = len(i0["body_G"])
        self.time_opt = int(np.asarray(i0["W"])[1, 1] != 0)
        self.obs_edges = np.array([a.shape[0] for a in i0["obs_A"]], dtype=np.int32)
        self.body_edges = np.array([a.shape[0] for a in i0["body_G"]], dtype=np.int32)
        for it in insts:
            if (np.asarray(it["init_traj"]).shape[0] != self.N
                    or [a.shape[0] for a in it["obs_A"]] != list(self.obs_edges)
                    or [a.shape[0] for a in it["body_G"]] != list(self.body_edges)
                    or int(np.asarray(it["W"])[1, 1] != 0) != self.time_opt):
                raise ValueError("[OBCA] all problems of a batch must share N, edge counts and time_opt")
        B = self.batch
        self.traj = np.ascontiguousarray(np.stack([np.asarray(it["init_traj"], dtype=np.float64) for it in insts]))
        self.obs_A = np.ascontiguousarray(np.stack([np.concatenate(it["obs_A"], axis=0) for it in insts]))
        self.obs_b = np.ascontiguousarray(np.stack([np.concatenate(it["obs_b"]) for it in insts]))
        self.body_G = np.ascontiguousarray(np.stack([np.concatenate(it["body_G"], axis=0) for it in insts]))
        self.body_g = np.ascontiguousarray(np.stack([np.concatenate(it["body_g"]) for it in insts]))
        self.params = np.ascontiguousarray(np.stack([params_of(it) for it in insts]))
        self.init_control = self._opt(insts, "init_control")
        self.init_mu = self._opt(insts, "init_mu")
        self.init_lambda = self._opt(insts, "init_lambda")
        TEo, TEb = int(self.obs_edges.sum()), int(self.body_edges.sum())
        self.mu_count, self.lam_count = TEb * self.M, TEo * self.K
        self.n_var = 5 * self.N + 2 * (self.N - 1) + self.N * (self.mu_count + self.lam_count) + \
            (self.N - 1) * self.time_opt + 5
        _ = B

    @staticmethod
    def _opt(insts, key):
        vals = [it.get(key) for it in insts]
        if all(v is None for v in vals):
            return None
        if any(v is None for v in vals):
            raise ValueError(f"[OBCA] {key} must be given for all or none of the problems")
        return np.ascontiguousarray(np.stack([np.asarray(v, dtype=np.float64) for v in vals]))

    def struct(self, ptrs=None):
        """ctypes htp_obca_batch over host arrays (or the given device pointers)."""
        def ptr(a):
            return None if a is None else a.ctypes.data
        b = ObcaBatch()
        b.batch, b.N, b.M, b.K, b.time_opt = self.batch, self.N, self.M, self.K, self.time_opt
        b.obs_edges, b.body_edges = self.obs_edges.ctypes.data, self.body_edges.ctypes.data
        src = ptrs or {}
        for name in ("traj", "obs_A", "obs_b", "body_G", "body_g", "params", "init_control", "init_mu", "init_lambda"):
            setattr(b, name, src[name] if name in src else ptr(getattr(self, name)))
        return b

    INPUTS = ("traj", "obs_A", "obs_b", "body_G", "body_g", "params", "init_control", "init_mu", "init_lambda")

    def chunk_struct(self, ptrs, lo, hi):
        """htp_obca_batch of problems [lo, hi) over base pointers `ptrs` (device or
        host) laid out like this batch's arrays (problem-major)."""
        b = self.struct(ptrs)
        b.batch = int(hi - lo)
        for name in self.INPUTS:
            a = getattr(self, name)
            base = ptrs[name] if name in ptrs else (None if a is None else a.ctypes.data)
            setattr(b, name, None if base is None else base + int(lo) * a.strides[0])
        return b

    @classmethod
    def concat(cls, parts):
        """One batch from same-shape PackedBatches (problem order kept)."""
        out = cls.__new__(cls)
        out.__dict__.update(parts[0].__dict__)
        out.batch = sum(p.batch for p in parts)
        for name in cls.INPUTS:
            a = [getattr(p, name) for p in parts]
            setattr(out, name, None if a[0] is None else np.ascontiguousarray(np.concatenate(a, axis=0)))
        return out


class ObcaPointsBatch(ctypes.Structure):  # htp_obca_points_batch
    _fields_ = [("batch", ctypes.c_int32), ("N", ctypes.c_int32), ("M", ctypes.c_int32),
                ("n_vertices", ctypes.c_int32), ("obs_edges", ctypes.c_void_p), ("traj", ctypes.c_void_p),
                ("obs_A", ctypes.c_void_p), ("obs_b", ctypes.c_void_p), ("vertices", ctypes.c_void_p),
                ("params", ctypes.c_void_p), ("init_control", ctypes.c_void_p)]


def points_params_of(inst):
    """HTP_P_* slots of a point-formulation instance (oracle/nlp_points.py format)."""
    p = np.zeros(NPARAM)
    p[P_DT] = inst["dT"]
    p[P_WHEELBASE] = inst["wheelbase"]
    p[P_MAXSTEER] = inst["max_steer"]
    p[P_MAXV] = inst["max_velocity"]
    p[P_MAXACC] = inst["max_accel"]
    p[P_MAXSR] = inst["max_steer_rate"]
    p[P_DMIN] = inst["min_dist"]
    xb = inst.get("x_bound", [-9999999, 9999999])
    yb = inst.get("y_bound", [-9999999, 9999999])
    p[P_XLO], p[P_XHI], p[P_YLO], p[P_YHI] = xb[0], xb[1], yb[0], yb[1]
    p[P_HAS_INIT_CONTROL] = inst.get("init_control") is not None
    return p


class PointsPackedBatch:
    """Contiguous problem-major arrays of a batch of point-formulation problems
    (R/obca_py/optimizer_points.py); all share N, obstacle edge counts and the
    number of hull vertices."""

    def __init__(self, insts):
        i0 = insts[0]
        self.batch = len(insts)
        self.N = int(np.asarray(i0["init_traj"]).shape[0])
        self.M = len(i0["obs_A"])
        self.n_vertices = int(np.asarray(i0["vertices"]).shape[0])
        self.obs_edges = np.array([a.shape[0] for a in i0["obs_A"]], dtype=np.int32)
        for it in insts:
            if (np.asarray(it["init_traj"]).shape[0] != self.N
                    or [a.shape[0] for a in it["obs_A"]] != list(self.obs_edges)
                    or np.asarray(it["vertices"]).shape[0] != self.n_vertices):
                raise ValueError("[OBCA points] all problems of a batch must share N, edge and vertex counts")
        self.traj = np.ascontiguousarray(np.stack([np.asarray(it["init_traj"], dtype=np.float64) for it in insts]))
        self.obs_A = np.ascontiguousarray(np.stack([np.concatenate(it["obs_A"], axis=0) for it in insts]))
        self.obs_b = np.ascontiguousarray(np.stack([np.concatenate(it["obs_b"]) for it in insts]))
        self.vertices = np.ascontiguousarray(np.stack([np.asarray(it["vertices"], dtype=np.float64) for it in insts]))
        self.params = np.ascontiguousarray(np.stack([points_params_of(it) for it in insts]))
        self.init_control = PackedBatch._opt(insts, "init_control")
        self.n_var = 5 * self.N + 2 * (self.N - 1) + self.N * int(self.obs_edges.sum())

    def struct(self, ptrs=None):
        def ptr(a):
            return None if a is None else a.ctypes.data
        b = ObcaPointsBatch()
        b.batch, b.N, b.M, b.n_vertices = self.batch, self.N, self.M, self.n_vertices
        b.obs_edges = self.obs_edges.ctypes.data
        src = ptrs or {}
        for name in ("traj", "obs_A", "obs_b", "vertices", "params", "init_control"):
            setattr(b, name, src[name] if name in src else ptr(getattr(self, name)))
        return b


class RpBatch(ctypes.Structure):  # htp_refpath_batch
    _fields_ = [("batch", ctypes.c_int32), ("cap_points", ctypes.c_int32), ("cap_rows", ctypes.c_int32),
                ("path_off", ctypes.c_void_p), ("xs", ctypes.c_void_p), ("ys", ctypes.c_void_p),
                ("dirs", ctypes.c_void_p), ("params", ctypes.c_void_p)]


class RpResult(ctypes.Structure):  # htp_refpath_result
    _fields_ = [("status", ctypes.c_void_p), ("n_rows", ctypes.c_void_p), ("traj", ctypes.c_void_p)]


RP_STATUS = {0: "ok", 1: "overflow", 2: "bad_segment", 3: "bad_input"}


class RefPathPacked:
    """CSR batch of warm-start paths for get_init_ref_path (R/obca_py/util.py:62-113).
    paths: list of (xs, ys, dirs) (yaw / curvature columns are not read by the reference);
    params: per path (WHEEL_BASE, desired_v, ds)."""

    def __init__(self, paths, params, cap_rows=None):
        self.batch = len(paths)
        lens = [len(p[0]) for p in paths]
        self.path_off = np.zeros(self.batch + 1, dtype=np.int32)
        self.path_off[1:] = np.cumsum(lens)
        cat = lambda k: np.ascontiguousarray(np.concatenate([np.asarray(p[k], dtype=np.float64) for p in paths])
                                             if paths else np.zeros(1))
        self.xs, self.ys, self.dirs = cat(0), cat(1), cat(2)
        self.params = np.ascontiguousarray(np.asarray(params, dtype=np.float64).reshape(self.batch, 3))
        self.cap_points = max(1, max(lens) if lens else 1)
        if cap_rows is None:  # arc length <= polyline length: ceil(len/ds) + 1 rows per segment, + 1 per segment
            cap_rows = 1
            for p, prm in zip(paths, self.params):
                L = float(np.sum(np.hypot(np.diff(p[0]), np.diff(p[1]))))
                nseg = 1 + int(np.count_nonzero(np.diff(np.asarray(p[2])) != 0))
                cap_rows = max(cap_rows, int(np.ceil(L / prm[2])) + 2 * nseg + 2)
        self.cap_rows = int(cap_rows)

    def struct(self, ptrs=None):
        b = RpBatch()
        b.batch, b.cap_points, b.cap_rows = self.batch, self.cap_points, self.cap_rows
        src = ptrs or {}
        for name in ("path_off", "xs", "ys", "dirs", "params"):
            setattr(b, name, src[name] if name in src else getattr(self, name).ctypes.data)
        return b


class RefPathResults:
    def __init__(self, packed):
        self.status = np.zeros(packed.batch, dtype=np.int32)
        self.n_rows = np.zeros(packed.batch, dtype=np.int32)
        self.traj = np.zeros((packed.batch, packed.cap_rows, 5))

    def struct(self):
        return RpResult(self.status.ctypes.data, self.n_rows.ctypes.data, self.traj.ctypes.data)

    def path(self, b):
        return self.traj[b, :self.n_rows[b]].copy()


class HostResults:
    def __init__(self, batch, n_var):
        self.x = np.zeros((batch, n_var))
        self.objective = np.zeros(batch)
        self.status = np.zeros(batch, dtype=np.int32)
        self.iterations = np.zeros(batch, dtype=np.int32)
        self.n_factor = np.zeros(batch, dtype=np.int32)
        self.nlp_error = np.zeros(batch)
        self.n_resto = np.zeros(batch, dtype=np.int32)

    def struct(self):
        r = ObcaResult()
        for name in ("x", "objective", "status", "iterations", "n_factor", "nlp_error", "n_resto"):
            setattr(r, name, getattr(self, name).ctypes.data)
        return r


def _clean_ring(poly):
    """Vertices without the repeated closing vertex or consecutive duplicates."""
    a = np.asarray(poly, dtype=np.float64).reshape(-1, 2)
    keep = [0]
    for i in range(1, a.shape[0]):
        if not np.array_equal(a[i], a[keep[-1]]):
            keep.append(i)
    a = a[keep]
    if a.shape[0] > 1 and np.array_equal(a[0], a[-1]):
        a = a[:-1]
    return a


def _ccw(a):
    area = np.sum(a[:, 0] * np.roll(a[:, 1], -1) - np.roll(a[:, 0], -1) * a[:, 1])
    return a if area > 0 else a[::-1].copy()


class HastarPacked:
    """htp_hastar_batch pools for a list of lowered hybrid A* problems (dicts
    made by path_planner.hybrid_a_star_search.lower_problem)."""

    def __init__(self, probs, cap_path=4096, cap_log=None):
        B = len(probs)
        polys, lane_len, guides, motions = [], [], [], []
        self.params = np.zeros((B, HA_NPARAM))
        self.desc = np.zeros((B, HA_NDESC), dtype=np.int32)
        ng = nm = 0
        for b, p in enumerate(probs):
            d = self.desc[b]
            d[HA_D_BODY] = len(polys)
            polys.append(_clean_ring(p["body"]))
            lane_len.append(0.0)
            d[HA_D_BLK0] = len(polys)
            for q in p["blockers"]:
                polys.append(_clean_ring(q))
                lane_len.append(0.0)
            d[HA_D_BLK1] = len(polys)
            d[HA_D_LANE0] = len(polys)
            for q, L in zip(p["lanes"], p["search_lengths"]):
                polys.append(_ccw(_clean_ring(q)))
                lane_len.append(float(L))
            d[HA_D_LANE1] = len(polys)
            if p["field"] is None:
                d[HA_D_FIELD] = -1
            else:
                d[HA_D_FIELD] = len(polys)
                polys.append(_clean_ring(p["field"]))
                lane_len.append(0.0)
            g = np.asarray(p["guide"], dtype=np.float64).reshape(-1, 4)
            d[HA_D_GUIDE0], d[HA_D_GUIDE1] = ng, ng + g.shape[0]
            guides.append(g)
            ng += g.shape[0]
            m = np.asarray(p["motions"], dtype=np.float64).reshape(-1, 2)
            d[HA_D_MOT0], d[HA_D_MOT1] = nm, nm + m.shape[0]
            motions.append(m)
            nm += m.shape[0]
            d[HA_D_KING] = 1 if p.get("king", True) else 0
            pr = self.params[b]
            pr[HA_P_SX:HA_P_SYAW + 1] = np.asarray(p["start"], dtype=np.float64)[:3]
            pr[HA_P_GX:HA_P_GYAW + 1] = np.asarray(p["goal"], dtype=np.float64)[:3]
            pr[HA_P_RES], pr[HA_P_YAWRES] = p["res"], p["yaw_res"]
            pr[HA_P_WB], pr[HA_P_MAXSTEER], pr[HA_P_CURV] = p["wheel_base"], p["max_steer"], p["curvature"]
            pr[HA_P_DEFLEN], pr[HA_P_MAXNODES] = p["default_search_length"], p["max_nodes"]
        self.batch = B
        self.poly_off = np.zeros(len(polys) + 1, dtype=np.int32)
        self.poly_off[1:] = np.cumsum([q.shape[0] for q in polys])
        self.vertices = np.ascontiguousarray(np.concatenate(polys, axis=0))
        self.lane_len = np.array(lane_len, dtype=np.float64)
        self.guide = np.ascontiguousarray(np.concatenate(guides, axis=0))
        self.motions = np.ascontiguousarray(np.concatenate(motions, axis=0))
        self.max_nodes_cap = int(max(int(p["max_nodes"]) for p in probs)) if B else 0
        self.cap_path = int(cap_path)
        self.cap_log = int(self.max_nodes_cap + 2 if cap_log is None else cap_log)

    def struct(self, ptrs=None):
        src = ptrs or {}
        b = HaBatch()
        b.batch, b.npoly, b.nvert = self.batch, len(self.poly_off) - 1, self.vertices.shape[0]
        b.nguide, b.nmotion = self.guide.shape[0], self.motions.shape[0]
        for n in ("params", "desc", "poly_off", "vertices", "lane_len", "guide", "motions"):
            setattr(b, n, src[n] if n in src else getattr(self, n).ctypes.data)
        b.max_nodes_cap, b.cap_path, b.cap_log = self.max_nodes_cap, self.cap_path, self.cap_log
        return b


class HastarResults:
    def __init__(self, packed):
        B, cp, cl = packed.batch, packed.cap_path, packed.cap_log
        self.status = np.zeros(B, np.int32)
        self.counter = np.zeros(B, np.int32)
        self.n_path = np.zeros(B, np.int32)
        self.n_expanded = np.zeros(B, np.int32)
        self.n_pose = np.zeros(B, np.int64)
        for n in ("x", "y", "yaw", "dir", "k"):
            setattr(self, n, np.zeros((B, cp)))
        self.expanded = np.zeros((B, cl, 3), np.int32)

    def struct(self):
        r = HaResult()
        for n in ("status", "counter", "n_path", "n_expanded", "n_pose", "x", "y", "yaw", "dir", "k", "expanded"):
            setattr(r, n, getattr(self, n).ctypes.data)
        return r

    def path(self, b):
        """(xs, ys, yaws, dirs, ks) of search b as lists (truncated to cap_path)."""
        n = min(int(self.n_path[b]), self.x.shape[1])
        return tuple(getattr(self, k)[b, :n].tolist() for k in ("x", "y", "yaw", "dir", "k"))

    def expansions(self, b):
        n = min(int(self.n_expanded[b]), self.expanded.shape[1])
        return [tuple(int(v) for v in r) for r in self.expanded[b, :n]]


class YparkPacked:
    """htp_ypark_batch pools for lowered Y-park searches (dicts made by
    path_planner.headland_path_planning.lower_ypark)."""

    def __init__(self, probs, cap_path=256):
        B = len(probs)
        polys, axis = [], []
        self.params = np.zeros((B, YP_NPARAM))
        self.desc = np.zeros((B, YP_NDESC), dtype=np.int32)
        for b, p in enumerate(probs):
            d = self.desc[b]
            d[0] = len(polys)
            polys.append(_clean_ring(p["body"]))
            d[1] = len(polys)
            for q in p["blockers"]:
                polys.append(_clean_ring(q))
            d[2] = len(polys)
            if p["field"] is None:
                d[3] = -1
            else:
                d[3] = len(polys)
                polys.append(_clean_ring(p["field"]))
            for a, key in enumerate(("backward_lengths", "forward_lengths", "backward_steers", "forward_steers")):
                vals = np.asarray(p[key], dtype=np.float64).reshape(-1)
                d[4 + 2 * a], d[5 + 2 * a] = len(axis), vals.size
                axis.extend(vals.tolist())
            self.params[b, :14] = [p["end_pose"][0], p["end_pose"][1], p["end_pose"][2], p["backward_steer_dir"],
                                   p["forward_steer_dir"], p["wheel_base"], p["step"], p["T"][0][0], p["T"][0][1],
                                   p["T"][1][0], p["T"][1][1], p["T"][0][3], p["T"][1][3], p["yaw_odom"]]
        self.batch = B
        self.poly_off = np.zeros(len(polys) + 1, dtype=np.int32)
        self.poly_off[1:] = np.cumsum([q.shape[0] for q in polys])
        self.vertices = np.ascontiguousarray(np.concatenate(polys, axis=0))
        self.axis = np.array(axis, dtype=np.float64)
        self.cap_path = int(cap_path)

    def struct(self, ptrs=None):
        src = ptrs or {}
        b = YpBatch()
        b.batch, b.npoly, b.nvert, b.naxis = self.batch, len(self.poly_off) - 1, self.vertices.shape[0], self.axis.size
        for n in ("params", "desc", "poly_off", "vertices", "axis"):
            setattr(b, n, src[n] if n in src else getattr(self, n).ctypes.data)
        b.cap_path = self.cap_path
        return b


class YparkResults:
    def __init__(self, packed):
        B = packed.batch
        self.status = np.zeros(B, np.int32)
        self.cand = np.zeros(B, np.int32)
        self.n_path = np.zeros(B, np.int32)
        self.params = np.zeros((B, 4))
        self.n_pose = np.zeros(B, np.int64)
        self.path = np.zeros((B, packed.cap_path, 5))

    def struct(self):
        r = YpResult()
        for n in ("status", "cand", "n_path", "params", "n_pose", "path"):
            setattr(r, n, getattr(self, n).ctypes.data)
        return r


# ------------------------------------------------------- orchard scene -> OBCA obstacles (htp_oge.hip)
OGE_NPARAM, OGE_MAXROWS, OGE_MAXPOLY, OGE_MAXV = 16, 32, 32, 12
OGE_STATUS = {0: "ok", 1: "bad_input", 2: "no_row_between", 3: "overflow", 4: "empty_side"}


class OgeBatch(ctypes.Structure):  # htp_oge_batch
    _fields_ = [("batch", ctypes.c_int32), ("max_rows", ctypes.c_int32), ("params", ctypes.c_void_p),
                ("row_draws", ctypes.c_void_p), ("eps_draws", ctypes.c_void_p)]


class OgeResult(ctypes.Structure):  # htp_oge_result
    _fields_ = [("status", ctypes.c_void_p), ("n_poly", ctypes.c_void_p), ("n_vert", ctypes.c_void_p),
                ("vertices", ctypes.c_void_p), ("n_facet", ctypes.c_void_p), ("A", ctypes.c_void_p),
                ("b", ctypes.c_void_p)]


class OgePacked:
    """Scenes for htp_oge_obstacles_batch.  A scene is a dict with nrows, row_width, row_length, slope,
    tree_width, headland_width, start, end, side (1 NEAR / -1 FAR) and the reference's random draws:
    row_draws (create_tree_rows, one per row) and eps_draws (create_headland_countour_lines, one per row)."""

    def __init__(self, scenes):
        B = len(scenes)
        self.batch = B
        self.max_rows = max(3, max((int(s["nrows"]) for s in scenes), default=3))
        if self.max_rows > OGE_MAXROWS:
            raise ValueError(f"[oge] at most {OGE_MAXROWS} tree rows per scene")
        self.params = np.zeros((B, OGE_NPARAM))
        self.row_draws = np.zeros((B, self.max_rows))
        self.eps_draws = np.zeros((B, self.max_rows))
        for b, s in enumerate(scenes):
            n = int(s["nrows"])
            self.params[b, :13] = [n, s["row_width"], s["row_length"], s["slope"], s["tree_width"],
                                   s["headland_width"], *np.asarray(s["start"], dtype=np.float64)[:3],
                                   *np.asarray(s["end"], dtype=np.float64)[:3], s.get("side", 1)]
            self.row_draws[b, :n] = s["row_draws"]
            self.eps_draws[b, :n] = s["eps_draws"]

    def struct(self, ptrs=None):
        p = ptrs or {}
        return OgeBatch(self.batch, self.max_rows, p.get("params", self.params.ctypes.data),
                        p.get("row_draws", self.row_draws.ctypes.data), p.get("eps_draws", self.eps_draws.ctypes.data))


class OgeResults:
    def __init__(self, batch, halfspaces=True):
        B = batch
        self.status = np.zeros(B, np.int32)
        self.n_poly = np.zeros(B, np.int32)
        self.n_vert = np.zeros((B, OGE_MAXPOLY), np.int32)
        self.vertices = np.zeros((B, OGE_MAXPOLY, OGE_MAXV, 2))
        self.n_facet = np.zeros((B, OGE_MAXPOLY), np.int32) if halfspaces else None
        self.A = np.zeros((B, OGE_MAXPOLY, OGE_MAXV, 2)) if halfspaces else None
        self.b = np.zeros((B, OGE_MAXPOLY, OGE_MAXV)) if halfspaces else None

    def struct(self):
        def ptr(a):
            return None if a is None else a.ctypes.data
        return OgeResult(self.status.ctypes.data, self.n_poly.ctypes.data, self.n_vert.ctypes.data,
                         self.vertices.ctypes.data, ptr(self.n_facet), ptr(self.A), ptr(self.b))

    def polygons(self, b):
        """Scene b's obstacle polygons [(n_v, 2) arrays] in the reference's order."""
        return [self.vertices[b, q, :self.n_vert[b, q]].copy() for q in range(int(self.n_poly[b]))]

    def halfspaces(self, b):
        """Scene b's [(A, b)] (compute_polytope_halfspaces of each polygon)."""
        out = []
        for q in range(int(self.n_poly[b])):
            f = int(self.n_facet[b, q])
            out.append((self.A[b, q, :f].copy(), self.b[b, q, :f].copy()))
        return out


# ------------------------------------------------------------ classic headland turns (htp_classic.hip)
CT_NPARAM = 12
CT_TYPES = {"dubins": 0, "circleback": 1, "fishtail": 2}
CT_STATUS = {0: "ok", 1: "overflow", 2: "no_word", 3: "bad_input", 4: "rs_error", 5: "no_dubins"}


class CtBatch(ctypes.Structure):  # htp_classic_batch
    _fields_ = [("batch", ctypes.c_int32), ("npoly", ctypes.c_int32), ("nvert", ctypes.c_int32),
                ("params", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("poly_off", ctypes.c_void_p),
                ("vertices", ctypes.c_void_p), ("cap_path", ctypes.c_int32), ("cap_samples", ctypes.c_int32)]


class CtResult(ctypes.Structure):  # htp_classic_result
    _fields_ = [("status", ctypes.c_void_p), ("n_path", ctypes.c_void_p), ("path", ctypes.c_void_p)]


class ClassicPacked:
    """Turns for htp_classic_turn_batch.  A turn is a dict: type ("dubins" / "circleback" / "fishtail"), side
    (map_utils NEAR_SIDE 1 / FAR_SIDE 2), start, end (x, y, yaw), wheel_base, max_steer, radius (the planners'
    turning-radius argument), step, body (car_poly ring), blockers (obs_poly_list rings; fish-tail only)."""

    def __init__(self, turns, cap_path=4096, cap_samples=4096):
        B = len(turns)
        self.batch, self.cap_path, self.cap_samples = B, int(cap_path), int(cap_samples)
        self.params = np.zeros((B, CT_NPARAM))
        self.desc = np.zeros((B, 3), np.int32)
        polys = []
        for b, t in enumerate(turns):
            self.params[b] = [CT_TYPES[t["type"]], t.get("side", 1), *np.asarray(t["start"], dtype=np.float64)[:3],
                              *np.asarray(t["end"], dtype=np.float64)[:3], t["wheel_base"], t["max_steer"],
                              t["radius"], t.get("step", 0.1)]
            self.desc[b, 0] = len(polys)
            polys.append(np.asarray(t["body"], dtype=np.float64).reshape(-1, 2))
            self.desc[b, 1] = len(polys)
            polys += [np.asarray(q, dtype=np.float64).reshape(-1, 2) for q in t.get("blockers", [])]
            self.desc[b, 2] = len(polys)
        self.poly_off = np.concatenate([[0], np.cumsum([len(q) for q in polys])]).astype(np.int32)
        self.vertices = np.ascontiguousarray(np.concatenate(polys) if polys else np.zeros((0, 2)))

    def struct(self, ptrs=None):
        p = ptrs or {}
        return CtBatch(self.batch, len(self.poly_off) - 1, self.vertices.shape[0],
                       p.get("params", self.params.ctypes.data), p.get("desc", self.desc.ctypes.data),
                       p.get("poly_off", self.poly_off.ctypes.data), p.get("vertices", self.vertices.ctypes.data),
                       self.cap_path, self.cap_samples)


class ClassicResults:
    def __init__(self, packed):
        B = packed.batch
        self.status = np.zeros(B, np.int32)
        self.n_path = np.zeros(B, np.int32)
        self.path = np.zeros((B, packed.cap_path, 5))

    def struct(self):
        return CtResult(self.status.ctypes.data, self.n_path.ctypes.data, self.path.ctypes.data)

    def rows(self, b):
        return self.path[b, :int(self.n_path[b])].copy()


class ChainBatch(ctypes.Structure):  # htp_chain_batch
    _fields_ = [("batch", ctypes.c_int32), ("N", ctypes.c_int32), ("M", ctypes.c_int32),
                ("scenes", OgeBatch), ("turns", CtBatch), ("margin", ctypes.c_void_p),
                ("n_vpoly", ctypes.c_int32), ("vpoly_nv", ctypes.c_int32 * 2), ("vpoly", ctypes.c_double * 32),
                ("dT", ctypes.c_double), ("wheel_base", ctypes.c_double), ("cap_rows", ctypes.c_int32),
                ("traj", ctypes.c_void_p), ("obs_A", ctypes.c_void_p), ("obs_b", ctypes.c_void_p),
                ("status", ctypes.c_void_p)]


class WorkQueue:
    """Host work queue of problem indices feeding one persistent solve launch
    (htp_queue_*: pinned, GPU-coherent host memory)."""

    def __init__(self, ctx, capacity):
        self.lib = ctx.lib
        self.q = self.lib.htp_queue_create(ctx.ctx, int(capacity))
        if not self.q:
            raise RuntimeError(f"[htp] htp_queue_create failed: {ctx.error()}")

    def publish(self, pids):
        a = np.ascontiguousarray(np.asarray(pids, dtype=np.int32))
        if self.lib.htp_queue_publish(self.q, a.ctypes.data, a.size) != 0:
            raise RuntimeError("[htp] htp_queue_publish failed (full, closed or index out of range)")

    def close(self):
        self.lib.htp_queue_close(self.q)

    def published(self):
        return int(self.lib.htp_queue_published(self.q))

    def claimed(self):
        return int(self.lib.htp_queue_claimed(self.q))

    def destroy(self):
        if self.q:
            self.lib.htp_queue_destroy(self.q)
            self.q = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class Context:
    """Owns one htp_ctx (device workspace)."""

    def __init__(self, device=0, options=None, lib=None):
        self.lib = lib or load()
        self.device = int(device)
        self.ctx = self.lib.htp_create(int(device))
        if not self.ctx:
            raise RuntimeError("[htp] htp_create failed")
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def set_option(self, name, value):
        if self.lib.htp_set_option(self.ctx, name.encode(), float(value)) != 0:
            raise ValueError(f"[htp] unknown option {name}")

    def error(self):
        return self.lib.htp_last_error(self.ctx).decode()

    def solve(self, packed):
        res = HostResults(packed.batch, packed.n_var)
        b, r = packed.struct(), res.struct()
        rc = self.lib.htp_obca_solve_batch(self.ctx, ctypes.byref(b), ctypes.byref(r))
        if rc != 0:
            raise RuntimeError(f"[htp] htp_obca_solve_batch failed: {self.error()}")
        return res

    def libm(self, name, x, y=None):
        """The device build of the planner libm over host arrays (through device buffers) -> float64 array."""
        import torch
        dev = torch.device("cuda", self.device)
        xt = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).to(dev)
        yt = None
        if y is not None:
            yt = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(y, np.shape(x)), dtype=np.float64)).to(dev)
        out = torch.empty_like(xt)
        s = torch.cuda.current_stream(dev)
        rc = self.lib.htp_libm_batch_device(self.ctx, LIBM_FN[name], xt.data_ptr(),
                                            yt.data_ptr() if yt is not None else None, out.data_ptr(), xt.numel(),
                                            ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"[htp] htp_libm_batch_device failed: {self.error()}")
        s.synchronize()
        return out.cpu().numpy()

    def mfma_f64(self, A, B, C):
        """htp_mfma_f64_probe over host tiles A [n,16,4], B [n,4,16], C [n,16,16] -> D [n,16,16]."""
        import torch
        dev = torch.device("cuda", self.device)
        t = [torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64)).to(dev) for v in (A, B, C)]
        n = t[0].shape[0]
        if t[0].shape != (n, 16, 4) or t[1].shape != (n, 4, 16) or t[2].shape != (n, 16, 16):
            raise ValueError("[htp] mfma_f64: tiles must be [n,16,4], [n,4,16], [n,16,16]")
        out = torch.empty_like(t[2])
        s = torch.cuda.current_stream(dev)
        rc = self.lib.htp_mfma_f64_probe(self.ctx, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), out.data_ptr(),
                                         n, ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"[htp] htp_mfma_f64_probe failed: {self.error()}")
        s.synchronize()
        return out.cpu().numpy()

    def solve_points(self, packed):
        """Batched optimizer_points.py solve (host buffers)."""
        res = HostResults(packed.batch, packed.n_var)
        b, r = packed.struct(), res.struct()
        rc = self.lib.htp_obca_points_solve_batch(self.ctx, ctypes.byref(b), ctypes.byref(r))
        if rc != 0:
            raise RuntimeError(f"[htp] htp_obca_points_solve_batch failed: {self.error()}")
        return res

    def classic_turns(self, packed):
        """Batched classic headland turns (host buffers) -> ClassicResults."""
        r = ClassicResults(packed)
        b, rs = packed.struct(), r.struct()
        if self.lib.htp_classic_turn_batch(self.ctx, ctypes.byref(b), ctypes.byref(rs)) != 0:
            raise RuntimeError(f"[htp] htp_classic_turn_batch failed: {self.error()}")
        return r

    def classic_last_ms(self):
        return self.lib.htp_classic_last_ms(self.ctx)

    def oge_obstacles(self, packed, halfspaces=True):
        """Batched orchard scene -> OBCA obstacle polygons (+ halfspaces), host buffers -> OgeResults."""
        r = OgeResults(packed.batch, halfspaces)
        b, rs = packed.struct(), r.struct()
        if self.lib.htp_oge_obstacles_batch(self.ctx, ctypes.byref(b), ctypes.byref(rs)) != 0:
            raise RuntimeError(f"[htp] htp_oge_obstacles_batch failed: {self.error()}")
        return r

    def oge_last_ms(self):
        return self.lib.htp_oge_last_ms(self.ctx)

    def init_ref_path(self, packed):
        """Batched get_init_ref_path (host buffers) -> RefPathResults."""
        res = RefPathResults(packed)
        b, r = packed.struct(), res.struct()
        if self.lib.htp_init_ref_path_batch(self.ctx, ctypes.byref(b), ctypes.byref(r)) != 0:
            raise RuntimeError(f"[htp] htp_init_ref_path_batch failed: {self.error()}")
        return res

    def init_ref_path_last_ms(self):
        return self.lib.htp_init_ref_path_last_ms(self.ctx)

    def solve_device(self, packed, dev_ptrs, out_ptrs, stream=None, lo=None, hi=None):
        """Device-resident solve of `packed` (or of its problems [lo, hi)) on `stream`."""
        b = packed.struct(dev_ptrs) if lo is None else packed.chunk_struct(dev_ptrs, lo, hi)
        r = ObcaResult()
        for k, v in out_ptrs.items():
            setattr(r, k, v)
        rc = self.lib.htp_obca_solve_batch_device(self.ctx, ctypes.byref(b), ctypes.byref(r), stream)
        if rc != 0:
            raise RuntimeError(f"[htp] htp_obca_solve_batch_device failed: {self.error()}")

    def last_kernel_ms(self):
        return self.lib.htp_last_kernel_ms(self.ctx)

    def resident_waves(self, packed):
        v = self.lib.htp_obca_resident_waves(self.ctx, ctypes.byref(packed.struct()))
        if v <= 0:
            raise RuntimeError(f"[htp] htp_obca_resident_waves failed: {self.error()}")
        return v

    def solve_queue_device(self, packed, dev_ptrs, queue, out_ptrs, stream=None, waves=0, max_wait_s=60.0):
        """Persistent launch over the resident problems of `packed`, fed by `queue` (WorkQueue)."""
        b = packed.struct(dev_ptrs)
        r = ObcaResult()
        for k, v in out_ptrs.items():
            setattr(r, k, v)
        rc = self.lib.htp_obca_solve_queue_device(self.ctx, ctypes.byref(b), queue.q, ctypes.byref(r), stream,
                                                  int(waves), float(max_wait_s))
        if rc != 0:
            raise RuntimeError(f"[htp] htp_obca_solve_queue_device failed: {self.error()}")

    def last_cycles(self, batch):
        """[batch, 8] shader-cycle counters: local sweeps, stage assembly,
        stage chain, KKT solves, total, errors+grad_lag, line search, update+re-eval."""
        out = np.zeros((batch, 8), dtype=np.int64)
        if self.lib.htp_last_cycles(self.ctx, out.ctypes.data, int(batch)) != 0:
            raise RuntimeError(self.error())
        return out

    def rs_all_paths(self, queries):
        """Reeds-Shepp calc_all_paths for a batch of queries [B, 8] =
        (sx, sy, syaw, gx, gy, gyaw, maxc, step_size); returns CSR numpy arrays
        (host buffers; a size query first, then the fill)."""
        q = np.ascontiguousarray(np.asarray(queries, dtype=np.float64).reshape(-1, 8))
        B = q.shape[0]
        out = {"path_offsets": np.zeros(B + 1, np.int64), "status": np.zeros(B, np.int32)}
        cap_p = cap_q = 0
        for _ in range(2):
            out.update(lengths=np.zeros((cap_p, 5)), ctypes=np.zeros((cap_p, 5), np.int8), L=np.zeros(cap_p),
                       point_offsets=np.zeros(cap_p + 1, np.int64), x=np.zeros(cap_q), y=np.zeros(cap_q),
                       yaw=np.zeros(cap_q), cs=np.zeros(cap_q), directions=np.zeros(cap_q, np.int8))
            st = RsPaths(cap_p, cap_q, 0, 0, *[out[k].ctypes.data for k in (
                "path_offsets", "status", "lengths", "ctypes", "L", "point_offsets", "x", "y", "yaw", "cs",
                "directions")])
            rc = self.lib.htp_rs_all_paths_batch(self.ctx, B, q.ctypes.data, ctypes.byref(st))
            if rc == 0:
                break
            if rc != RS_CAPACITY:
                raise RuntimeError(f"[htp] htp_rs_all_paths_batch failed: {self.error()}")
            cap_p, cap_q = int(st.n_paths), int(st.n_points)
        else:
            raise RuntimeError("[htp] htp_rs_all_paths_batch: capacity negotiation failed")
        out["n_paths"], out["n_points"] = int(st.n_paths), int(st.n_points)
        return out

    def rs_all_paths_device(self, batch, q_ptr, out_ptrs, caps, totals_ptr, stream=None):
        st = RsPaths(int(caps[0]), int(caps[1]), 0, 0, *[out_ptrs.get(k) for k in (
            "path_offsets", "status", "lengths", "ctypes", "L", "point_offsets", "x", "y", "yaw", "cs",
            "directions")])
        rc = self.lib.htp_rs_all_paths_batch_device(self.ctx, int(batch), q_ptr, ctypes.byref(st), totals_ptr, stream)
        if rc != 0:
            raise RuntimeError(f"[htp] htp_rs_all_paths_batch_device failed: {self.error()}")

    def rs_last_ms(self):
        return self.lib.htp_rs_last_ms(self.ctx)

    def hastar(self, packed):
        """Hybrid A* searches of a HastarPacked batch (host buffers, synchronous)."""
        res = HastarResults(packed)
        b, r = packed.struct(), res.struct()
        rc = self.lib.htp_hastar_search_batch(self.ctx, ctypes.byref(b), ctypes.byref(r))
        if rc != 0:
            raise RuntimeError(f"[htp] htp_hastar_search_batch failed: {self.error()}")
        return res

    def hastar_device(self, packed, dev_ptrs, out_ptrs, stream=None):
        b = packed.struct(dev_ptrs)
        r = HaResult()
        for k, v in out_ptrs.items():
            setattr(r, k, v)
        rc = self.lib.htp_hastar_search_batch_device(self.ctx, ctypes.byref(b), ctypes.byref(r), stream)
        if rc != 0:
            raise RuntimeError(f"[htp] htp_hastar_search_batch_device failed: {self.error()}")

    def hastar_last_ms(self):
        return self.lib.htp_hastar_last_ms(self.ctx)

    def ypark(self, packed):
        """Y-park grid searches of a YparkPacked batch (host buffers, synchronous)."""
        res = YparkResults(packed)
        b, r = packed.struct(), res.struct()
        rc = self.lib.htp_ypark_search_batch(self.ctx, ctypes.byref(b), ctypes.byref(r))
        if rc != 0:
            raise RuntimeError(f"[htp] htp_ypark_search_batch failed: {self.error()}")
        return res

    def ypark_last_ms(self):
        return self.lib.htp_ypark_last_ms(self.ctx)

    def close(self):
        if self.ctx:
            self.lib.htp_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
