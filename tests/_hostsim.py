"""TEST-ONLY: ctypes access to the serial host build of the solver core
(headland_trajectory_planning_amd/csrc/htp_hostsim.cpp).  Used to debug the
kernel logic against the oracle without a GPU; the product never loads it."""
import ctypes
import os
import subprocess

import numpy as np

from headland_trajectory_planning_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "headland_trajectory_planning_amd", "csrc")
SO = os.path.join(ROOT, "build", "libhtp_hostsim.so")
# the same sources with the platform libm (-DHTP_LIBM_PLATFORM, csrc/htp_libm.h): the build that reproduces the
# reference's own doubles where CPython's math module (glibc) produced them -- golden-vector tests only
SO_PLAT = os.path.join(ROOT, "build", "libhtp_hostsim_plat.so")
TSO = os.path.join(ROOT, "build", "libhtp_threadsim.so")


def build(platform=False):
    so = SO_PLAT if platform else SO
    os.makedirs(os.path.dirname(so), exist_ok=True)
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    if os.path.exists(so) and os.path.getmtime(so) >= max(os.path.getmtime(s) for s in srcs):
        return so
    extra = ["-DHTP_LIBM_PLATFORM"] if platform else []
    subprocess.check_call(["g++", "-O2", "-fno-builtin", "-std=c++17", "-shared", "-fPIC"] + extra + ["-o", so,
                           os.path.join(CSRC, "htp_hostsim.cpp"), os.path.join(CSRC, "rs_hostsim.cpp"),
                           os.path.join(CSRC, "hastar_hostsim.cpp"), os.path.join(CSRC, "ypark_hostsim.cpp"),
                           os.path.join(CSRC, "refpath_hostsim.cpp"), os.path.join(CSRC, "oge_hostsim.cpp"),
                           os.path.join(CSRC, "classic_hostsim.cpp"), os.path.join(CSRC, "chain_hostsim.cpp")])
    return so


_libs = {}


def lib(platform=False):
    if platform not in _libs:
        L = ctypes.CDLL(build(platform))
        L.htp_hostsim_obca_solve.argtypes = [ctypes.POINTER(_native.ObcaBatch), ctypes.POINTER(_native.ObcaResult),
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.htp_hostsim_obca_solve.restype = ctypes.c_int
        _libs[platform] = L
    return _libs[platform]


def init_ref_path_host(packed, platform=False):
    """refpath_core.h through the serial host build (same CSR batch as the GPU)."""
    L = lib(platform)
    L.htp_hostsim_init_ref_path.argtypes = [ctypes.POINTER(_native.RpBatch), ctypes.POINTER(_native.RpResult)]
    L.htp_hostsim_init_ref_path.restype = ctypes.c_int
    res = _native.RefPathResults(packed)
    b, r = packed.struct(), res.struct()
    assert L.htp_hostsim_init_ref_path(ctypes.byref(b), ctypes.byref(r)) == 0
    return res


def solve_points(insts, options=None):
    """Point formulation (optimizer_points.py) through the serial host build."""
    L = lib()
    L.htp_hostsim_obca_points_solve.argtypes = [ctypes.POINTER(_native.ObcaPointsBatch),
                                                ctypes.POINTER(_native.ObcaResult), ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_int]
    L.htp_hostsim_obca_points_solve.restype = ctypes.c_int
    pk = _native.PointsPackedBatch(insts)
    res = _native.HostResults(pk.batch, pk.n_var)
    opts = options or {}
    names = (ctypes.c_char_p * max(1, len(opts)))(*[k.encode() for k in opts])
    vals = (ctypes.c_double * max(1, len(opts)))(*[float(v) for v in opts.values()])
    b, r = pk.struct(), res.struct()
    rc = L.htp_hostsim_obca_points_solve(ctypes.byref(b), ctypes.byref(r), names, vals, len(opts))
    assert rc == 0, rc
    return res


def solve(insts, options=None):
    pk = _native.PackedBatch(insts)
    res = _native.HostResults(pk.batch, pk.n_var)
    opts = options or {}
    names = (ctypes.c_char_p * max(1, len(opts)))(*[k.encode() for k in opts])
    vals = (ctypes.c_double * max(1, len(opts)))(*[float(v) for v in opts.values()])
    b, r = pk.struct(), res.struct()
    rc = lib().htp_hostsim_obca_solve(ctypes.byref(b), ctypes.byref(r), names, vals, len(opts))
    assert rc == 0, rc
    return res


ESO = os.path.join(ROOT, "build", "libhtp_emusim.so")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def build_emusim():
    """The bit-exact host emulation of the device solver (csrc/htp_emusim.cpp, emu_wave.h): clang with the
    device build's contraction (fused only within an expression) and FMA; the device's wave-reduction and
    matrix-core order.  TEST-ONLY."""
    os.makedirs(os.path.dirname(ESO), exist_ok=True)
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(ROOT, "include", "htp.h")]
    if not (os.path.exists(ESO) and os.path.getmtime(ESO) >= max(os.path.getmtime(s) for s in srcs)):
        subprocess.check_call([CLANG, "-O2", "-std=c++20", "-ffp-contract=on", "-mfma", "-shared", "-fPIC", "-o", ESO,
                               os.path.join(CSRC, "htp_emusim.cpp"), "-lpthread"])
    L = ctypes.CDLL(ESO)
    L.htp_emusim_obca_solve.argtypes = [ctypes.POINTER(_native.ObcaBatch), ctypes.POINTER(_native.ObcaResult),
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.htp_emusim_obca_solve.restype = ctypes.c_int
    L.htp_emusim_obca_points_solve.argtypes = [ctypes.POINTER(_native.ObcaPointsBatch),
                                               ctypes.POINTER(_native.ObcaResult), ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_int]
    L.htp_emusim_obca_points_solve.restype = ctypes.c_int
    return L


def _opts(options):
    opts = dict(options or {})
    names = (ctypes.c_char_p * max(1, len(opts)))(*[k.encode() for k in opts])
    vals = (ctypes.c_double * max(1, len(opts)))(*[float(v) for v in opts.values()])
    return names, vals, len(opts)


def solve_emusim(insts, options=None):
    """OBCA problems through the device emulation -> HostResults (the device's doubles, bit for bit)."""
    L = build_emusim()
    pk = _native.PackedBatch(insts)
    res = _native.HostResults(pk.batch, pk.n_var)
    b, r = pk.struct(), res.struct()
    assert L.htp_emusim_obca_solve(ctypes.byref(b), ctypes.byref(r), *_opts(options)) == 0
    return res


def solve_points_emusim(insts, options=None):
    L = build_emusim()
    pk = _native.PointsPackedBatch(insts)
    res = _native.HostResults(pk.batch, pk.n_var)
    b, r = pk.struct(), res.struct()
    assert L.htp_emusim_obca_points_solve(ctypes.byref(b), ctypes.byref(r), *_opts(options)) == 0
    return res


def build_threadsim():
    """64-thread wavefront simulation (std::barrier per sync) of the same core."""
    os.makedirs(os.path.dirname(TSO), exist_ok=True)
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    if not (os.path.exists(TSO) and os.path.getmtime(TSO) >= max(os.path.getmtime(s) for s in srcs)):
        subprocess.check_call(["g++", "-O2", "-std=c++20", "-shared", "-fPIC", "-o", TSO,
                               os.path.join(CSRC, "htp_threadsim.cpp"), "-lpthread"])
    lib_ = ctypes.CDLL(TSO)
    lib_.htp_threadsim_obca_solve.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib_.htp_threadsim_obca_solve.restype = ctypes.c_int
    return lib_


def solve_threadsim(insts, max_iter=-1):
    lib_ = build_threadsim()
    pk = _native.PackedBatch(insts)
    res = _native.HostResults(pk.batch, pk.n_var)
    rc = lib_.htp_threadsim_obca_solve(ctypes.byref(pk.struct()), ctypes.byref(res.struct()), max_iter)
    assert rc == 0
    return res


def rs_host(queries, platform=False):
    """Host build of csrc/rs_core.h (same CSR dict as Context.rs_all_paths),
    one query per call.  TEST-ONLY."""
    l = lib(platform)
    f = l.htp_hostsim_rs
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 11
    q = np.ascontiguousarray(np.asarray(queries, dtype=np.float64).reshape(-1, 8))
    parts = {k: [] for k in ("lengths", "ctypes", "L", "x", "y", "yaw", "cs", "directions")}
    status, npaths, npts_path = [], [], []
    np1, nq = np.zeros(1, np.int32), np.zeros(1, np.int64)
    for row in q:
        cp, cq = 0, 0
        for _ in range(2):
            ln, ct, L = np.zeros((cp, 5)), np.zeros((cp, 5), np.int8), np.zeros(cp)
            off = np.zeros(cp + 1, np.int64)
            x, y, yaw, cs = (np.zeros(cq) for _ in range(4))
            d = np.zeros(cq, np.int8)
            st = f(row.ctypes.data, cp, cq, np1.ctypes.data, nq.ctypes.data, ln.ctypes.data, ct.ctypes.data,
                   L.ctypes.data, off.ctypes.data, x.ctypes.data, y.ctypes.data, yaw.ctypes.data, cs.ctypes.data,
                   d.ctypes.data)
            if cp >= np1[0] and cq >= nq[0]:
                break
            cp, cq = int(np1[0]), int(nq[0])
        status.append(st)
        npaths.append(int(np1[0]))
        npts_path.extend(np.diff(off).tolist())
        for k, v in zip(("lengths", "ctypes", "L", "x", "y", "yaw", "cs", "directions"), (ln, ct, L, x, y, yaw, cs, d)):
            parts[k].append(v)
    out = {k: np.concatenate(v) if v else np.zeros(0) for k, v in parts.items()}
    out["status"] = np.array(status, np.int32)
    out["path_offsets"] = np.concatenate([[0], np.cumsum(npaths)]).astype(np.int64)
    out["point_offsets"] = np.concatenate([[0], np.cumsum(npts_path)]).astype(np.int64)
    out["n_paths"], out["n_points"] = int(out["path_offsets"][-1]), int(out["point_offsets"][-1])
    return out


def oge_host(packed, halfspaces=True, platform=False):
    """oge_core.h through the serial host build (same batch/result structs as the GPU).  TEST-ONLY."""
    L = lib(platform)
    L.htp_hostsim_oge.argtypes = [ctypes.POINTER(_native.OgeBatch), ctypes.POINTER(_native.OgeResult)]
    L.htp_hostsim_oge.restype = ctypes.c_int
    res = _native.OgeResults(packed.batch, halfspaces)
    b, r = packed.struct(), res.struct()
    assert L.htp_hostsim_oge(ctypes.byref(b), ctypes.byref(r)) == 0
    return res


def chain_host(inputs, platform=False):
    """The orchard workload chain (chain_core.h) through the serial host build -> (instances, status).
    `inputs` from e2e.host_inputs.  TEST-ONLY."""
    L = lib(platform)
    L.htp_hostsim_chain.argtypes = [ctypes.POINTER(_native.ChainBatch)]
    L.htp_hostsim_chain.restype = ctypes.c_int
    sc, tu = inputs["scenes"], inputs["turns"]
    B, N, M = sc.batch, inputs["N"], inputs["M"]
    params = sc.params.copy()
    traj, A, b = np.zeros((B, N, 5)), np.zeros((B, 4 * M, 2)), np.zeros((B, 4 * M))
    status = np.zeros(B, np.int32)
    cb = _native.ChainBatch()
    cb.batch, cb.N, cb.M = B, N, M
    cb.scenes = sc.struct({"params": params.ctypes.data})
    cb.turns = tu.struct()
    margin = np.ascontiguousarray(inputs["margin"], dtype=np.float64)
    cb.margin = margin.ctypes.data
    cb.n_vpoly = len(inputs["polys"])
    vp = np.zeros((2, 8, 2))
    for k, p in enumerate(inputs["polys"]):
        cb.vpoly_nv[k] = p.shape[0]
        vp[k, :p.shape[0]] = p
    for i, v in enumerate(vp.reshape(-1)):
        cb.vpoly[i] = float(v)
    t = inputs["template"]
    cb.dT, cb.wheel_base, cb.cap_rows = float(t["dT"]), 1.9, 1024
    cb.traj, cb.obs_A, cb.obs_b, cb.status = traj.ctypes.data, A.ctypes.data, b.ctypes.data, status.ctypes.data
    assert L.htp_hostsim_chain(ctypes.byref(cb)) == 0
    insts = [dict(init_traj=traj[k], obs_A=[A[k, 4 * m:4 * m + 4] for m in range(M)],
                  obs_b=[b[k, 4 * m:4 * m + 4] for m in range(M)]) for k in range(B)]
    return insts, status


def classic_host(packed, platform=False):
    """classic_core.h through the serial host build (same batch/result structs as the GPU).  TEST-ONLY."""
    L = lib(platform)
    L.htp_hostsim_classic.argtypes = [ctypes.POINTER(_native.CtBatch), ctypes.POINTER(_native.CtResult)]
    L.htp_hostsim_classic.restype = ctypes.c_int
    res = _native.ClassicResults(packed)
    b, r = packed.struct(), res.struct()
    assert L.htp_hostsim_classic(ctypes.byref(b), ctypes.byref(r)) == 0
    return res


def hastar_host(problems, cap_path=4096, platform=False):
    """Host build of csrc/hastar_core.h (serial lane), same result object as
    Context.hastar.  TEST-ONLY."""
    l = lib(platform)
    f = l.htp_hostsim_hastar
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.POINTER(_native.HaBatch), ctypes.POINTER(_native.HaResult)]
    pk = _native.HastarPacked(problems, cap_path=cap_path)
    res = _native.HastarResults(pk)
    assert f(ctypes.byref(pk.struct()), ctypes.byref(res.struct())) == 0
    return res


def as_dicts(res):
    out = []
    for b in range(len(res.status)):
        xs, ys, yaws, dirs, ks = res.path(b)
        out.append(dict(xs=xs, ys=ys, yaws=yaws, dirs=dirs, ks=ks, counter=int(res.counter[b]),
                        status=int(res.status[b]), expanded=res.expansions(b), n_pose=int(res.n_pose[b])))
    return out


def ypark_host(problems, cap_path=256, platform=False):
    """Host build of csrc/ypark_core.h (serial lane), same result object as
    Context.ypark.  TEST-ONLY."""
    l = lib(platform)
    f = l.htp_hostsim_ypark
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.POINTER(_native.YpBatch), ctypes.POINTER(_native.YpResult)]
    pk = _native.YparkPacked(problems, cap_path=cap_path)
    res = _native.YparkResults(pk)
    assert f(ctypes.byref(pk.struct()), ctypes.byref(res.struct())) == 0
    return res


def ypark_dicts(res):
    return [dict(status=int(res.status[b]), cand=int(res.cand[b]), params=res.params[b].tolist(),
                 path=res.path[b, :int(res.n_path[b])].copy(), n_pose=int(res.n_pose[b]))
            for b in range(len(res.status))]


ASAN_EXE = os.path.join(ROOT, "build", "hastar_asan")


def hastar_asan(problems, cap_path=4096, sanitize=True):
    """The host build of hastar_core.h (csrc/hastar_asan.cpp) as a standalone executable built
    with -fsanitize=address,undefined: any out-of-bounds access or UB aborts it.  Same result
    object as hastar_host.  TEST-ONLY."""
    import tempfile
    exe = ASAN_EXE if sanitize else ASAN_EXE + "_plain"
    src = os.path.join(CSRC, "hastar_asan.cpp")
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + [src]
    if not (os.path.exists(exe) and os.path.getmtime(exe) >= max(os.path.getmtime(d) for d in deps)):
        os.makedirs(os.path.dirname(exe), exist_ok=True)
        flags = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"] \
            if sanitize else []
        subprocess.check_call(["g++", "-O1", "-g", "-std=c++17"] + flags + ["-o", exe, src])
    pk = _native.HastarPacked(problems, cap_path=cap_path)
    res = _native.HastarResults(pk)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fin, "wb") as f:
            np.array([pk.batch, len(pk.poly_off) - 1, pk.vertices.shape[0], pk.guide.shape[0], pk.motions.shape[0],
                      pk.max_nodes_cap, pk.cap_path, pk.cap_log], np.int32).tofile(f)
            for a, t in ((pk.params, np.float64), (pk.desc, np.int32), (pk.poly_off, np.int32),
                         (pk.vertices, np.float64), (pk.lane_len, np.float64), (pk.guide, np.float64),
                         (pk.motions, np.float64)):
                np.ascontiguousarray(a, dtype=t).tofile(f)
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
        p = subprocess.run([exe, fin, fout], env=env, capture_output=True, text=True, timeout=1800)
        if p.returncode != 0:
            raise RuntimeError(f"hastar_asan exit {p.returncode}: {p.stderr[-4000:]}")
        with open(fout, "rb") as f:
            for n in ("status", "counter", "n_path", "n_expanded", "n_pose", "x", "y", "yaw", "dir", "k", "expanded"):
                a = getattr(res, n)
                a[...] = np.fromfile(f, dtype=a.dtype, count=a.size).reshape(a.shape)
    return res
