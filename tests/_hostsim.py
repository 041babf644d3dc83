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
TSO = os.path.join(ROOT, "build", "libhtp_threadsim.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    if os.path.exists(SO) and os.path.getmtime(SO) >= max(os.path.getmtime(s) for s in srcs):
        return SO
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO,
                           os.path.join(CSRC, "htp_hostsim.cpp")])
    return SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        _lib.htp_hostsim_obca_solve.argtypes = [ctypes.POINTER(_native.ObcaBatch), ctypes.POINTER(_native.ObcaResult),
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib.htp_hostsim_obca_solve.restype = ctypes.c_int
    return _lib


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
