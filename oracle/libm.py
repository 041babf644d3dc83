"""Which libm the oracle's transcendental functions come from.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference's solve runs CasADi's SX virtual machine, which evaluates sin / cos / tan / log through the C
library (std::sin ... = glibc on Linux) inside IPOPT's iterations (R/obca_py/optimizer.py:489-507).  The oracle
evaluates the same expressions with numpy ufuncs; on an AVX-512 host numpy's float64 sin / cos / tan / log are its
own SIMD kernels, which differ from glibc in the last bits of a fraction of arguments (tools/libm_check.py,
profiles/r04_libm_check.json).  Both are valid libms for the reference algorithm; this module lets a fixture
script run the oracle with either:

    MODE = "numpy"   the default (every committed fixture)
    MODE = "glibc"   CPython's math module, i.e. the glibc functions CasADi's SX VM calls

Used by tests/golden/make_witness.py's libm witnesses: where the oracle's numpy and glibc runs of the same
instance end with different statuses, the reference algorithm's outcome on that instance is decided by the last
bits of its libm, so a device outcome that differs from the numpy oracle there is not a device defect.
"""
import math

import numpy as np

MODE = "numpy"

_G = {name: np.frompyfunc(getattr(math, name), 1, 1) for name in ("sin", "cos", "tan", "log")}


def _f(name):
    ufunc = getattr(np, name)
    g = _G[name]

    def fn(x):
        if MODE == "glibc":
            r = g(x)
            return np.asarray(r, dtype=np.float64) if isinstance(r, np.ndarray) else float(r)
        return ufunc(x)
    fn.__name__ = name
    return fn


sin, cos, tan, log = _f("sin"), _f("cos"), _f("tan"), _f("log")


def set_mode(mode):
    global MODE
    if mode not in ("numpy", "glibc"):
        raise ValueError(mode)
    MODE = mode
