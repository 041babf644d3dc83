"""Flat-import drop-in for R/obca_py/cubic_spline.py: the notebooks put this directory on
sys.path and import `cubic_spline` by its bare name (R/test/obca.ipynb:39-57); the
module object is headland_trajectory_planning_amd.obca_py.util itself."""
import os as _os
import sys as _sys

_ROOT = _os.path.abspath(_os.path.join(_os.path.dirname(__file__), "..", "..", ".."))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)
from headland_trajectory_planning_amd.obca_py import util as _m  # noqa: E402

_sys.modules[__name__] = _m
