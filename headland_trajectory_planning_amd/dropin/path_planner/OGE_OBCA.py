"""Flat-import drop-in for R/path_planner/OGE_OBCA.py: the notebooks put this directory on
sys.path and import `OGE_OBCA` by its bare name (R/test/obca.ipynb:39-57); the
module object is headland_trajectory_planning_amd.path_planner.OGE_OBCA itself."""
import os as _os
import sys as _sys

_ROOT = _os.path.abspath(_os.path.join(_os.path.dirname(__file__), "..", "..", ".."))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)
from headland_trajectory_planning_amd.path_planner import OGE_OBCA as _m  # noqa: E402

_sys.modules[__name__] = _m
