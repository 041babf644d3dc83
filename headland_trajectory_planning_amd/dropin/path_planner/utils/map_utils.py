"""Flat-import drop-in for R/path_planner/utils/map_utils.py: the notebooks put this directory on
sys.path and import `map_utils` by its bare name (R/test/obca.ipynb:39-57); the
module object is headland_trajectory_planning_amd.path_planner.map_utils itself."""
import os as _os
import sys as _sys

_ROOT = _os.path.abspath(_os.path.join(_os.path.dirname(__file__), "..", "..", "..", ".."))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)
from headland_trajectory_planning_amd.path_planner import map_utils as _m  # noqa: E402

_sys.modules[__name__] = _m
