"""MI355X-native batched headland-turn trajectory planner.

Drop-in for the OBCA hot path of AgRoboticsResearch/headland_trajectory_planning
(R/obca_py/optimizer.py: OBCAOptimizer) backed by hand-written HIP kernels for
gfx950 behind a C ABI (include/htp.h, libhtp.so).
"""
__version__ = "0.1.0"
