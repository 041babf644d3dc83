"""Point formulation GPU vs host-build diagnostics (experiments only)."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from headland_trajectory_planning_amd import _native, synth  # noqa: E402
import _hostsim as H  # noqa: E402

ctx = _native.Context(0)
insts = [synth.make_points_instance(pid, N=12, M=2) for pid in range(24)]
g = ctx.solve_points(_native.PointsPackedBatch(insts))
h = H.solve_points(insts)
for k in range(len(insts)):
    print(k, "gpu", g.status[k], g.iterations[k], f"{g.objective[k]:.10g}", "host", h.status[k], h.iterations[k],
          f"{h.objective[k]:.10g}", f"dx {np.max(np.abs(g.x[k] - h.x[k])):.2e}", flush=True)
