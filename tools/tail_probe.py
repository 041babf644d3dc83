"""How much of a persistent launch is tail: solve config D's batch once (htp_obca_solve_batch, tickets claimed in
order by 1 024 wavefronts), read every problem's cycle count, and replay the claim order as list scheduling
(each ticket goes to the first free wavefront).  makespan / (sum / waves) - 1 is the tail + imbalance share.

Usage: python tools/tail_probe.py [config] [batch] [cache_dir] [save.npz]
The optional npz keeps every problem's cycle count, iterations and status for tools/scale_projection.py."""
import heapq
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from headland_trajectory_planning_amd import _native  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "D"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
cache = sys.argv[3] if len(sys.argv) > 3 else None
bench.SCENE = "orchard"
own = bench.cached_own_slice(B, cfg, 0, 1, 16, cache)   # generated (forked) before any GPU call
ctx = _native.Context(0)
ctx.set_option("max_cpu_time", 20.0)
res = ctx.solve(own)
kms = ctx.last_kernel_ms()
cyc = ctx.last_cycles(B)[:, 4].astype(np.float64)
waves = ctx.resident_waves(own)
free = [0.0] * waves
heapq.heapify(free)
for c in cyc:
    heapq.heappush(free, heapq.heappop(free) + c)
makespan = max(free)
mean = cyc.sum() / waves
order = np.argsort(-cyc)
out = {"config": cfg, "batch": B, "waves": waves, "kernel_ms": kms,
       "solves_per_s": B / (kms * 1e-3), "mean_iters": float(res.iterations.mean()),
       "sum_cycles_over_waves": mean, "simulated_makespan_cycles": makespan,
       "tail_share": makespan / mean - 1.0,
       "longest_solves": [{"pid": int(p), "cycles": float(cyc[p]), "iterations": int(res.iterations[p]),
                           "status": int(res.status[p])} for p in order[:8]],
       "cycles_per_ms": makespan / kms}
print(json.dumps(out, indent=1))
if len(sys.argv) > 4:
    np.savez_compressed(sys.argv[4], cycles=cyc, iterations=res.iterations, status=res.status, waves=waves,
                        kernel_ms=kms, cycles_per_ms=makespan / kms)
