"""Config E diagnosis (experiments): solve pids in chunks with a device wall-clock limit so
slow or stuck problems stop with Maximum_CpuTime_Exceeded; print their pids, iterations and
restoration counts.   python tools/e_probe.py CHUNK NCHUNK LIMIT_S"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native  # noqa: E402
import bench  # noqa: E402

chunk, nchunk, lim = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
ctx = _native.Context(0)
ctx.set_option("max_cpu_time", lim)
for k in range(nchunk):
    pids = list(range(k * chunk, (k + 1) * chunk))
    pk = _native.PackedBatch(bench.make_batch(pids, "E", 16))
    t = time.time()
    r = ctx.solve(pk)
    slow = [(pids[j], int(r.status[j]), int(r.iterations[j]), int(r.n_resto[j])) for j in range(len(pids))
            if r.status[j] not in (0, 1)]
    print(f"chunk {k}: {time.time() - t:.1f}s kernel {ctx.last_kernel_ms():.0f} ms status {np.bincount(r.status, minlength=9)} "
          f"iters mean {r.iterations.mean():.1f} max {r.iterations.max()} | not converged {slow[:12]}", flush=True)
