"""A/B the occupancy builds (libhtp.so, libhtp_w2.so, libhtp_w4.so) on one batch, interleaved."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native, synth  # noqa: E402
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
insts = bench.make_batch(list(range(B)), 80, 6, "none", 16)
pk = _native.PackedBatch(insts)
libs = {name: _native.load(_native.LIB_PATH.replace("libhtp.so", name)) for name in ("libhtp.so", "libhtp_w2.so", "libhtp_w4.so")}
ctxs = {k: _native.Context(0, lib=v) for k, v in libs.items()}
ref = None
for rnd in range(2):
    for k, ctx in ctxs.items():
        t = time.time()
        r = ctx.solve(pk)
        dt = time.time() - t
        same = "" if ref is None else f" identical_x={np.array_equal(ref.x, r.x)}"
        if ref is None:
            ref = r
        print(f"round {rnd} {k}: {dt:.3f}s  kernel {ctx.last_kernel_ms():.1f} ms  {B / dt:.0f} solves/s{same}", flush=True)
