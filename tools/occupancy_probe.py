"""Residency-cap probe (experiments only): config-D batch solved with
HTP_WG_LDS_BYTES = 0 (4 waves/CU), 48K (3), 64K (2), 96K (1); kernel time,
mean per-iteration cycles and the slowest solve's per-iteration cycles."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native  # noqa: E402
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
caps = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "49152", "65536", "98304", "0"]
pk = _native.PackedBatch(bench.make_batch(list(range(B)), "D", 16))
ctx = _native.Context(0)
ref = None
for cap in caps:
    os.environ["HTP_WG_LDS_BYTES"] = cap
    for rep in range(2):
        r = ctx.solve(pk)
        kms = ctx.last_kernel_ms()
        cyc = ctx.last_cycles(B).astype(float)
        it = np.maximum(1, r.iterations)
        k = int(np.argmax(cyc[:, 4]))
        same = "" if ref is None else f" same_x={np.array_equal(ref.x, r.x)}"
        ref = r if ref is None else ref
        print(f"cap {cap:>6}: kernel {kms:7.1f} ms  {B / kms * 1e3:7.0f} solves/s  per-iter {np.mean(cyc[:, 4] / it):.3g} "
              f"slowest {cyc[k, 4]:.3g} cyc ({r.iterations[k]} it, {cyc[k, 4] / it[k]:.3g}/it){same}", flush=True)
