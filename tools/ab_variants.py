"""A/B timing of libhtp_<name>.so variants on one config-D batch, interleaved
(experiments only).  python tools/ab_variants.py B name1 name2 ..."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native  # noqa: E402
import bench  # noqa: E402

B = int(sys.argv[1])
names = sys.argv[2:]
insts = bench.make_batch(list(range(B)), "D", 16)
pk = _native.PackedBatch(insts)
ctxs = {}
for n in names:
    path = _native.LIB_PATH if n == "base" else _native.LIB_PATH.replace("libhtp.so", f"libhtp_{n}.so")
    ctxs[n] = _native.Context(0, lib=_native.load(path))
ref = None
for rnd in range(2):
    for k, ctx in ctxs.items():
        t = time.time()
        r = ctx.solve(pk)
        dt = time.time() - t
        ok = "" if ref is None else f" max|dx|={np.max(np.abs(ref.x - r.x)):.2e} st_eq={np.array_equal(ref.status, r.status)}"
        if ref is None:
            ref = r
        print(f"round {rnd} {k}: kernel {ctx.last_kernel_ms():.1f} ms  {B / (ctx.last_kernel_ms() / 1e3):.0f} solves/s "
              f"iters {r.iterations.mean():.2f}{ok}", flush=True)
