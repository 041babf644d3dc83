import sys
import numpy as np
sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native  # noqa: E402
import bench  # noqa: E402
B = 4096
pk = _native.PackedBatch(bench.make_batch(list(range(B)), "D", 16))
res = {}
for name in ("libhtp.so", "libhtp_w4.so"):
    ctx = _native.Context(0, lib=_native.load(_native.LIB_PATH.replace("libhtp.so", name)))
    r = ctx.solve(pk)
    res[name] = r
    print(name, "status", np.bincount(r.status, minlength=6), "iters mean", r.iterations.mean(), "max", r.iterations.max(),
          "obj mean", r.objective.mean(), "kernel ms", ctx.last_kernel_ms(), flush=True)
a, b = res["libhtp.so"], res["libhtp_w4.so"]
d = np.abs(a.x[:, :400] - b.x[:, :400]).max(axis=1)
print("state max diff: median", np.median(d), "max", d.max(), "n>1e-4", int((d > 1e-4).sum()),
      "iters equal", int((a.iterations == b.iterations).sum()))
