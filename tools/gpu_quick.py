"""Quick GPU timing probe: solves one config batch and prints stats."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "B"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else None
b, N, M, imp = synth.CONFIGS[cfg]
import bench
batch = batch or b
t = time.time()
insts = bench.make_batch(list(range(batch)), cfg, 16)
print(f"gen {batch} problems: {time.time() - t:.1f}s", flush=True)
pk = _native.PackedBatch(insts)
ctx = _native.Context(0)
for rep in range(2):
    t = time.time()
    res = ctx.solve(pk)
    dt = time.time() - t
    print(f"rep {rep}: wall {dt:.3f}s kernel {ctx.last_kernel_ms():.1f}ms  solves/s {batch / dt:.1f} "
          f"(kernel-only {batch / (ctx.last_kernel_ms() / 1e3):.1f})", flush=True)
print("status counts", np.bincount(res.status, minlength=6), "iters mean", res.iterations.mean(),
      "p99", np.percentile(res.iterations, 99), "max", res.iterations.max(), "nfactor mean", res.n_factor.mean())
cyc = ctx.last_cycles(batch).astype(float)
tot = cyc[:, 4].sum()
names = ["local", "assemble", "chain", "kktsolve", "total", "errors", "linesearch", "update"]
print("cycle share:", " ".join(f"{names[k]} {cyc[:, k].sum() / tot:.3f}" for k in (0, 1, 2, 3, 5, 6, 7)),
      "| other %.3f" % (1 - sum(cyc[:, k].sum() for k in (0, 1, 2, 3, 5, 6, 7)) / tot),
      "| per-iter cycles %.3g" % (cyc[:, 4] / np.maximum(1, res.iterations)).mean())
