"""Stage-chain sub-step cycles (experiments only; libhtp_prof.so = -DHTP_PROF_ON):
per IPM iteration, riccati_factor steps (0 prefetch/copy, 1 PJx/PB, 2 Rt/St/AtPA,
3 chol/K, 5 P update) and riccati_solve (6 backward, 7 forward) for the straggler
alone and for a 1024-problem round."""
import sys

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native  # noqa: E402
import bench  # noqa: E402

insts = bench.make_batch(list(range(1024)), 80, 6, "none", 16)
ctx = _native.Context(0, lib=_native.load(_native.LIB_PATH.replace("libhtp.so", "libhtp_prof.so")))
names = {0: "prefetch/copy", 1: "PJx/PB", 2: "Rt/St/AtPA", 3: "chol/K", 5: "P update", 6: "solve back",
         7: "solve fwd"}
for tag, sel in (("alone", [663]), ("1024", list(range(1024)))):
    pk = _native.PackedBatch([insts[i] for i in sel])
    res = ctx.solve(pk)
    cyc = ctx.last_cycles(len(sel)).astype(float)
    it = np.maximum(1, res.iterations).astype(float)
    nf = np.maximum(1, res.n_factor).astype(float)
    print(f"[{tag}] kernel {ctx.last_kernel_ms():.1f} ms iters {res.iterations.mean():.1f} nfactor "
          f"{res.n_factor.mean():.1f} total/iter {np.mean(cyc[:, 4] / it):.3g}", flush=True)
    for k, nm in names.items():
        print(f"[{tag}]   {nm:14s} per iter {np.mean(cyc[:, k] / it):.3g}  per factor {np.mean(cyc[:, k] / nf):.3g}"
              f"  per stage-step {np.mean(cyc[:, k] / nf) / 79:.3g}", flush=True)
