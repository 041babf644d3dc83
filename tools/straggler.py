"""Straggler probe (experiments only): config-D batch, then the slowest problem
alone, per-phase cycle shares of both (is the kernel bound by its longest solve?)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native  # noqa: E402
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
insts = bench.make_batch(list(range(B)), "D", 16)
ctx = _native.Context(0)
names = ["local", "assemble", "chain", "kktsolve", "total", "errors", "linesearch", "update"]


def run(sel, tag):
    pk = _native.PackedBatch([insts[i] for i in sel])
    res = ctx.solve(pk)
    kms = ctx.last_kernel_ms()
    cyc = ctx.last_cycles(len(sel)).astype(float)
    it = np.maximum(1, res.iterations)
    per = cyc[:, 4] / it
    k = int(np.argmax(cyc[:, 4]))
    print(f"[{tag}] batch {len(sel)} kernel {kms:.1f} ms; iters mean {res.iterations.mean():.1f} max "
          f"{res.iterations.max()}; per-iter cycles mean {per.mean():.3g}; longest solve {cyc[k, 4]:.3g} cycles "
          f"({res.iterations[k]} iters, {per[k]:.3g}/iter, pid {sel[k]})", flush=True)
    sh = cyc.sum(0) / cyc[:, 4].sum()
    print(f"[{tag}] shares " + " ".join(f"{names[j]} {sh[j]:.3f}" for j in (0, 1, 2, 3, 5, 6, 7)), flush=True)
    return res, cyc


res, cyc = run(list(range(B)), "batch")
order = np.argsort(-res.iterations)
print("top iteration counts", res.iterations[order[:12]].tolist(), "statuses", res.status[order[:12]].tolist())
run([int(order[0])], "alone")
run([int(i) for i in order[:64]], "top64")
run(list(range(1024)), "1024")
