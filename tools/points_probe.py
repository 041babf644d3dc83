"""Point-formulation phase profile (experiments): solve make_points_instance(pid, N, M) for pids
[0, B) on the GPU and print the per-phase cycle shares, cycles per iteration and the slowest
problems (htp_last_cycles).   python tools/points_probe.py [B] [N] [M]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 80
M = int(sys.argv[3]) if len(sys.argv) > 3 else 6
pk = _native.PointsPackedBatch([synth.make_points_instance(p, N=N, M=M) for p in range(B)])
ctx = _native.Context(0)
for rep in range(2):
    r = ctx.solve_points(pk)
    ms = ctx.last_kernel_ms()
cyc = ctx.last_cycles(B).astype(float)
tot = cyc[:, 4].sum()
names = ["local", "assemble", "chain", "kktsolve", "total", "errors", "linesearch", "update"]
it = np.maximum(1, r.iterations)
print(f"B={B} N={N} M={M} kernel {ms:.1f} ms -> {B / (ms / 1e3):.0f} solves/s; iters mean {r.iterations.mean():.1f} "
      f"max {r.iterations.max()}; status {np.bincount(r.status, minlength=9)}")
print("cycle share: " + " ".join(f"{names[j]} {cyc[:, j].sum() / tot:.3f}" for j in (0, 1, 2, 3, 5, 6, 7)))
print(f"cycles per iteration: mean over problems {np.mean(cyc[:, 4] / it):.3g}; "
      f"solved-only {np.mean((cyc[:, 4] / it)[r.n_resto == 0]):.3g}; with restoration {np.mean((cyc[:, 4] / it)[r.n_resto > 0]) if (r.n_resto > 0).any() else 0:.3g}")
slow = np.argsort(-cyc[:, 4])[:8]
print("slowest:", [(int(p), int(r.status[p]), int(r.iterations[p]), int(r.n_resto[p]), f"{cyc[p, 4]:.3g}") for p in slow])
