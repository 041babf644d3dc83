"""Per-problem device cost of chosen config problems under A/B variants of libhtp.so (same inputs, max_cpu_time
off, an iteration cap): kernel ms, iterations, factorizations -- for solves dominated by inertia correction.

    python tools/slow_probe.py CFG MAX_ITER PID[,PID...] variant[,variant...]     ("base" = libhtp.so)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from headland_trajectory_planning_amd import _native, synth  # noqa: E402

cfg, mi = sys.argv[1], int(sys.argv[2])
pids = [int(p) for p in sys.argv[3].split(",")]
names = sys.argv[4].split(",")
insts = [synth.config_instance(cfg, p) for p in pids]
pk = _native.PackedBatch(insts)
for n in names:
    path = os.path.join(ROOT, "headland_trajectory_planning_amd", "libhtp.so" if n == "base" else f"libhtp_{n}.so")
    ctx = _native.Context(0, lib=_native.load(path))
    ctx.set_option("max_cpu_time", 0.0)
    ctx.set_option("max_iter", mi)
    for rnd in range(2):
        r = ctx.solve(pk)
        ms = ctx.lib.htp_last_kernel_ms(ctx.ctx)
    print(f"{n}: kernel {ms:.1f} ms status {r.status.tolist()} iters {r.iterations.tolist()} "
          f"n_factor {r.n_factor.tolist()} x0 {float(np.sum(r.x)):.17g}", flush=True)
