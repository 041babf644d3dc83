"""Full-size oracle fixtures (tests/golden/obca_full/<name>.npz, their own instances) solved under A/B variants of
libhtp.so: status, iterations, restorations, kernel ms -- to find which change moves a chaotic solve.

    python tools/fixture_probe.py NAME[,NAME...] variant[,variant...]     ("base" = libhtp.so)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

from _fixture_io import load_instance  # noqa: E402
from headland_trajectory_planning_amd import _native  # noqa: E402

names = sys.argv[1].split(",")
variants = sys.argv[2].split(",")
for n in names:
    g = np.load(os.path.join(ROOT, "tests", "golden", "obca_full", f"{n}.npz"))
    pk = _native.PackedBatch([load_instance(g)])
    print(f"{n}: oracle status {int(g['status'])} iters {int(g['iters'])} resto {int(g['n_resto'])}", flush=True)
    for v in variants:
        path = os.path.join(ROOT, "headland_trajectory_planning_amd", "libhtp.so" if v == "base" else f"libhtp_{v}.so")
        ctx = _native.Context(0, lib=_native.load(path))
        ctx.set_option("max_cpu_time", 0.0)
        r = ctx.solve(pk)
        print(f"  {v}: status {int(r.status[0])} iters {int(r.iterations[0])} resto {int(r.n_resto[0])} "
              f"n_factor {int(r.n_factor[0])} kernel {ctx.lib.htp_last_kernel_ms(ctx.ctx):.0f} ms", flush=True)
