"""Dump GPU Reeds-Shepp CSR output for seeded queries (debug aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _rs_util as U  # noqa: E402
from headland_trajectory_planning_amd import _native  # noqa: E402

ctx = _native.Context(0)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for n, seed in [(1500, 2024), (20000, 77)]:
    q = U.random_queries(n, seed=seed)
    out = ctx.rs_all_paths(q)
    keep = [k for k, v in out.items() if isinstance(v, np.ndarray) and (n <= 2000 or v.shape[0] <= 40 * n)]
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"rs_dump_{n}_{seed}.npz"), queries=q,
                        **{k: out[k] for k in keep})
print("dumped")
