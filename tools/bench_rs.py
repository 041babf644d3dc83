"""Reeds-Shepp batch throughput: calc_all_paths for B pose
pairs on one GPU, buffers resident in HBM, timed with hipEvents around the
five launches (htp_rs_last_ms) and with the host clock.

    python tools/bench_rs.py [--batch 65536] [--steps 5] [--cpu-budget 10]

Prints one JSON line.  Output bytes per launch = 61 B per path (lengths,
ctypes, L, offset) + 33 B per sample (x, y, yaw, cs, direction)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    args = ap.parse_args()
    import torch

    import _rs_util as U
    from headland_trajectory_planning_amd import _native
    dev = torch.device("cuda", 0)
    q = U.random_queries(args.batch, seed=1)
    ctx = _native.Context(0)
    sizes = ctx.rs_all_paths(q[:1])  # warm the library
    t = time.perf_counter()
    ref = ctx.rs_all_paths(q)
    host_api_s = time.perf_counter() - t
    P, Q = ref["n_paths"], ref["n_points"]
    B = args.batch
    qd = torch.from_numpy(q).to(dev)
    bufs = {"path_offsets": torch.empty(B + 1, dtype=torch.int64, device=dev),
            "status": torch.empty(B, dtype=torch.int32, device=dev),
            "lengths": torch.empty((P, 5), dtype=torch.float64, device=dev),
            "ctypes": torch.empty((P, 5), dtype=torch.int8, device=dev),
            "L": torch.empty(P, dtype=torch.float64, device=dev),
            "point_offsets": torch.empty(P + 1, dtype=torch.int64, device=dev),
            "directions": torch.empty(Q, dtype=torch.int8, device=dev)}
    for k in ("x", "y", "yaw", "cs"):
        bufs[k] = torch.empty(Q, dtype=torch.float64, device=dev)
    ptrs = {k: v.data_ptr() for k, v in bufs.items()}
    totals = torch.zeros(2, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)

    def step():
        ctx.rs_all_paths_device(B, qd.data_ptr(), ptrs, (P, Q), totals.data_ptr(), stream=s.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        torch.cuda.synchronize(dev)
        ms.append(ctx.rs_last_ms())
    el = time.perf_counter() - t0
    assert totals.cpu().tolist() == [P, Q]
    out_bytes = 61 * P + 33 * Q
    kms = float(np.mean(ms))
    line = {"metric": "reeds-shepp calc_all_paths queries/s", "value": B * args.steps / el, "unit": "queries/s",
            "batch": B, "paths": P, "samples": Q, "ms_per_step": el / args.steps * 1e3, "kernel_ms_avg": kms,
            "paths_per_s": P / (kms * 1e-3), "samples_per_s": Q / (kms * 1e-3),
            "output_GBps": out_bytes / (kms * 1e-3) / 1e9, "host_api_s": host_api_s}
    if args.cpu_budget > 0:
        from oracle import reeds_shepp as ors
        t = time.perf_counter()
        n = 0
        while time.perf_counter() - t < args.cpu_budget and n < B:
            ors.calc_all_paths(*[float(v) for v in q[n]])
            n += 1
        dt = time.perf_counter() - t
        line["cpu_baseline"] = {"value": n / dt, "unit": "queries/s", "cores": 1, "kind": "port",
                                "sample": f"first {n} queries through oracle/reeds_shepp.py (pure Python, "
                                          f"same arithmetic as the reference) in {dt:.1f} s"}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
