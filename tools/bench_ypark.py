"""Y-park grid-search throughput: B seeded row-enter
searches (notebook grid: 3.0..1.0 m back, 2.0..1.0 m forward, steers
0/0.1/0.2 back, 0.5/0.6 forward) in one launch, inputs resident in HBM,
kernel time from hipEvents (htp_ypark_last_ms); CPU baseline: the serial host
build of the same core on a bounded sample.  Prints one JSON line."""
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
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=32)
    args = ap.parse_args()
    import torch

    import _hostsim as H
    import _yp_util as U
    from headland_trajectory_planning_amd import _native
    dev = torch.device("cuda", 0)
    uniq = [U.scenario(s) for s in range(min(args.batch, 256))]
    probs = [uniq[i % len(uniq)] for i in range(args.batch)]
    ctx = _native.Context(0)
    pk = _native.YparkPacked(probs)
    B = pk.batch
    dv = {n: torch.from_numpy(np.ascontiguousarray(getattr(pk, n))).to(dev)
          for n in ("params", "desc", "poly_off", "vertices", "axis")}
    out = {"status": torch.empty(B, dtype=torch.int32, device=dev), "cand": torch.empty(B, dtype=torch.int32, device=dev),
           "n_path": torch.empty(B, dtype=torch.int32, device=dev), "params": torch.empty((B, 4), dtype=torch.float64, device=dev),
           "n_pose": torch.empty(B, dtype=torch.int64, device=dev),
           "path": torch.empty((B, pk.cap_path, 5), dtype=torch.float64, device=dev)}
    b = pk.struct({k: v.data_ptr() for k, v in dv.items()})
    r = _native.YpResult(*[out[k].data_ptr() for k in ("status", "cand", "n_path", "params", "n_pose", "path")])
    import ctypes
    stream = torch.cuda.current_stream().cuda_stream
    ms = []
    for it in range(args.steps + 1):
        assert ctx.lib.htp_ypark_search_batch_device(ctx.ctx, ctypes.byref(b), ctypes.byref(r), stream) == 0
        if it:
            ms.append(ctx.ypark_last_ms())
    torch.cuda.synchronize()
    kms = float(np.mean(ms))
    npose = int(out["n_pose"].sum().item())
    st = out["status"].cpu().numpy()
    n = min(args.cpu_sample, B)
    t = time.perf_counter()
    hres = H.ypark_host(probs[:n])
    cpu_s = time.perf_counter() - t
    print(json.dumps({"metric": "Y-park grid searches/s", "value": B / (kms / 1e3), "unit": "searches/s", "batch": B,
                      "kernel_ms": kms, "pose_tests_per_s": npose / (kms / 1e3),
                      "status_hist": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                      "cpu_baseline": {"value": n / cpu_s, "unit": "searches/s", "cores": 1, "kind": "port",
                                       "sample": f"first {n} searches, serial host build of csrc/ypark_core.h",
                                       "pose_tests_per_s": float(hres.n_pose.sum()) / cpu_s}}))


if __name__ == "__main__":
    main()
