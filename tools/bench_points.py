"""Point-formulation OBCA throughput (R/obca_py/optimizer_points.py):
B seeded headland turns of the config-B shape (N=80, 6 quad obstacles, body hull)
solved in one launch, inputs resident in HBM, kernel time from hipEvents
(htp_last_kernel_ms).  CPU baseline: the same core's C++ build (libhtp_cpu.so,
htp_cpu_obca_points_solve_range, one problem per OpenMP thread) on a bounded sample of the same problems (about
20 s), threads capped at OMP_NUM_THREADS (the job's CPU share on the GPU pool).  Prints one JSON line."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=80)
    ap.add_argument("--M", type=int, default=6)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    args = ap.parse_args()
    import torch

    from headland_trajectory_planning_amd import _native, synth
    dev = torch.device("cuda", 0)
    t0 = time.time()
    uniq = [synth.make_points_instance(pid, N=args.N, M=args.M) for pid in range(min(args.batch, 512))]
    insts = [uniq[i % len(uniq)] for i in range(args.batch)]
    pk = _native.PointsPackedBatch(insts)
    gen_s = time.time() - t0
    B = pk.batch
    names = ("traj", "obs_A", "obs_b", "vertices", "params")
    dv = {n: torch.from_numpy(np.ascontiguousarray(getattr(pk, n))).to(dev) for n in names}
    out = {"x": torch.empty((B, pk.n_var), dtype=torch.float64, device=dev),
           "objective": torch.empty(B, dtype=torch.float64, device=dev),
           "status": torch.empty(B, dtype=torch.int32, device=dev),
           "iterations": torch.empty(B, dtype=torch.int32, device=dev),
           "n_factor": torch.empty(B, dtype=torch.int32, device=dev),
           "nlp_error": torch.empty(B, dtype=torch.float64, device=dev)}
    ctx = _native.Context(0)
    b = pk.struct({k: v.data_ptr() for k, v in dv.items()})
    r = _native.ObcaResult(*[out[k].data_ptr() for k in ("x", "objective", "status", "iterations", "n_factor",
                                                          "nlp_error")])
    stream = torch.cuda.current_stream().cuda_stream
    ms = []
    for it in range(args.steps + 1):
        assert ctx.lib.htp_obca_points_solve_batch_device(ctx.ctx, ctypes.byref(b), ctypes.byref(r), stream) == 0
        torch.cuda.synchronize()
        if it:
            ms.append(ctx.last_kernel_ms())
        print(f"[bench_points] step {it} {ctx.last_kernel_ms():.1f} ms", file=sys.stderr, flush=True)
    kms = float(np.mean(ms))
    st = out["status"].cpu().numpy()
    iters = out["iterations"].cpu().numpy()
    # CPU baseline: the same core on the host cores, over the first problems of the same batch, chunk by chunk
    lib = _native.cpu_lib()
    lib.htp_cpu_obca_points_solve_range.argtypes = [ctypes.POINTER(_native.ObcaPointsBatch),
                                                    ctypes.POINTER(_native.ObcaResult), ctypes.c_int64,
                                                    ctypes.c_int64, ctypes.c_int]
    lib.htp_cpu_obca_points_solve_range.restype = ctypes.c_int
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    hb = pk.struct()
    hres = _native.HostResults(pk.batch, pk.n_var)
    hr = hres.struct()
    done, t = 0, time.perf_counter()
    while done < B and time.perf_counter() - t < args.cpu_seconds:
        n = min(threads, B - done)
        assert lib.htp_cpu_obca_points_solve_range(ctypes.byref(hb), ctypes.byref(hr), done, n, threads) == 0
        done += n
    cpu_s = time.perf_counter() - t
    cit = int(hres.iterations[:done].sum())
    print(json.dumps({"metric": "point-formulation OBCA solves/s", "value": B / (kms / 1e3), "unit": "solves/s",
                      "batch": B, "N": args.N, "M": args.M, "n_vertices": pk.n_vertices, "kernel_ms": kms,
                      "success_rate": float(np.mean(np.isin(st, (0, 1)))), "mean_iters": float(iters.mean()),
                      "status_counts": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                      "gen_s": gen_s,
                      "cpu_baseline": {"value": done / cpu_s, "unit": "solves/s", "cores": threads, "kind": "port",
                                       "sample": f"first {done} problems of the same batch (N={args.N}) by "
                                                 f"libhtp_cpu.so (the same core, g++ -O3 -fopenmp, {threads} threads), "
                                                 f"{cit} iterations in {cpu_s:.1f} s"}}))


if __name__ == "__main__":
    main()
