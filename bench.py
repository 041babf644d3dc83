"""Headline benchmark: headland-turn OBCA solves/sec (batch, N=80, 6 obs).

Workload (BASELINE.json configs[3], "D"): randomized row-spacing / heading
headlands, horizon N=80, M=6 convex obstacles, K=1 vehicle body, time-scaling
on; the config's global batch of 32768 problems split over the GPUs (strong
scaling: all 32768 on one GPU, 4096 per GPU at 8).  A "step" is one batched
solve of all of a rank's problems to IPOPT convergence (libhtp.so
htp_obca_solve_batch_device, inputs resident in HBM).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch GLOBAL_B] [--config D]

Multi-GPU: launched by torch.distributed.run, one process per GPU; each rank
solves its own contiguous slice of problem ids (no data-path collective); the
timed region is bracketed by barrier + synchronize and the max over ranks is
reported.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from headland_trajectory_planning_amd import _native, costmodel, sharding, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def _gen(args):
    pid, N, M, imp = args
    return synth.make_instance(pid, N=N, M=M, implement=imp)


def make_batch(pids, N, M, imp, procs=16):
    if len(pids) <= 64 or procs <= 1:
        return [_gen((p, N, M, imp)) for p in pids]
    import multiprocessing as mp
    nproc = max(1, min(procs, (os.cpu_count() or 4)))
    with mp.get_context("fork").Pool(nproc) as pool:
        return pool.map(_gen, [(p, N, M, imp) for p in pids], chunksize=32)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(pk, budget_s=20.0):
    """SURVEY 8(d) CPU baseline: the build's own C++ implementation of the same
    solver (csrc/htp_cpu.cpp = obca_core.h compiled with g++ -O3 -fopenmp, one
    problem per OpenMP thread, dynamic schedule) on this box's host cores, over
    the first problems of the same packed workload, in chunks until the budget."""
    import ctypes
    so = os.path.join(ROOT, "headland_trajectory_planning_amd", "libhtp_cpu.so")
    lib = ctypes.CDLL(so)
    lib.htp_cpu_obca_solve_range.argtypes = [ctypes.POINTER(_native.ObcaBatch), ctypes.POINTER(_native.ObcaResult),
                                             ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    lib.htp_cpu_obca_solve_range.restype = ctypes.c_int
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        threads = os.cpu_count() or 1
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    res = _native.HostResults(pk.batch, pk.n_var)
    b, r = pk.struct(), res.struct()
    t0 = time.perf_counter()
    done, chunk = 0, threads
    while done < pk.batch and time.perf_counter() - t0 < budget_s:
        n = min(chunk, pk.batch - done)
        if lib.htp_cpu_obca_solve_range(ctypes.byref(b), ctypes.byref(r), done, n, threads) != 0:
            raise RuntimeError("htp_cpu_obca_solve_range failed")
        done += n
    dt = time.perf_counter() - t0
    st = res.status[:done]
    return {"value": done / dt, "unit": "solves/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
            "success_rate": float(np.isin(st, [0, 1]).mean()) if done else None,
            "sample": f"first {done} problems (pids 0..{done - 1}) of the same workload solved to convergence by "
                      f"libhtp_cpu.so (obca_core.h, g++ -O3 -fopenmp, {threads} threads, one problem per thread) "
                      f"in {dt:.1f} s; {int(res.iterations[:done].sum())} IPM iterations. History: the reference's "
                      f"CasADi/IPOPT solve of its N=66 notebook problem took 0.213 s setup + 2.662 s solve "
                      f"(R/test/obca.ipynb:400,405; 0.35 solves/s/core, unknown CPU)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="D")
    ap.add_argument("--batch", type=int, default=0,
                    help="global batch split over the ranks (default: the config's BASELINE batch, D = 32768)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--gen-procs", type=int, default=16, help="CPU worker processes for instance generation")
    ap.add_argument("--streams", type=int, default=2,
                    help="batches in flight: consecutive steps alternate over this many HIP streams (each with its "
                         "own solver context and workspace), so a batch's slowest solves overlap the next batch")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", init_method="env://")
    dev = torch.device("cuda", local)

    Bcfg, N, M, imp = synth.CONFIGS[args.config]
    GB = args.batch or Bcfg
    pids = sharding.rank_slice(rank, world, GB)
    B = len(pids)
    t = time.perf_counter()
    insts = make_batch(pids, N, M, imp, args.gen_procs)
    gen_s = time.perf_counter() - t
    pk = _native.PackedBatch(insts)

    def dt_(a):
        return None if a is None else torch.from_numpy(a).to(dev)

    dev_in = {k: dt_(getattr(pk, k)) for k in ("traj", "obs_A", "obs_b", "body_G", "body_g", "params",
                                                "init_control", "init_mu", "init_lambda")}
    ptrs = {k: (v.data_ptr() if v is not None else None) for k, v in dev_in.items()}
    # one output set, solver context (device workspace) and HIP stream per batch in flight
    nstr = max(1, args.streams)
    lanes = []
    for _ in range(nstr):
        o = dict(x=torch.empty((B, pk.n_var), dtype=torch.float64, device=dev),
                 objective=torch.empty(B, dtype=torch.float64, device=dev),
                 status=torch.empty(B, dtype=torch.int32, device=dev),
                 iterations=torch.empty(B, dtype=torch.int32, device=dev),
                 n_factor=torch.empty(B, dtype=torch.int32, device=dev),
                 nlp_error=torch.empty(B, dtype=torch.float64, device=dev),
                 n_resto=torch.empty(B, dtype=torch.int32, device=dev))
        lanes.append(dict(out=o, ptr={k: v.data_ptr() for k, v in o.items()}, ctx=_native.Context(local),
                          stream=torch.cuda.Stream(dev)))

    def step(k):
        ln = lanes[k % nstr]
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record(ln["stream"])
        ln["ctx"].solve_device(pk, ptrs, ln["ptr"], stream=ln["stream"].cuda_stream)
        ev1.record(ln["stream"])
        return ev0, ev1

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs.append(step(args.warmup + k))
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in evs]   # per launch, on the stream it was launched on
    last = lanes[(args.warmup + args.steps - 1) % nstr]["out"]
    it_np = last["iterations"].cpu().numpy()
    st_np = last["status"].cpu().numpy()
    nr_np = last["n_resto"].cpu().numpy()
    elapsed, all_iters, all_ok = sharding.reduce_stats(dist, dev, elapsed, float(it_np.sum()),
                                                       float(np.isin(st_np, [0, 1]).sum()))
    total_solves = GB * args.steps
    value = total_solves / elapsed

    topt = pk.time_opt
    biter = int(costmodel.bytes_per_iteration(N, M, int(pk.K), int(topt), [int(e) for e in pk.obs_edges],
                                              [int(e) for e in pk.body_edges]))
    launch_bytes = biter * float(it_np.sum())     # this rank's launch
    avg_ms = float(np.mean(kernel_ms))
    achieved = launch_bytes / (avg_ms * 1e-3) / 1e9
    job_achieved = launch_bytes * args.steps / elapsed / 1e9   # all launches of this rank over the timed region
    traffic = None
    # HBM bytes per launch measured with rocprofv3 PMC passes (tools/profile.sh ->
    # profiles/*_traffic.json) for this exact workload; scaled to this launch's
    # iteration count (bytes per problem-iteration x iterations).
    tf = os.environ.get("HTP_TRAFFIC_JSON", os.path.join(ROOT, "profiles", "r02_traffic.json"))
    if tf and os.path.exists(tf):
        tj = json.load(open(tf))
        if tj.get("workload") == args.config and tj.get("batch") == B and tj.get("bytes_per_problem_iter") \
                and tj.get("solver_sha") == _native.core_sha():
            traffic = tj["bytes_per_problem_iter"] * float(it_np.sum())

    line = {
        "metric": "headland-turn solves/sec (batch, N=80, 6 obs) at 1/2/4/8 MI355X",
        "value": value, "unit": "solves/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (Philox-seeded orchard headlands, synth.py)",
        "config": {"workload": f"config {args.config}: global batch {GB} split over {world} GPU(s) ({B} on rank 0), "
                               f"N={N} horizon, M={M} obstacles, K={pk.K} bodies ({imp}), time-opt on; "
                               f"IPOPT-restated IPM to tol 1e-8",
                   "batch_per_gpu": B, "global_batch": GB, "N": N, "M": M, "K": pk.K,
                   "parallelism": f"problem-sharded x{world}"},
        "pipelining": f"{nstr} batch(es) in flight on {nstr} HIP stream(s); each step solves its whole batch",
        "solver": {"success_rate": all_ok / GB, "mean_iters": all_iters / GB,
                   "restorations_rank0": int(nr_np.sum()), "problems_with_restoration_rank0": int((nr_np > 0).sum()),
                   "p99_iters_rank0": float(np.percentile(it_np, 99)), "max_iters_rank0": int(it_np.max()),
                   "gen_s": gen_s},
        "roofline": {"bound": "hbm", "limiter": "latency: one wavefront per problem, the slowest solve sets the launch",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "bytes_per_iter_per_problem": biter, "kernel_ms_avg": avg_ms,
                     "job_achieved_GBps": job_achieved, "job_frac": job_achieved / HBM_PEAK_GBS},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(pk, args.cpu_budget)
    if rank == 0:
        print(json.dumps(line, default=float), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
