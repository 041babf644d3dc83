"""Headline benchmark: headland-turn OBCA solves/sec (batch, N=80, 6 obs).

Workload (BASELINE.json configs[3], "D"): randomized row-spacing / heading
headlands, horizon N=80, M=6 convex obstacles, K=1 vehicle body, time-scaling
on; the config's global batch of 32768 problems split over the GPUs (strong
scaling: all 32768 on one GPU, 4096 per GPU at 8).  A "step" is one batched
solve of the whole global batch to IPOPT convergence (libhtp.so
htp_obca_solve_batch_device, inputs resident in HBM).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch GLOBAL_B] [--config D]

Execution: each rank runs ONE persistent launch (as many wavefronts as the GPU
holds at once) for all K timed steps; its waves claim problem tickets from a
host work queue (libhtp htp_queue_*), so a slow solve holds one wavefront, never
the launch, and step k+1's problems fill the chip while step k's last solves
finish.  The default of 6 timed steps measures the sustained rate: with a
persistent launch only the last step's slowest solves form a tail (a few
restoration-phase problems run >1000 IPM iterations), and 3 steps leave ~15 %
of the run in that tail (DESIGN.md s.5 gives both).  Multi-GPU: one process per GPU (torch.distributed.run); the K steps'
tickets are cut into chunks, every rank starts on its contiguous share and, once
that is empty, steals tail chunks of the busiest rank (scheduler.py: one
all-gather of next-chunk counters per round).  The timed region is bracketed by
barrier + synchronize; the max over ranks is reported.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from headland_trajectory_planning_amd import _native, costmodel, scheduler, sharding, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
OUT_KEYS = ("objective", "status", "iterations", "n_factor", "nlp_error", "n_resto")


def _gen(args):
    pid, cfg = args
    return synth.config_instance(cfg, pid)


def make_batch(pids, cfg, procs=16):
    """Instances of config `cfg` (shape, implement and turn type: synth.TURNS) for problem ids `pids`."""
    if len(pids) <= 64 or procs <= 1:
        return [_gen((p, cfg)) for p in pids]
    import multiprocessing as mp
    nproc = max(1, min(procs, (os.cpu_count() or 4)))
    with mp.get_context("fork").Pool(nproc) as pool:
        return pool.map(_gen, [(p, cfg) for p in pids], chunksize=32)


def make_global_batch(GB, cfg, rank, world, dist, procs):
    """Every rank needs every problem's inputs (a stolen chunk can be any
    problem): rank r generates its slice, the slices are exchanged through
    files under /dev/shm (not a device collective), then each rank packs all."""
    pids = sharding.rank_slice(rank, world, GB)
    insts = make_batch(pids, cfg, procs)
    turns = {}
    for inst in insts:
        turns[inst["meta"]["turn"]] = turns.get(inst["meta"]["turn"], 0) + 1
    own = _native.PackedBatch(insts)
    own.turns = turns
    if world == 1:
        return own
    tag = os.environ.get("MASTER_PORT", "0")
    path = lambda r: f"/dev/shm/htp_bench_{tag}_{r}.npz"  # noqa: E731
    np.savez(path(rank), **{k: getattr(own, k) for k in own.INPUTS if getattr(own, k) is not None})
    dist.barrier()
    parts = []
    for r in range(world):
        if r == rank:
            parts.append(own)
            continue
        z = np.load(path(r))
        p = _native.PackedBatch.__new__(_native.PackedBatch)
        p.__dict__.update(own.__dict__)
        for k in own.INPUTS:
            setattr(p, k, z[k] if k in z.files else None)
        p.batch = int(p.traj.shape[0])
        parts.append(p)
    dist.barrier()
    os.unlink(path(rank))
    out = _native.PackedBatch.concat(parts)
    out.turns = turns
    return out


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
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="D")
    ap.add_argument("--batch", type=int, default=0,
                    help="global batch split over the ranks (default: the config's BASELINE batch, D = 32768)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--gen-procs", type=int, default=16, help="CPU worker processes for instance generation")
    ap.add_argument("--chunk", type=int, default=256,
                    help="problems per work-stealing chunk (multi-GPU)")
    ap.add_argument("--max-cpu-time", type=float, default=20.0,
                    help="per-problem time limit in seconds (device wall clock), as the reference's "
                         "OBCAOptimizer.solve(max_cpu_time=20) passes to IPOPT (R/obca_py/optimizer.py:475,486); "
                         "0 = off")
    ap.add_argument("--waves", type=int, default=0,
                    help="wavefronts of the persistent launch (default: as many as are resident at once)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # ranks beyond the visible GPUs share them (a 2-rank rehearsal on a 1-GPU box;
    # RCCL refuses two ranks on one GPU, so such a rehearsal sets HTP_DIST_BACKEND=gloo)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    backend = os.environ.get("HTP_DIST_BACKEND", "nccl")
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, init_method="env://")
    dev = torch.device("cuda", local)
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    Bcfg, N, M, imp = synth.CONFIGS[args.config]
    GB = args.batch or Bcfg
    t = time.perf_counter()
    pk = make_global_batch(GB, args.config, rank, world, dist, args.gen_procs)
    gen_s = time.perf_counter() - t

    dev_in = {k: torch.from_numpy(getattr(pk, k)).to(dev) for k in pk.INPUTS if getattr(pk, k) is not None}
    ptrs = {k: v.data_ptr() for k, v in dev_in.items()}
    ctx = _native.Context(local)
    ctx.set_option("max_cpu_time", args.max_cpu_time)
    stream = torch.cuda.Stream(dev)
    x_out = torch.empty((GB, pk.n_var), dtype=torch.float64, device=dev)
    waves = args.waves or ctx.resident_waves(pk)
    gather = None
    if dist:   # host-side counters: a gloo group (see scheduler.py for why not RCCL inside the loop)
        gather = scheduler.torch_allgather(dist, "cpu", dist.new_group(backend="gloo"))

    def run_job(nsteps):
        """One persistent launch solving `nsteps` passes over the global batch:
        tickets = step-major problem ids, split into chunks that this rank
        publishes into its device work queue (all at once on one GPU; by the
        work-stealing plan on several)."""
        T = nsteps * GB
        order = np.tile(np.arange(GB, dtype=np.int32), nsteps)
        chunks = scheduler.chunk_ranges(T, args.chunk if world > 1 else T)
        outs = {k: torch.full((T,), -1 if k == "status" else 0,
                              dtype=torch.float64 if k in ("objective", "nlp_error") else torch.int32, device=dev)
                for k in OUT_KEYS}
        optr = {k: v.data_ptr() for k, v in outs.items()}
        optr["x"] = x_out.data_ptr()
        q = _native.WorkQueue(ctx, T)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        loop = scheduler.WorkStealingLoop(len(chunks), rank, world, gather or scheduler.local_allgather)
        low = 2 * waves                     # published-but-unclaimed tickets kept ahead of the waves

        def want():
            if world == 1:
                return len(chunks)
            backlog = q.published() - q.claimed()
            return max(0, -(-(low - backlog) // args.chunk))

        def publish(cid):
            lo, hi = chunks[cid]
            q.publish(order[lo:hi])

        try:
            if world > 1:                   # initial backlog from the own range before the launch
                loop.run_rounds(want, publish, 1)
            ev0.record(stream)
            ctx.solve_queue_device(pk, ptrs, q, optr, stream=stream.cuda_stream, waves=waves)
            ev1.record(stream)
            loop.run(want, publish)
        finally:
            q.close()                       # every wave of the launch retires once the queue is drained
        torch.cuda.synchronize(dev)
        n = q.published()
        st = outs["status"][:n].cpu().numpy()
        return dict(loop=loop, ms=ev0.elapsed_time(ev1), n=n, status=st, iters=outs["iterations"][:n].cpu().numpy(),
                    n_resto=outs["n_resto"][:n].cpu().numpy(), q=q)

    if args.warmup:
        run_job(args.warmup)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    job = run_job(args.steps)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    timed_st, timed_it, timed_nr = job["status"], job["iters"], job["n_resto"]
    if (timed_st < 0).any():
        raise RuntimeError(f"[bench] {(timed_st < 0).sum()} published tickets were not solved")
    it_sum = float(timed_it.sum())
    ok_sum = float(np.isin(timed_st, [0, 1]).sum())
    loop = job["loop"]
    elapsed, all_iters, all_ok = sharding.reduce_stats(dist, red_dev, elapsed, it_sum, ok_sum)
    n_solved = sharding.sum_ints(dist, red_dev, [job["n"], len(loop.solved), loop.q.stolen[rank]])
    if n_solved[0] != GB * args.steps:
        raise RuntimeError(f"[bench] work-stealing lost or duplicated problems: {n_solved[0]} solved, "
                           f"{GB * args.steps} queued")
    total_solves = GB * args.steps
    value = total_solves / elapsed
    mine = timed_st >= 0

    topt = pk.time_opt
    biter = int(costmodel.bytes_per_iteration(N, M, int(pk.K), int(topt), [int(e) for e in pk.obs_edges],
                                              [int(e) for e in pk.body_edges]))
    # Roofline of the dominant kernel (obca_solve_kernel): one persistent launch
    # per rank solves the whole timed job, so bytes per launch / launch duration
    # (HIP events on the launch stream) is the job rate of this GPU.
    kernel_ms = job["ms"]
    achieved = biter * it_sum / (kernel_ms * 1e-3) / 1e9
    traffic = None
    # HBM bytes per problem-iteration measured with rocprofv3 FETCH_SIZE/WRITE_SIZE
    # passes (tools/gpu_pmc.sh -> profiles/*_traffic.json) for this workload, scaled
    # to the same iteration count as `achieved`.
    tf = os.environ.get("HTP_TRAFFIC_JSON", os.path.join(ROOT, "profiles", f"r02_traffic_{args.config}.json"))
    if tf and os.path.exists(tf):
        tj = json.load(open(tf))
        if tj.get("workload") == args.config and tj.get("bytes_per_problem_iter") \
                and tj.get("solver_sha") == _native.core_sha():
            traffic = tj["bytes_per_problem_iter"] * it_sum / (kernel_ms * 1e-3) / 1e9
    mfma = None
    mf = os.environ.get("HTP_MFMA_JSON", os.path.join(ROOT, "profiles", f"r02_mfma_{args.config}.json"))
    if mf and os.path.exists(mf):
        mj = json.load(open(mf))
        if mj.get("solver_sha") == _native.core_sha():
            mfma = {k: mj[k] for k in ("mfma_f64_per_problem_iter", "mfma_busy_frac", "mfma_f64_tflops", "mfma_f64_frac_of_peak", "valu_per_problem_iter")
                    if k in mj}

    line = {
        "metric": "headland-turn solves/sec (batch, N=80, 6 obs) at 1/2/4/8 MI355X",
        "value": value, "unit": "solves/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (Philox-seeded orchard headlands, synth.py)",
        "config": {"workload": f"config {args.config}: global batch {GB} split over {world} GPU(s), "
                               f"N={N} horizon, M={M} obstacles, K={pk.K} bodies ({imp}), time-opt on; "
                               f"IPOPT-restated IPM to tol 1e-8, max_cpu_time {args.max_cpu_time:g} s per problem",
                   "global_batch": GB, "N": N, "M": M, "K": pk.K, "turn_types": synth.TURNS[args.config],
                   "turn_histogram_rank0_slice": getattr(pk, "turns", None),
                   "parallelism": f"problem-sharded x{world}, work stealing"},
        "execution": {"launch": f"one persistent launch per GPU ({waves} wavefronts) fed by a host work queue",
                      "chunk": args.chunk if world > 1 else GB * args.steps, "chunks_rank0": len(loop.solved),
                      "stolen_chunks_total": n_solved[2], "rounds_rank0": loop.rounds, "gen_s": gen_s},
        "solver": {"success_rate": all_ok / total_solves, "mean_iters": all_iters / total_solves,
                   "status_counts_rank0": {str(k): int(v) for k, v in zip(*np.unique(timed_st, return_counts=True))},
                   "restorations_rank0": int(timed_nr[mine].sum()),
                   "p99_iters_rank0": float(np.percentile(timed_it[mine], 99)) if mine.any() else None,
                   "max_iters_rank0": int(timed_it[mine].max()) if mine.any() else None},
        "roofline": {"bound": "latency", "model": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "limiter": "per-iteration latency of one wavefront per problem (1 wave/SIMD); the slowest "
                                "solve of the last step sets the tail",
                     "bytes_per_iter_per_problem": biter, "kernel_ms_avg": kernel_ms,
                     "traffic_unit": "GB/s (PMC bytes per problem-iteration x iterations / launch time)",
                     "mfma": mfma},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(pk, args.cpu_budget)
    if rank == 0:
        print(json.dumps(line, default=float), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
