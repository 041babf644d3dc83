"""World-size-2 gloo test of the multi-process path (sharding + reductions)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from headland_trajectory_planning_amd import sharding, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pids = sharding.rank_pids(rank, 3)
    traj = np.stack([synth.make_instance(p, N=10, M=2)["init_traj"] for p in pids])
    el, it, ok = sharding.reduce_stats(dist, torch.device("cpu"), 1.0 + rank, 10 * (rank + 1), 3)
    out[rank] = (pids, float(traj.sum()), el, it, ok)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_and_reductions():
    world, port = 2, _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    ids = sorted(out[0][0] + out[1][0])
    assert ids == list(range(6))                      # disjoint cover of the global id range
    for r in range(world):
        assert out[r][2:] == (2.0, 30.0, 6.0)           # max time, summed iterations / converged
    # a rank's problem equals the same id generated in a single process
    solo = np.stack([synth.make_instance(p, N=10, M=2)["init_traj"] for p in out[1][0]])
    assert float(solo.sum()) == out[1][1]


# ------------------------------------------------------------- work stealing
from headland_trajectory_planning_amd import scheduler  # noqa: E402


def test_steal_plan_covers_every_chunk_once():
    rng = np.random.default_rng(3)
    for world in (1, 2, 3, 8):
        for n in (0, 1, 5, 17, 64):
            q = scheduler.StealQueues(n, world)
            seen = []
            while q.remaining():
                plan = q.plan(rng.integers(0, 3, size=world))
                for r, cids in plan.items():
                    seen += cids
            assert sorted(seen) == list(range(n))


def test_steal_plan_idle_rank_takes_victim_tail():
    q = scheduler.StealQueues(8, 2)                 # rank 0: 0..3, rank 1: 4..7
    assert q.plan([1, 0]) == {0: [0], 1: []}
    assert q.plan([0, 0]) == {0: [], 1: []}
    q.head[0] = q.tail[0]                           # rank 0 drained its own range
    assert q.plan([2, 1]) == {0: [7, 6], 1: [4]}    # own head for rank 1, tails stolen by rank 0
    assert q.stolen == [2, 0] and q.remaining() == 1


def _cpu_solver_lib():
    import ctypes
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "headland_trajectory_planning_amd", "libhtp_cpu.so")
    if not os.path.exists(so):
        import sys
        sys.path.insert(0, root)
        import __graft_entry__ as g
        import subprocess
        for out, srcs in g.CPU_LIBS.items():
            subprocess.check_call(["g++", "-O3", "-march=x86-64-v3", "-fopenmp", "-std=c++17", "-shared", "-fPIC",
                                   "-o", out] + srcs)
    lib = ctypes.CDLL(so)
    from headland_trajectory_planning_amd import _native
    lib.htp_cpu_obca_solve_range.argtypes = [ctypes.POINTER(_native.ObcaBatch), ctypes.POINTER(_native.ObcaResult),
                                             ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    lib.htp_cpu_obca_solve_range.restype = ctypes.c_int
    return lib


SMALL = dict(N=12, M=2, implement="mower")


def _steal_worker(rank, world, port, out, n_prob, chunk, slow_rank):
    """The bench's rank loop on CPU: chunk launches run in threads through the
    C++ build of the same solver core; rank `slow_rank` is slowed so the other
    rank runs dry and steals its tail chunks."""
    import ctypes
    import time
    from concurrent.futures import ThreadPoolExecutor

    import torch
    import torch.distributed as dist

    from headland_trajectory_planning_amd import _native
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = _cpu_solver_lib()
    pk = _native.PackedBatch([synth.make_instance(p, **SMALL) for p in range(n_prob)])
    res = _native.HostResults(pk.batch, pk.n_var)
    res.status[:] = -1
    b, r = pk.struct(), res.struct()
    ranges = scheduler.chunk_ranges(n_prob, chunk)
    pool = ThreadPoolExecutor(2)
    futs = {}

    def job(lo, hi):
        if rank == slow_rank:
            time.sleep(0.3)
        assert lib.htp_cpu_obca_solve_range(ctypes.byref(b), ctypes.byref(r), lo, hi - lo, 1) == 0

    def start(cid, s):
        futs[s] = pool.submit(job, *ranges[cid])

    slots = scheduler.SlotPool(2, start, lambda s: futs[s].done())
    loop = scheduler.WorkStealingLoop(len(ranges), rank, world, scheduler.torch_allgather(dist, "cpu"))
    solved = loop.run(slots.reap, slots.launch, slots.inflight)
    for f in futs.values():
        f.result()
    mine = res.status >= 0
    out[rank] = (solved, loop.q.stolen[rank], np.nonzero(mine)[0].tolist(), res.x[mine].copy(),
                 res.status[mine].copy(), res.iterations[mine].copy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_work_stealing_solve_matches_single_process():
    from headland_trajectory_planning_amd import _native
    world, port, n_prob, chunk = 2, _free_port(), 12, 1
    out = mp.Manager().dict()
    mp.spawn(_steal_worker, args=(world, port, out, n_prob, chunk, 1), nprocs=world, join=True)
    chunks = sorted(out[0][0] + out[1][0])
    assert chunks == list(range(n_prob))                 # every chunk solved exactly once
    assert out[0][1] > 0                                  # the fast rank stole from the slow one
    assert set(out[0][2]).isdisjoint(out[1][2]) and sorted(out[0][2] + out[1][2]) == list(range(n_prob))
    lib = _cpu_solver_lib()
    import ctypes
    pk = _native.PackedBatch([synth.make_instance(p, **SMALL) for p in range(n_prob)])
    ref = _native.HostResults(pk.batch, pk.n_var)
    b, r = pk.struct(), ref.struct()
    assert lib.htp_cpu_obca_solve_range(ctypes.byref(b), ctypes.byref(r), 0, n_prob, 1) == 0
    for rk in range(world):
        ids = np.array(out[rk][2])
        assert np.array_equal(out[rk][3], ref.x[ids])     # the union equals a one-process solve, bit for bit
        assert np.array_equal(out[rk][4], ref.status[ids])
        assert np.array_equal(out[rk][5], ref.iterations[ids])


# ------------------------------------------------- bench.py's multi-rank instance path
def _bench_gen_worker(rank, world, port, out):
    """bench.py's order: generate this rank's slice (fork pool, before any torch/GPU init), publish it
    to /dev/shm, then bring up the process group and assemble the global batch from every slice."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import bench
    own = bench.generate_own_slice(12, "D", rank, world, procs=2)
    bench.publish_slice(own, rank)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pk = bench.assemble_global_batch(own, rank, world, dist)
    out[rank] = (pk.batch, float(pk.traj.sum()), float(pk.obs_A.sum()), float(np.nansum(np.where(np.isfinite(pk.params), pk.params, 0.0))))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_instances_generated_before_the_process_group_and_assembled():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    world, port = 2, _free_port()
    out = mp.Manager().dict()
    mp.spawn(_bench_gen_worker, args=(world, port, out), nprocs=world, join=True)
    solo = bench.generate_own_slice(12, "D", 0, 1, procs=1)
    ref = (solo.batch, float(solo.traj.sum()), float(solo.obs_A.sum()), float(np.nansum(np.where(np.isfinite(solo.params), solo.params, 0.0))))
    assert out[0] == ref and out[1] == ref        # every rank holds the whole global batch, in pid order
