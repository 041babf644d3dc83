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
