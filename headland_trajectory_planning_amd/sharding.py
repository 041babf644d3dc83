"""Problem sharding across GPUs (one process per GPU).

Problems are independent, so rank r of W solves a contiguous slice of the
global id range [0, B) (rank_slice: sizes differ by at most one).  Problem ids seed the
generator (Philox key [20251015, pid]), so a problem is identical at any world
size.  rank_slice is each rank's starting share; scheduler.py moves tail chunks
between ranks (work stealing over an all-gather of next-chunk counters).  The
other collectives are the timing barrier and these tiny reductions (RCCL on
GPUs, gloo on CPU); no problem data crosses GPUs.
"""


def rank_pids(rank, per_rank):
    return list(range(rank * per_rank, (rank + 1) * per_rank))


def rank_slice(rank, world, total):
    """Contiguous slice of [0, total) for `rank` of `world` (balanced to +-1)."""
    lo = rank * total // world
    hi = (rank + 1) * total // world
    return list(range(lo, hi))


def reduce_stats(dist, device, elapsed, iters_sum, ok_sum):
    """-> (max elapsed over ranks, total iterations, total converged)."""
    if dist is None:
        return float(elapsed), float(iters_sum), float(ok_sum)
    import torch
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([float(iters_sum), float(ok_sum)], dtype=torch.float64, device=device)
    dist.all_reduce(s)
    return float(t.item()), float(s[0].item()), float(s[1].item())


def sum_ints(dist, device, vals):
    """Sum of a few integers over ranks."""
    if dist is None:
        return [int(v) for v in vals]
    import torch
    t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return [int(v) for v in t.tolist()]
