"""Multi-GPU work stealing over chunks of independent turn problems.

One process per GPU.  The work is a list of chunks (a chunk = a contiguous range
of the job's problem tickets); rank r starts with the contiguous range of chunk
ids rank_slice(r) and consumes it from the head.  Every round each rank
all-gathers ONE small int64 record -- (next-chunk counter, chunks wanted now,
launches in flight).  From the gathered vector every rank computes the same
deterministic plan: a rank that wants work takes its own head chunks first;
once its own range is empty it steals the TAIL chunk of the rank with the most
chunks left (ties: lowest rank).  The chunk queues are replicated state changed
only by that plan, so no chunk is solved twice and none is lost, and nothing
but the counters crosses GPUs (problem inputs are resident on every GPU; results
stay on the GPU that solved them).

On the GPUs a rank's chunks feed its persistent solve launch through a host
work queue (libhtp htp_queue_*): "wanted" = room below the queue's low-water
mark of published-but-unclaimed tickets.  The counters are all-gathered on a
gloo group (host TCP): the persistent launch holds every wavefront slot of its
GPU, so a collective kernel (RCCL) issued while it runs could wait for a slot
that only frees at the end of the job.  RCCL carries the timing barrier and the
result reductions outside the loop.  The loop never blocks on a solve.  All
ranks leave it in the same round.
"""
import time


def chunk_ranges(n_items, chunk):
    """[(lo, hi)] contiguous chunks of [0, n_items)."""
    chunk = max(1, int(chunk))
    return [(lo, min(n_items, lo + chunk)) for lo in range(0, n_items, chunk)]


class StealQueues:
    """Replicated per-rank chunk queues [head_r, tail_r) over chunk ids."""

    def __init__(self, n_chunks, world):
        self.world = world
        self.head = [r * n_chunks // world for r in range(world)]
        self.tail = [(r + 1) * n_chunks // world for r in range(world)]
        self.stolen = [0] * world          # chunks each rank took from others

    def remaining(self, r=None):
        if r is None:
            return sum(t - h for h, t in zip(self.head, self.tail))
        return self.tail[r] - self.head[r]

    def plan(self, free):
        """Deterministic assignment for one round; free[r] = free launch slots of
        rank r.  Returns {rank: [chunk ids]} and advances the queues."""
        out = {r: [] for r in range(self.world)}
        want = [max(0, int(f)) for f in free]
        # pass 1: own chunks from the head
        for r in range(self.world):
            while want[r] and self.head[r] < self.tail[r]:
                out[r].append(self.head[r])
                self.head[r] += 1
                want[r] -= 1
        # pass 2: idle slots steal tail chunks, one per slot, round-robin over thieves
        while any(want) and self.remaining():
            for r in range(self.world):
                if not want[r] or not self.remaining():
                    continue
                victim = max(range(self.world), key=lambda v: (self.tail[v] - self.head[v], -v))
                self.tail[victim] -= 1
                out[r].append(self.tail[victim])
                self.stolen[r] += 1
                want[r] -= 1
        return out


class WorkStealingLoop:
    """Drives one rank.  Each round: `want()` = chunks this rank can take now
    (free launch slots, or room in its device work queue), one all-gather of
    (next-chunk counter, want, in flight), the replicated plan, then
    `launch(chunk_id)` for each chunk assigned to this rank (asynchronous).
    `allgather(list[int]) -> list[list[int]]` gathers one record per rank
    (identity for one process).  Ends, on every rank in the same round, once
    no chunk is left anywhere and -- when `inflight` is given -- no launch is
    still running anywhere (a persistent device queue drains by itself)."""

    def __init__(self, n_chunks, rank, world, allgather, poll_s=5e-4):
        self.q = StealQueues(n_chunks, world)
        self.rank, self.world = rank, world
        self.allgather = allgather
        self.poll_s = poll_s
        self.rounds = 0
        self.solved = []                   # chunk ids this rank launched, in order

    def run(self, want, launch, inflight=None):
        return self.run_rounds(want, launch, None, inflight)

    def run_rounds(self, want, launch, max_rounds, inflight=None):
        """`run`, stopping after `max_rounds` rounds (None: until done); every
        rank must make the same calls."""
        k = 0
        while max_rounds is None or k < max_rounds:
            k += 1
            w = int(want())
            busy = inflight() if inflight else 0
            rec = [self.q.head[self.rank], w, int(busy)]
            g = self.allgather(rec)
            self.rounds += 1
            for r in range(self.world):     # replicated state must agree with each rank's own counter
                if g[r][0] != self.q.head[r]:
                    raise RuntimeError(f"[htp] work-stealing queues diverged: rank {r} reports next chunk "
                                       f"{g[r][0]}, replica holds {self.q.head[r]}")
            if self.q.remaining() == 0 and sum(x[2] for x in g) == 0:
                return self.solved
            mine = self.q.plan([x[1] for x in g])[self.rank]
            for cid in mine:
                launch(cid)
                self.solved.append(cid)
            if not mine:
                time.sleep(self.poll_s)
        return self.solved


class SlotPool:
    """Fixed launch slots polled by `done(slot)` (adapter for WorkStealingLoop)."""

    def __init__(self, n, start, done):
        self.free = list(range(n))
        self.busy = {}
        self.start, self.done = start, done

    def reap(self):
        for s in list(self.busy):
            if self.done(s):
                del self.busy[s]
                self.free.append(s)
        self.free.sort()
        return len(self.free)

    def launch(self, cid):
        s = self.free.pop(0)
        self.busy[s] = cid
        self.start(cid, s)

    def inflight(self):
        return len(self.busy)


def torch_allgather(dist, device, group=None):
    """All-gather of one small int64 record per rank (gloo on host tensors, or
    RCCL on device tensors) over `group` (default: the world group)."""
    import torch

    def ag(rec):
        t = torch.tensor(rec, dtype=torch.int64, device=device)
        out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(out, t, group=group)
        return [o.tolist() for o in out]
    return ag


def local_allgather(rec):
    return [list(rec)]
