"""GPU: the persistent work-queue launch that bench.py runs (htp_queue_* + htp_obca_solve_queue_device).

* tickets published AFTER the launch, in two batches with a delay, as a permuted problem list with
  repeats: every ticket's status / iterations / objective / restorations and every x row equal, bit
  for bit, the static-range solve of the same problems (same kernel, one wave per problem);
* closing early: tickets that were never published stay unwritten and the launch drains;
* launches of one context are ordered: a second launch (any stream) waits for the first; only a launch behind
  a queue launch whose queue is still open is rejected (it would wait forever)."""
import time

import numpy as np
import pytest

from headland_trajectory_planning_amd import _native, synth

pytestmark = pytest.mark.gpu

KEYS = ("objective", "status", "iterations", "n_factor", "nlp_error", "n_resto")


def _setup(nprob=12):
    import torch
    insts = [synth.make_instance(pid, N=20, M=3, implement="mower") for pid in range(nprob)]
    pk = _native.PackedBatch(insts)
    dev = torch.device("cuda", 0)
    dev_in = {k: torch.from_numpy(getattr(pk, k)).to(dev) for k in pk.INPUTS if getattr(pk, k) is not None}
    return torch, pk, dev, dev_in, {k: v.data_ptr() for k, v in dev_in.items()}


def _outs(torch, dev, T, n_var, nprob):
    outs = {k: torch.full((T,), -1 if k == "status" else 0,
                          dtype=torch.float64 if k in ("objective", "nlp_error") else torch.int32, device=dev)
            for k in KEYS}
    x = torch.zeros((nprob, n_var), dtype=torch.float64, device=dev)
    ptr = {k: v.data_ptr() for k, v in outs.items()}
    ptr["x"] = x.data_ptr()
    return outs, x, ptr


def test_queue_tickets_published_after_launch_match_static_solve():
    torch, pk, dev, dev_in, ptrs = _setup()
    ctx = _native.Context(0)
    ref = ctx.solve(pk)
    order1 = [5, 0, 11, 3, 3, 7]
    order2 = [1, 2, 4, 6, 8, 9, 10, 5, 0]
    order = order1 + order2
    T = len(order)
    outs, x, optr = _outs(torch, dev, T, pk.n_var, pk.batch)
    q = _native.WorkQueue(ctx, T + 4)
    stream = torch.cuda.Stream(dev)
    try:
        ctx.solve_queue_device(pk, ptrs, q, optr, stream=stream.cuda_stream, waves=4, max_wait_s=30.0)
        with pytest.raises(RuntimeError, match="still open"):   # behind an open queue launch: rejected
            ctx.solve_queue_device(pk, ptrs, q, optr, stream=stream.cuda_stream, waves=4, max_wait_s=30.0)
        time.sleep(0.2)
        q.publish(order1)
        time.sleep(0.5)
        q.publish(order2)
    finally:
        q.close()
    torch.cuda.synchronize(dev)
    assert q.published() == T and q.claimed() >= T
    got = {k: v.cpu().numpy() for k, v in outs.items()}
    xs = x.cpu().numpy()
    for t, p in enumerate(order):
        for k in KEYS:
            assert got[k][t] == getattr(ref, {"iterations": "iterations"}.get(k, k))[p], (t, p, k)
    for p in set(order):
        assert np.array_equal(xs[p], ref.x[p]), p
    q.destroy()


def test_queue_closed_early_leaves_unpublished_tickets_unwritten():
    torch, pk, dev, dev_in, ptrs = _setup(6)
    ctx = _native.Context(0)
    cap = 8
    outs, x, optr = _outs(torch, dev, cap, pk.n_var, pk.batch)
    q = _native.WorkQueue(ctx, cap)
    stream = torch.cuda.Stream(dev)
    try:
        ctx.solve_queue_device(pk, ptrs, q, optr, stream=stream.cuda_stream, waves=2, max_wait_s=30.0)
        q.publish([4, 1, 2])
    finally:
        q.close()
    t0 = time.time()
    torch.cuda.synchronize(dev)
    assert time.time() - t0 < 25.0                     # drained on close, not on the max_wait timeout
    st = outs["status"].cpu().numpy()
    assert np.all(st[:3] >= 0) and np.all(st[3:] == -1), st
    with pytest.raises(RuntimeError):                  # closed: no more tickets
        q.publish([0])
    # the context is idle again: a static solve runs
    res = ctx.solve(pk)
    assert np.array_equal(res.status[[4, 1, 2]], st[:3])
    q.destroy()


def test_back_to_back_launches_on_two_streams_are_ordered():
    """Two static-range launches enqueued at once on two streams share the context's workspace: the second
    is ordered after the first (event wait), and both return the host-API solve's results."""
    torch, pk, dev, dev_in, ptrs = _setup(8)
    ctx = _native.Context(0)
    ref = ctx.solve(pk)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    o1, x1, p1 = _outs(torch, dev, pk.batch, pk.n_var, pk.batch)
    o2, x2, p2 = _outs(torch, dev, pk.batch, pk.n_var, pk.batch)
    ctx.solve_device(pk, ptrs, p1, stream=s1.cuda_stream)
    ctx.solve_device(pk, ptrs, p2, stream=s2.cuda_stream)
    torch.cuda.synchronize(dev)
    for o, x in ((o1, x1), (o2, x2)):
        assert np.array_equal(o["status"].cpu().numpy(), ref.status)
        assert np.array_equal(x.cpu().numpy(), ref.x)
