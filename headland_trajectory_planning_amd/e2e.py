"""The orchard workload end to end on the device: scene draws (host, the reference's np.random streams) ->
classic turn -> init guess -> resample + headland width -> OGE_OBCA obstacle producer -> quads -> OBCA solve,
with every intermediate and the solver's inputs in HBM (htp_orchard_chain_device + the OBCA launch).

The device-built problems equal synth.config_instance's host-built ones (tests/test_gpu_e2e.py); bench.py
--e2e times the chain and the solve together (a "solve" including its warm start)."""
import ctypes

import numpy as np

from . import _native, geometry, synth


def host_inputs(metas, cfg):
    """Host arrays of the chain's inputs for problems described by make_orchard_instance metas."""
    _, N, M, imp = synth.CONFIGS[cfg]
    scenes = _native.OgePacked([synth.orchard_scene(m) for m in metas])
    turns = _native.ClassicPacked([synth.classic_turn(m) for m in metas])
    veh = synth.VEHICLE
    polys = [geometry.body_rectangle(veh["axle_to_front"], veh["axle_to_back"], veh["width"])]
    if synth.IMPLEMENTS[imp] is not None:
        polys.append(geometry.implement_rectangle(synth.IMPLEMENTS[imp]))
    base = synth.config_instance(cfg, int(metas[0]["pid"]))   # shape / parameter template (same for all)
    return dict(N=N, M=M, scenes=scenes, turns=turns, polys=polys, margin=np.array([m["margin"] for m in metas]),
                template=base)


class DeviceChain:
    """Device buffers (torch) for one batch of the chain and the OBCA solve of its output."""

    def __init__(self, ctx, inputs, cap_rows=1024, copies=1):
        import torch
        self.ctx, self.torch = ctx, torch
        dev = torch.device("cuda", ctx.device)
        self.dev = dev
        sc, tu = inputs["scenes"], inputs["turns"]
        B, N, M = sc.batch, inputs["N"], inputs["M"]
        self.B, self.N, self.M, self.cap_rows, self.copies = B, N, M, cap_rows, copies
        B = B * copies   # output slots: one slice of B problems per build(k)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
        self.sc_in = {k: t(getattr(sc, k)) for k in ("params", "row_draws", "eps_draws")}
        self.tu_in = {k: t(getattr(tu, k)) for k in ("params", "desc", "poly_off", "vertices")}
        self.margin = t(inputs["margin"])
        self.traj = torch.zeros(B, N, 5, dtype=torch.float64, device=dev)
        self.obs_A = torch.zeros(B, 4 * M, 2, dtype=torch.float64, device=dev)
        self.obs_b = torch.zeros(B, 4 * M, dtype=torch.float64, device=dev)
        self.status = torch.zeros(B, dtype=torch.int32, device=dev)
        tmpl = inputs["template"]
        self.params = t(np.tile(_native.params_of(tmpl), (B, 1)))
        self.body_G = t(np.tile(np.concatenate(tmpl["body_G"]), (B, 1, 1)))
        self.body_g = t(np.tile(np.concatenate(tmpl["body_g"]), (B, 1)))
        self.K = len(tmpl["body_G"])
        self.body_edges = np.array([a.shape[0] for a in tmpl["body_G"]], np.int32)
        self.obs_edges = np.full(M, 4, np.int32)
        self.time_opt = int(np.asarray(tmpl["W"])[1, 1] != 0)
        cb = _native.ChainBatch()
        cb.batch, cb.N, cb.M = self.B, N, M
        cb.scenes = sc.struct({k: v.data_ptr() for k, v in self.sc_in.items()})
        cb.turns = tu.struct({k: v.data_ptr() for k, v in self.tu_in.items()})
        cb.margin = self.margin.data_ptr()
        polys = inputs["polys"]
        cb.n_vpoly = len(polys)
        vp = np.zeros((2, 8, 2))
        for k, p in enumerate(polys):
            cb.vpoly_nv[k] = p.shape[0]
            vp[k, :p.shape[0]] = p
        for i, v in enumerate(vp.reshape(-1)):
            cb.vpoly[i] = float(v)
        cb.dT, cb.wheel_base = float(tmpl["dT"]), float(synth.VEHICLE["wheelbase"])
        cb.cap_rows = cap_rows
        cb.traj, cb.obs_A, cb.obs_b = self.traj.data_ptr(), self.obs_A.data_ptr(), self.obs_b.data_ptr()
        cb.status = self.status.data_ptr()
        self.cb = cb

    def build(self, stream=None, copy=0):
        """Enqueue the chain on `stream` (a torch.cuda.Stream; default: the current stream), writing output
        slice `copy` (problems [copy * B, (copy + 1) * B))."""
        s = stream or self.torch.cuda.current_stream(self.dev)
        cb = self.cb
        o = copy * self.B
        cb.traj = self.traj[o:].data_ptr()
        cb.obs_A, cb.obs_b, cb.status = self.obs_A[o:].data_ptr(), self.obs_b[o:].data_ptr(), self.status[o:].data_ptr()
        if self.ctx.lib.htp_orchard_chain_device(self.ctx.ctx, ctypes.byref(cb), ctypes.c_void_p(s.cuda_stream)) != 0:
            raise RuntimeError(f"[htp] htp_orchard_chain_device failed: {self.ctx.error()}")

    def struct(self, ptrs=None):
        """PackedBatch-style hook: htp_obca_batch over every output slot (for the persistent launch)."""
        b = self.obca_batch()
        b.batch = self.B * self.copies
        return b

    def obca_batch(self):
        """htp_obca_batch over the chain's device outputs (+ the constant body / parameter arrays)."""
        b = _native.ObcaBatch()
        b.batch, b.N, b.M, b.K, b.time_opt = self.B, self.N, self.M, self.K, self.time_opt
        b.obs_edges, b.body_edges = self.obs_edges.ctypes.data, self.body_edges.ctypes.data
        b.traj, b.obs_A, b.obs_b = self.traj.data_ptr(), self.obs_A.data_ptr(), self.obs_b.data_ptr()
        b.body_G, b.body_g, b.params = self.body_G.data_ptr(), self.body_g.data_ptr(), self.params.data_ptr()
        b.init_control = b.init_mu = b.init_lambda = None
        return b

    def instances(self):
        """The device-built problems as host instance dicts (oracle/nlp.py format), for checks."""
        traj, A, bb = self.traj.cpu().numpy(), self.obs_A.cpu().numpy(), self.obs_b.cpu().numpy()
        out = []
        for k in range(self.B * self.copies):
            out.append(dict(init_traj=traj[k], obs_A=[A[k, 4 * m:4 * m + 4] for m in range(self.M)],
                            obs_b=[bb[k, 4 * m:4 * m + 4] for m in range(self.M)]))
        return out


OUT_KEYS = ("objective", "status", "iterations", "n_factor", "nlp_error", "n_resto")


def solve_outputs(torch, dev, B, n_var):
    outs = {k: torch.zeros(B, dtype=torch.float64 if k in ("objective", "nlp_error") else torch.int32, device=dev)
            for k in OUT_KEYS}
    outs["x"] = torch.zeros(B, n_var, dtype=torch.float64, device=dev)
    return outs


def solve_chain(ctx, chain, outs, stream):
    """htp_obca_solve_batch_device on the chain's device outputs, enqueued on `stream`."""
    r = _native.ObcaResult()
    for k, v in outs.items():
        setattr(r, k, v.data_ptr())
    b = chain.obca_batch()
    if ctx.lib.htp_obca_solve_batch_device(ctx.ctx, ctypes.byref(b), ctypes.byref(r), stream.cuda_stream) != 0:
        raise RuntimeError(f"[htp] htp_obca_solve_batch_device failed: {ctx.error()}")


def run_bench(insts, cfg, steps, warmup, max_cpu_time=20.0, device=0):
    """Time `steps` passes of chain + solve over the problems whose make_orchard_instance metas `insts` carry:
    the chain runs once per step (into its own output slice), then one persistent OBCA launch fed by a work
    queue solves every step's problems (as bench.py's headline job), all on one stream."""
    import time

    import torch
    metas = [it["meta"] for it in insts]
    inputs = host_inputs(metas, cfg)
    ctx = _native.Context(device)
    ctx.set_option("max_cpu_time", max_cpu_time)
    chain = DeviceChain(ctx, inputs, copies=max(steps, warmup, 1))
    dev = chain.dev
    n_var = _native.PackedBatch([inputs["template"]]).n_var
    outs = solve_outputs(torch, dev, chain.B * chain.copies, n_var)
    optr = {k: v.data_ptr() for k, v in outs.items()}
    waves = ctx.resident_waves(chain)
    stream = torch.cuda.Stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

    def job(k):
        T = k * chain.B
        q = _native.WorkQueue(ctx, T)
        ev[0].record(stream)
        for c in range(k):
            chain.build(stream, copy=c)
        ev[1].record(stream)
        try:
            ctx.solve_queue_device(chain, None, q, optr, stream=stream.cuda_stream, waves=waves)
            ev[2].record(stream)
            q.publish(np.arange(T, dtype=np.int32))
        finally:
            q.close()
        stream.synchronize()
        return ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), T

    if warmup:
        job(warmup)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    chain_ms, solve_ms, T = job(steps)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    st = outs["status"][:T].cpu().numpy()
    it = outs["iterations"][:T].cpu().numpy()
    chain_st = chain.status[:T].cpu().numpy()
    return dict(value=T / elapsed, elapsed=elapsed, chain_ms=chain_ms / steps, solve_ms=solve_ms / steps,
                chain_status={str(k): int(v) for k, v in zip(*np.unique(chain_st, return_counts=True))},
                status_counts={str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
                success_rate=float(np.isin(st, [0, 1]).mean()), mean_iters=float(it.mean()), batch=chain.B,
                iters_sum=float(it.sum()), waves=waves)
