"""GPU parity of the orchard scene -> OBCA obstacle producer (htp_oge_obstacles_batch, csrc/oge_core.h;
R/path_planner/OGE_OBCA.py:306-677 + map_utils.create_tree_rows) against its host build, which
tests/test_oge_cpu.py pins to the Python restatement of the reference.  Device libm (tan, sin, atan,
sqrt) may differ from glibc in the last bit: vertices <= 1e-12, halfspace counts exact and values
<= 1e-7 (their 7-decimal rounding grid).  The same scenes also go through the device API with
device-resident buffers (the e2e chain's path)."""
import numpy as np
import pytest
import torch

import _hostsim as H
from headland_trajectory_planning_amd import _native, synth
from test_oge_cpu import _meta

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return _native.Context(0)


def _scenes():
    metas = [synth.config_instance(cfg, pid)["meta"] for cfg in "ACDE" for pid in range(8)]
    scenes = [synth.orchard_scene(m) for m in metas]
    rng = np.random.default_rng(11)
    for k in range(200):
        nrows = int(rng.integers(6, 16))
        s_row = int(rng.integers(0, nrows - 3))
        e_row = int(min(s_row + rng.integers(1, 4), nrows - 2))
        side = 1 if k % 2 == 0 else -1
        m = _meta(int(rng.integers(0, 2 ** 31 - 1)), nrows, rng.uniform(2.2, 3.5), rng.uniform(-15, 15),
                  float(rng.choice([0.0, 1.0])), rng.uniform(5.0, 9.0), s_row, e_row, rng.uniform(-1, 1),
                  rng.uniform(0, 3.66), side)
        scenes.append(dict(synth.orchard_scene(m), side=side))
    return scenes


def _check(g, h, B):
    assert np.array_equal(g.status, h.status) and np.array_equal(g.n_poly, h.n_poly)
    assert np.array_equal(g.n_vert, h.n_vert) and np.array_equal(g.n_facet, h.n_facet)
    for b in range(B):
        for pg, ph in zip(g.polygons(b), h.polygons(b)):
            assert np.max(np.abs(pg - ph)) <= 1e-12, b
        for (Ag, bg), (Ah, bh) in zip(g.halfspaces(b), h.halfspaces(b)):
            assert np.max(np.abs(Ag - Ah)) <= 1e-7 and np.max(np.abs(bg - bh)) <= 1e-7, b


def test_gpu_matches_host_core(ctx):
    scenes = _scenes()
    pk = _native.OgePacked(scenes)
    g = ctx.oge_obstacles(pk)
    h = H.oge_host(pk)
    assert np.all(g.status == 0)
    _check(g, h, pk.batch)
    assert ctx.oge_last_ms() > 0.0


def test_gpu_device_buffers(ctx):
    """htp_oge_obstacles_batch_device on torch-allocated device buffers, enqueued on a stream."""
    scenes = _scenes()[:96]
    pk = _native.OgePacked(scenes)
    dev = torch.device("cuda:0")
    t_in = {k: torch.from_numpy(getattr(pk, k)).to(dev) for k in ("params", "row_draws", "eps_draws")}
    B, P, V = pk.batch, _native.OGE_MAXPOLY, _native.OGE_MAXV
    o = dict(status=torch.zeros(B, dtype=torch.int32, device=dev), n_poly=torch.zeros(B, dtype=torch.int32, device=dev),
             n_vert=torch.zeros(B, P, dtype=torch.int32, device=dev),
             vertices=torch.zeros(B, P, V, 2, dtype=torch.float64, device=dev),
             n_facet=torch.zeros(B, P, dtype=torch.int32, device=dev),
             A=torch.zeros(B, P, V, 2, dtype=torch.float64, device=dev), b=torch.zeros(B, P, V, dtype=torch.float64,
                                                                                        device=dev))
    bs = pk.struct({k: v.data_ptr() for k, v in t_in.items()})
    rs = _native.OgeResult(*[o[k].data_ptr() for k in ("status", "n_poly", "n_vert", "vertices", "n_facet", "A", "b")])
    stream = torch.cuda.Stream(dev)
    import ctypes
    assert ctx.lib.htp_oge_obstacles_batch_device(ctx.ctx, ctypes.byref(bs), ctypes.byref(rs),
                                                  ctypes.c_void_p(stream.cuda_stream)) == 0
    stream.synchronize()
    g = _native.OgeResults(B)
    for k in ("status", "n_poly", "n_vert", "vertices", "n_facet", "A", "b"):
        setattr(g, k, o[k].cpu().numpy())
    _check(g, H.oge_host(pk), B)
