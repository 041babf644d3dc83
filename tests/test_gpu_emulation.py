"""The device solver reproduced on the host bit for bit.  csrc/htp_emusim.cpp runs the kernel's ObcaSolver
instantiation on 64 lane threads (csrc/emu_wave.h) with the device's wave-reduction order, the matrix core's
rounding (tests/test_gpu_mfma_model.py pins the model), the device build's contraction and the shared
deterministic solver libm (obca_core.h HTP_SOLVER_DETLIBM: htp_fastm.h sin / cos / tan / log, htp_libm.h pow); it must return the device's doubles exactly -- solution vector, objective, status,
iteration and restoration counts:

  * live on short solves (configs A, C, D and small restoration cases, both formulations);
  * on the committed emulation fixtures of the long restoration cycles where the device and the oracle part
    ways (D347, E6, E84, P19; tests/golden/make_emulation.py).  The serial host build, whose summation order is
    the oracle's, ends where the oracle ends on those (tests/test_gpu_obca.py), so their divergence is the
    summation order and nothing else."""
import os

import numpy as np
import pytest

import _hostsim as H
from headland_trajectory_planning_amd import _native, synth

pytestmark = pytest.mark.gpu

EMU = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "emulation")


@pytest.fixture(scope="module")
def ctx():
    return _native.Context(0)


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.int64)


def _same(dev, emu):
    assert np.array_equal(dev.status, emu.status), (dev.status, emu.status)
    assert np.array_equal(dev.iterations, emu.iterations), (dev.iterations, emu.iterations)
    assert np.array_equal(dev.n_resto, emu.n_resto), (dev.n_resto, emu.n_resto)
    bad = np.where(np.any(_bits(dev.x) != _bits(emu.x), axis=1))[0]
    assert len(bad) == 0, (bad, [float(np.max(np.abs(dev.x[k] - emu.x[k]))) for k in bad])
    assert np.array_equal(_bits(dev.objective), _bits(emu.objective))


class _Stored:
    def __init__(self, z, g):
        self.x, self.status, self.iterations = z[f"g{g}_x"], z[f"g{g}_status"], z[f"g{g}_iters"]
        self.n_resto, self.objective = z[f"g{g}_n_resto"], z[f"g{g}_objective"]


def test_short_solves_equal_the_emulation(ctx):
    """Configs D (3 problems), C, A and two small restoration cases.  The emulation's result is cached in
    tests/golden/emulation/short_solves.npz (make_emulation.py short) under a hash of the solver core and the
    emulation sources; with a stale or missing cache the emulation runs live (minutes of host time)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_emulation import emu_key, group_hash, short_groups
    path = os.path.join(EMU, "short_solves.npz")
    z = np.load(path) if os.path.exists(path) else None
    cached = z is not None and str(z["key"]) == emu_key()
    for g, group in enumerate(short_groups()):   # one shape per launch
        dev = ctx.solve(_native.PackedBatch(group))
        if cached:
            assert str(z[f"g{g}_hash"]) == group_hash(group), g   # the cache was made on these very instances
            _same(dev, _Stored(z, g))
        else:
            _emusim_built_or_fail()
            _same(dev, H.solve_emusim(group))


def _emusim_built_or_fail():
    """A live emulation needs build/libhtp_emusim.so: when build() recorded that building it failed, this is a
    failure of the evidence, not a reason to skip."""
    import json
    info = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "build_info.json")
    if os.path.exists(info):
        act = json.load(open(info)).get("actions", {}).get("libhtp_emusim.so (test-only)", {})
        if act.get("action") == "failed":
            pytest.fail(f"the host emulation library failed to build: {act.get('error')}")


def test_point_formulation_equals_the_emulation(ctx):
    insts = [synth.make_points_instance(p, N=12, M=2) for p in (0, 5, 7)]
    _emusim_built_or_fail()
    _same(ctx.solve_points(_native.PointsPackedBatch(insts)), H.solve_points_emusim(insts))


@pytest.mark.parametrize("name", ["P19", "D347", "E84", "E6", "E12", "E54"])
def test_divergent_fixtures_equal_the_emulation(ctx, name):
    path = os.path.join(EMU, f"{name}.npz")
    if not os.path.exists(path):
        pytest.skip(f"no emulation fixture {name} (tests/golden/make_emulation.py)")
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_emulation import instance
    z = np.load(path)
    inst, kind = instance(name)
    dev = (ctx.solve_points(_native.PointsPackedBatch([inst])) if kind == "points"
           else ctx.solve(_native.PackedBatch([inst])))
    assert int(dev.status[0]) == int(z["status"]) and int(dev.iterations[0]) == int(z["iters"]), \
        (name, dev.status[0], dev.iterations[0], int(z["status"]), int(z["iters"]))
    assert int(dev.n_resto[0]) == int(z["n_resto"])
    assert np.array_equal(_bits(dev.x[0]), _bits(z["x"])), float(np.max(np.abs(dev.x[0] - z["x"])))
    assert _bits(dev.objective[:1])[0] == _bits(np.array([float(z["objective"])]))[0]
