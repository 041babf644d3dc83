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


def test_short_solves_equal_the_emulation(ctx):
    insts = [synth.config_instance("D", p) for p in range(3)] + [synth.config_instance("C", 0),
                                                                  synth.config_instance("A", 1)]
    W = np.diag([10.0, 0.1])
    insts += [synth.make_instance(p, N=12, M=2, implement="mower", W=W) for p in (0, 3)]   # restoration phases
    for group in ([insts[k] for k in (0, 1, 2)], [insts[3]], [insts[4]], insts[5:]):   # one shape per launch
        _same(ctx.solve(_native.PackedBatch(group)), H.solve_emusim(group))


def test_point_formulation_equals_the_emulation(ctx):
    insts = [synth.make_points_instance(p, N=12, M=2) for p in (0, 5, 7)]
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
