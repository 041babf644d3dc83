"""GPU parity of the classic headland turns (htp_classic_turn_batch, csrc/classic_core.h; SURVEY.md 8(f)
row 4) against their host build, which tests/test_classic_core_cpu.py pins to the restated reference
planners.  Both builds evaluate sin, cos, tan, atan, atan2, asin, acos, hypot and pow with the same correctly
rounded libm (csrc/htp_libm.h, tests/test_gpu_libm.py), so every turn has the host build's row count (a spline
piece's len(np.arange(0, S + ds, ds)) hangs on the last bit of S) and its rows to 1e-12.  A mixed batch of config C scenes (Dubins, circle-back and fish-tail in
one launch) plus the A and B scenes; the chosen path then feeds the device init-guess kernel."""
import numpy as np
import pytest

import _hostsim as H
from headland_trajectory_planning_amd import _native, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return _native.Context(0)


def test_gpu_matches_host_core(ctx):
    metas = [synth.config_instance(cfg, pid)["meta"] for cfg, n in (("C", 48), ("A", 8), ("B", 8)) for pid in range(n)]
    pk = _native.ClassicPacked([synth.classic_turn(m) for m in metas])
    g = ctx.classic_turns(pk)
    h = H.classic_host(pk)
    assert np.array_equal(g.status, h.status) and np.all(g.status == 0)
    assert np.array_equal(g.n_path, h.n_path), np.where(g.n_path != h.n_path)
    worst = max(float(np.max(np.abs(g.rows(b) - h.rows(b)))) for b in range(pk.batch))
    assert worst <= 1e-12, worst
    assert {m["turn"] for m in metas} == {"dubins", "circleback", "fishtail"}
    assert ctx.classic_last_ms() > 0.0
    # device turn -> device init guess (get_init_ref_path), as the workload generator chains them on the host
    from headland_trajectory_planning_amd.obca_py.util import get_init_ref_path
    from headland_trajectory_planning_amd.obca_py.car_model_obca import CarModel
    car = CarModel(with_aux=False)
    paths = [g.rows(b) for b in range(6)]
    rp = ctx.init_ref_path(_native.RefPathPacked([(p[:, 0], p[:, 1], p[:, 4]) for p in paths],
                                                 [(car.WHEEL_BASE, 0.5, 0.2)] * len(paths)))
    for b, p in enumerate(paths):
        ref = get_init_ref_path(car, p[:, 0], p[:, 1], p[:, 2], p[:, 3], p[:, 4], desired_v=0.5, ds=0.2)
        assert np.max(np.abs(rp.path(b) - ref)) < 1e-9
