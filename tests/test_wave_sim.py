"""The lane-parallel code of the kernel, executed by 64 CPU threads with a
barrier per c.sync() (test-only simulation), must equal the serial build."""
import numpy as np

import _hostsim
from headland_trajectory_planning_amd import synth


def test_64_lane_simulation_matches_serial():
    insts = [synth.make_instance(pid, N=10, M=2, implement="mower") for pid in range(2)]
    a = _hostsim.solve_threadsim(insts)
    b = _hostsim.solve(insts)
    assert np.array_equal(a.status, b.status)
    assert np.array_equal(a.iterations, b.iterations)
    assert np.max(np.abs(a.x - b.x)) <= 1e-9
