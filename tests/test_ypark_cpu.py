"""Y-type parking grid search (headland_path_planning.py:382-451)
on the CPU: the serial host build of the device core (csrc/ypark_core.h)
against the oracle -- same status, same chosen candidate and parameters, the
same manoeuvre (1e-12; the reference's odom transform is a BLAS product)."""
import numpy as np
import pytest

import _hostsim as H
import _yp_util as U


@pytest.mark.parametrize("seed", range(8))
def test_host_core_matches_oracle(seed):
    p = U.scenario(seed)
    assert U.compare(U.run_oracle(p), H.ypark_dicts(H.ypark_host([p]))[0]) == []


def test_end_pose_blocked_and_batch():
    p = U.scenario(0)
    blocked = dict(p, blockers=list(p["blockers"]) + [np.array([[-50.0, -50.0], [50.0, -50.0], [50.0, 50.0],
                                                                 [-50.0, 50.0]])])
    probs = [p, blocked, U.scenario(6)]
    hs = H.ypark_dicts(H.ypark_host(probs))
    assert [h["status"] for h in hs] == [0, 2, 0]
    for q, h in zip(probs, hs):
        assert U.compare(U.run_oracle(q), h) == []
