"""Y-park grid search on the MI355X (htp_ypark_search_batch) against its
serial host build and the oracle: identical status / candidate / parameters,
manoeuvre within 1e-9."""
import numpy as np
import pytest

import _hostsim as H
import _yp_util as U
from headland_trajectory_planning_amd import _native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return _native.Context(0)


def test_gpu_matches_host_and_oracle(ctx):
    probs = [U.scenario(s) for s in range(24)]
    g = H.ypark_dicts(ctx.ypark(_native.YparkPacked(probs)))
    h = H.ypark_dicts(H.ypark_host(probs))
    for a, b in zip(h, g):
        assert U.compare(a, b, tol=1e-9) == []
    for p, b in list(zip(probs, g))[:8]:
        assert U.compare(U.run_oracle(p), b, tol=1e-9) == []
    assert {r["status"] for r in g} >= {0, 1}
