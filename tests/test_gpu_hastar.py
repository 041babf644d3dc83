"""Hybrid A* on the MI355X (libhtp.so htp_hastar_search_batch): one batched
launch against the serial host build of the same core and against the oracle.
Structure (status, counter, expansion order) must be identical; path samples
within 1e-9 (the device's trig may differ from glibc in the last ulp)."""
import numpy as np
import pytest

import _ha_util as U
import _hostsim as H
from headland_trajectory_planning_amd import _native
from headland_trajectory_planning_amd.path_planner.hybrid_a_star_search import (HybridAStarSearch,
                                                                                 hybrid_a_star_search_batch)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return _native.Context(0)


def _gpu(ctx, probs):
    return H.as_dicts(ctx.hastar(_native.HastarPacked(probs)))


def test_gpu_matches_oracle(ctx):
    probs = [U.scenario(s, max_nodes=60) for s in (0, 1, 2, 5, 7, 8)]
    g = _gpu(ctx, probs)
    for p, r in zip(probs, g):
        assert U.compare(U.run_oracle(p), r, exact=False) == []


def test_gpu_matches_host_core_batch(ctx):
    probs = [U.scenario(s, max_nodes=120) for s in range(48)]
    g = _gpu(ctx, probs)
    h = H.as_dicts(H.hastar_host(probs))
    bad = [(i, U.compare(a, b, exact=False)) for i, (a, b) in enumerate(zip(h, g)) if U.compare(a, b, exact=False)]
    assert bad == []
    assert len({r["status"] for r in g}) >= 2


def test_gpu_pawn_matches_host_and_oracle(ctx):
    probs = [U.scenario_pawn(s, n_obs=1 + s % 3) for s in range(16)]
    g = _gpu(ctx, probs)
    h = H.as_dicts(H.hastar_host(probs))
    for a, b in zip(h, g):
        assert U.compare(a, b, exact=False) == []
    for p, b in list(zip(probs, g))[:6]:
        assert U.compare(U.run_oracle(p), b, exact=False) == []
    assert {r["status"] for r in g} >= {0, 2}


def test_gpu_edge_cases_and_bad_input(ctx):
    base = U.scenario(0, max_nodes=30)
    probs = [dict(base, max_nodes=0), dict(base, goal=base["start"].copy()), dict(base, field=None)]
    g = _gpu(ctx, probs)
    for p, r in zip(probs, g):
        assert U.compare(U.run_oracle(p), r, exact=False) == []
    # a search length that needs more than 64 poses per primitive is rejected, not run
    bad = dict(base, default_search_length=100.0)
    assert _gpu(ctx, [bad])[0]["status"] == 6


def test_dropin_shim_search_and_batch(ctx):
    p, (env, car, heur, start, goal) = U.scenario(5, max_nodes=60, return_objects=True)
    hs = HybridAStarSearch(start, goal, env, car, heur, motion_type="King", plan_resolution=0.2)
    xs, ys, yaws, dirs, ks, counter = hs.hybrid_a_star_search(max_nodes=60)
    o = U.run_oracle(p)
    assert counter == o["counter"] and len(xs) == len(o["xs"])
    assert np.allclose(xs, o["xs"], atol=1e-9) and np.allclose(ks, o["ks"], atol=1e-9)
    out = hybrid_a_star_search_batch([hs, hs], max_nodes=60)
    assert out[0][5] == out[1][5] == counter


def test_combined_king_pawn_kernel_matches_split_kernels(ctx, monkeypatch):
    """Round-1 note: a combined King+Pawn kernel once returned wrong
    Pawn statuses.  The combined body (Search::run dispatch, the default) must
    give the split kernels' results (HTP_HA_SPLIT=1) on a mixed batch, and the
    host build's."""
    probs = [U.scenario_pawn(s, n_obs=1 + s % 3) for s in range(16)] + [U.scenario(s, max_nodes=80) for s in range(16)]
    probs = [p for pair in zip(probs[:16], probs[16:]) for p in pair]
    comb = _gpu(ctx, probs)
    monkeypatch.setenv("HTP_HA_SPLIT", "1")
    split = _gpu(ctx, probs)
    monkeypatch.delenv("HTP_HA_SPLIT")
    host = H.as_dicts(H.hastar_host(probs))
    for a, b, h in zip(split, comb, host):
        assert U.compare(a, b, exact=False, tol=1e-12) == []
        assert U.compare(h, b, exact=False) == []
