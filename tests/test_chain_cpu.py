"""The orchard workload chain (csrc/chain_core.h: turn -> init guess -> resample + headland width -> obstacle
producer -> quads, the stage sequence of htp_orchard_chain_device) through its serial host build, compared
with the host generator synth.make_orchard_instance on the same accepted scene draws: the init guess and the
obstacle halfspaces of every problem equal (<= 1e-12 / bit-exact), for every turn type and implement."""
import numpy as np
import pytest

from headland_trajectory_planning_amd import e2e, synth

from _hostsim import chain_host


@pytest.mark.parametrize("cfg,n", [("A", 6), ("B", 8), ("C", 24), ("D", 16), ("E", 6)])
def test_chain_host_build_equals_the_generator(cfg, n):
    insts = [synth.config_instance(cfg, p) for p in range(n)]
    got, status = chain_host(e2e.host_inputs([it["meta"] for it in insts], cfg))
    assert np.all(status == 0), status
    for k, (g, h) in enumerate(zip(got, insts)):
        assert np.max(np.abs(g["init_traj"] - h["init_traj"])) <= 1e-11, (k, h["meta"]["turn"])
        for A, Ah, b, bh in zip(g["obs_A"], h["obs_A"], g["obs_b"], h["obs_b"]):
            assert np.array_equal(A, Ah) and np.array_equal(b, bh), k
