"""Oracle self-divergence witnesses (tests/golden/witness, tests/golden/make_witness.py) -- CPU only.

For every fixture where the device's outcome differs from the oracle fixture's (tests/test_gpu_obca.py
FAILURE_CLASS_ONLY / DIVERGENT_AFTER_RESTORATION / ROUNDING_DECIDED), a committed run of the ORACLE itself shows
that the reference algorithm does not determine the outcome at rounding level: a second valid elimination order,
the glibc libm CasADi calls, or the same instance with one input double moved by one ulp ends with a different
status or at a point more than the 1e-4 state tolerance away.  Runs that agree with the fixture are kept too, as
the record of how often the oracle's outcome holds."""
import os

import numpy as np
import pytest

W = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "witness")
STATE_TOL = 1e-4

# fixture -> the witness files that must show a divergence
REQUIRED = {"D347": ["D347"], "E6": ["E6"], "E84": ["E84"], "P19": ["P19"], "E12": ["E12_ulp3", "E12_ulp6"],
            "E54": ["E54_libm", "E54_ulp1"]}


def _diverges(w):
    return int(w["status_a"]) != int(w["status_b"]) or float(np.max(np.abs(w["states_a"] - w["states_b"]))) > STATE_TOL


@pytest.mark.parametrize("name", sorted(REQUIRED))
def test_oracle_witness_diverges(name):
    for f in REQUIRED[name]:
        w = np.load(os.path.join(W, f + ".npz"))
        assert _diverges(w), (f, int(w["status_a"]), int(w["status_b"]))


def test_e12_status_split_and_record():
    """E12: the fixture (Solve_Succeeded, 229 iterations) against its 1-ulp neighbours: one ends
    Infeasible_Problem_Detected, one converges elsewhere after 85 restoration phases, the rest agree."""
    w = np.load(os.path.join(W, "E12_ulp3.npz"))
    assert int(w["status_a"]) == 0 and int(w["status_b"]) == 7
    agree = [f for f in os.listdir(W) if f.startswith("E12_") and not _diverges(np.load(os.path.join(W, f)))]
    assert len(agree) >= 5, agree


def test_e54_status_split():
    """E54: the fixture (Infeasible_Problem_Detected, 1418 iterations / 32 phases) against the same instance with
    init_traj[0, 1] one ulp up: the oracle converges (Solve_Succeeded after 652 / 2 phases)."""
    w = np.load(os.path.join(W, "E54_ulp1.npz"))
    assert int(w["status_a"]) == 7 and int(w["status_b"]) == 0


def test_ulp_witnesses_record_the_moved_cell():
    """Every one-ulp witness stores the init_traj cell it moved, and it is the one tests/_neighbours.ulp_cell
    assigns to its index (the mapping the GPU neighbourhood test solves with)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from _neighbours import ulp_cell
    files = sorted(f for f in os.listdir(W) if "_ulp" in f)
    assert files
    for f in files:
        w = np.load(os.path.join(W, f))
        k = int(f[:-4].split("_ulp")[1])
        assert tuple(int(v) for v in w["cell"]) == ulp_cell(k, len(w["states_a"]) // 5), f
