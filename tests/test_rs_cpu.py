"""Reeds-Shepp on the CPU: the oracle and the host build of the
device core (csrc/rs_core.h) against golden vectors made by the reference
itself (tests/golden/make_golden.py), bit-for-bit, plus seeded random and
edge-case parity between the two and the reference's check_path properties.  Bit-for-bit comparisons with
the reference's doubles use the platform-libm host build (CPython's math module = glibc, as the golden vectors
were made); the product build (the correctly rounded libm of csrc/htp_libm.h, shared with the device) keeps
the same structure (words, sample counts, directions) and values within 1e-12 of it."""
import math

import numpy as np
import pytest

import _hostsim as H
import _rs_util as U
from oracle import reeds_shepp as ors


def test_oracle_matches_reference_goldens_bit_exact():
    g = U.golden()
    assert U.compare(g, U.oracle_csr(g["queries"])) == []
    assert g["path_offsets"][-1] == 728 and len(g["x"]) == 90703


def test_host_core_matches_reference_goldens_bit_exact():
    g = U.golden()
    assert U.compare(g, H.rs_host(g["queries"], platform=True)) == []
    assert U.compare(g, H.rs_host(g["queries"]), atol=1e-12) == []


def test_host_core_matches_oracle_on_seeded_queries():
    q = U.random_queries(400, seed=11)
    o = U.oracle_csr(q)
    assert U.compare(o, H.rs_host(q, platform=True)) == []
    assert U.compare(o, H.rs_host(q), atol=1e-12) == []
    assert o["path_offsets"][-1] > 2000


def test_candidate_table_is_the_reference_order():
    c = ors.candidates()
    assert len(c) == 46
    assert c[0] == ("SLS", "id", False) and c[1] == ("SLS", "refl", False)
    assert [w for w, _, b in c if b] == ["LRL"] * 4 + ["LRSL"] * 4 + ["LRSR"] * 4


def test_edge_cases():
    # start == goal: every word has zero length -> the reference asserts (set_path :83)
    q = np.array([[1.0, 2.0, 0.3, 1.0, 2.0, 0.3, 0.5, 0.2]])
    with pytest.raises(AssertionError):
        ors.calc_all_paths(*q[0])
    h = H.rs_host(q)
    assert h["status"].tolist() == [1] and h["n_paths"] == 0
    # beyond MAX_LENGTH (normalised) every word is filtered: empty list, like the reference
    q = np.array([[0.0, 0.0, 0.0, 3000.0, 0.0, 0.0, 0.5, 0.2]])
    assert ors.calc_all_paths(*q[0]) == []
    h = H.rs_host(q)
    assert h["status"].tolist() == [0] and h["n_paths"] == 0
    # straight ahead, pure rotation on the spot, tiny offset, huge step
    qs = np.array([[0.0, 0.0, 0.0, 5.0, 0.0, 0.0, 0.5, 0.2],
                   [0.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.5, 0.1],
                   [0.0, 0.0, 0.0, 1e-3, 1e-3, 1e-3, 0.5, 0.1],
                   [0.0, 0.0, 1.0, 4.0, -2.0, -2.0, 0.2, 5.0],
                   [-1.0, 3.0, math.pi, 2.0, -3.0, -math.pi, 1.0, 0.05]])
    o = U.oracle_csr(qs)
    assert U.compare(o, H.rs_host(qs, platform=True)) == []
    assert U.compare(o, H.rs_host(qs), atol=1e-12) == []


def test_path_properties_follow_the_reference():
    """check_path (:668-690): every path starts at the start pose; words of the
    SCS/CSC/CCSC/CCSCC families end at the goal.  The reference's CCC and
    CCCC words can miss the goal (its tau/omega and wrap conventions); parity
    keeps that, so those families are only checked for the start pose."""
    q = U.random_queries(600, seed=5, degenerate=False)
    assert U.check_path_properties(U.oracle_csr(q), q) == 0
    q = U.random_queries(600, seed=6)
    assert U.check_path_properties(U.oracle_csr(q), q, goal=False) == 0


def test_sampler_indexerror_convention():
    """A short pure rotation whose every sample lands back on local x == 0.0:
    the reference's trailing-zero pop empties the list and raises IndexError
    (reeds_shepp.py:523); the ABI reports status 2 and keeps the path with no
    samples."""
    q = np.array([[-6.77841483700109, -3.5908784796717637, 2.3469009462205817, -6.77841483700109,
                   -3.5908784796717637, 2.4648799751813466, 0.3226869543621767, 0.3]])
    with pytest.raises(IndexError):
        ors.calc_all_paths(*q[0])
    h = H.rs_host(q)
    assert h["status"].tolist() == [2]
    assert U.compare(U.oracle_csr(q), h) == []
