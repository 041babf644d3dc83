"""R/test/classic_planner.ipynb (cells 3-15) on the GPU: the Reeds-Shepp words of the
classic warm starts come from the HIP drop-in (libhtp.so htp_rs_all_paths_batch).
Pins as tests/test_classic_pins.py, plus identity with the CPU-restatement run."""
import numpy as np
import pytest

import _classic as C
from oracle import reeds_shepp as ors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def runs():
    return C.run(None), C.run(ors)


def test_gpu_classic_flow_matches_notebook_pins(runs):
    g, _ = runs
    np.testing.assert_allclose(g["start"], C.PIN_START_EXIT, atol=5e-9)
    np.testing.assert_allclose(g["safe"][0], C.PIN_SAFE_START, atol=5e-9)
    assert g["feasible"] == [C.PIN_WORD]
    np.testing.assert_allclose(g["ref"][0], C.PIN_REF0, atol=5e-9)


def test_gpu_classic_flow_matches_restatement(runs):
    g, c = runs
    assert g["n_paths"] == c["n_paths"]
    np.testing.assert_allclose(g["path"], c["path"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(g["ref"], c["ref"], rtol=0, atol=1e-9)
    assert g["circle_back"].shape == c["circle_back"].shape
    np.testing.assert_allclose(g["circle_back"], c["circle_back"], rtol=0, atol=1e-9)
