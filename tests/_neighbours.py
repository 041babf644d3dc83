"""One-ulp input neighbours of a parity fixture (TEST INFRASTRUCTURE).

Neighbour k of a fixture is its instance with ONE double of the initial guess `init_traj` moved up by one ulp
(np.nextafter towards +inf): an instance the reference cannot tell apart from the fixture's after its own float
parsing and arithmetic (`R/obca_py/optimizer.py:110-138` reads `init_traj` as given).  The oracle's witnesses
(tests/golden/make_witness.py NAME:ulpK) and the device runs of tests/test_gpu_obca.py::test_neighbourhood_*
use this one mapping, and every witness file stores the (row, col) it moved.

k < 10 keeps the mapping the round-5 witnesses were made with: k = 0..3 -> rows 0-1, columns 0-1;
k = 4..7 -> (k + 1, 0); k = 8, 9 -> (k - 4, 1).  k >= 10 walks rows 11, 18, 25, ... (step 7, modulo N) through
the columns x, y, v, yaw.  The steer column is left out: the synthetic warm starts sit on the steering bound
(|steer| = max_steer = 0.55) at most rows, and IPOPT's bound push moves an initial point that close to its bound
into the interior by the same amount either way, so a one-ulp move there leaves the solve unchanged (the device
run on such a "neighbour" is bit-identical to the fixture's: gpurun_out r06a)."""
import numpy as np


def ulp_cell(k, N):
    """(row, col) of init_traj moved by neighbour k of an N-row instance."""
    if k < 4:
        rc = (k // 2, k % 2)
    elif k < 8:
        rc = (k + 1, 0)
    elif k < 10:
        rc = (k - 4, 1)
    else:
        i = k - 10
        rc = ((11 + 7 * (i // 4)) % N, i % 4)
    assert 0 <= rc[0] < N, (k, N, rc)
    return rc


def neighbour(inst, k):
    """The instance with init_traj[ulp_cell(k)] moved up by one ulp, and the cell."""
    tr = np.array(inst["init_traj"], dtype=np.float64)
    row, col = ulp_cell(k, tr.shape[0])
    tr[row, col] = np.nextafter(tr[row, col], np.inf)
    return dict(inst, init_traj=tr), (row, col)
