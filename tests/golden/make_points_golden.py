"""Generate full-size point-formulation parity fixtures (tests/golden/points_full/P<pid>.npz).

TEST INFRASTRUCTURE: the oracle (oracle/ipm.py IPOPT restatement over oracle/nlp_points.py with the
structured KKT of oracle/structured.py StructuredPointKKT) solves make_points_instance(pid, N=80, M=6)
-- the instances tools/bench_points.py solves -- with max_cpu_time off.  Selected pids include
problems the solver does not solve (picked by tools/screen_points.py), so the GPU's failure statuses
are pinned against the oracle's.  Each fixture stores its input (tests/_fixture_io.py).

    python tests/golden/make_points_golden.py [PID ...]
"""
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.path.join(ROOT, "tests", "golden", "points_full")
N, M = 80, 6
PIDS = [0, 1, 257, 84, 468]


def run(pid):
    from _fixture_io import instance_arrays
    from headland_trajectory_planning_amd import synth
    from oracle.ipm import IpoptRestatement
    from oracle.nlp_points import PointNLP
    from oracle.structured import StructuredPointKKT
    inst = synth.make_points_instance(pid, N=N, M=M)
    nlp = PointNLP(inst)
    t = time.time()
    r = IpoptRestatement(nlp, kkt=StructuredPointKKT(nlp)).solve()
    dt = time.time() - t
    np.savez(os.path.join(OUT, f"P{pid}.npz"), states=r["x"][:5 * N], x=r["x"], f=r["f"], status=r["status"],
             iters=r["iters"], n_resto=r["n_resto"], N=N, M=M, seconds=dt, status_str=r["status_str"],
             **instance_arrays(inst))
    return f"P{pid} {r['status_str']} iters={r['iters']} n_resto={r['n_resto']} f={r['f']:.12g} ({dt:.0f} s)"


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    pids = [int(a) for a in sys.argv[1:]] or PIDS
    with mp.Pool(min(8, len(pids))) as pool:
        for line in pool.imap_unordered(run, pids):
            print(line, flush=True)
