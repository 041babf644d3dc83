"""The serial host build of the solver core (HostLane: csrc/htp_hostsim.cpp, the oracle's summation order, the
scalar Riccati) on a fixture's one-ulp neighbours -- the third draw beside the oracle's witnesses and the device's
runs (tools/neighbour_probe.py).  TEST INFRASTRUCTURE.

    python tools/host_neighbours.py D15863 --k 26 --procs 2 > gpurun_out/trace/D15863_host_nb.json
"""
import argparse
import json
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def one(job):
    name, k = job
    import _hostsim as H
    from _fixture_io import load_instance
    from _neighbours import neighbour
    g = np.load(os.path.join(ROOT, "tests", "golden", "obca_full", f"{name}.npz"))
    inst = load_instance(g)
    if k >= 0:
        inst = neighbour(inst, k)[0]
    r = H.solve([inst], {"max_cpu_time": 0.0})
    N = int(g["N"])
    return {"k": k, "status": int(r.status[0]), "iters": int(r.iterations[0]), "n_resto": int(r.n_resto[0]),
            "dx_fixture": float(np.max(np.abs(r.x[0, :5 * N] - g["states"])))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--k", type=int, default=26)
    ap.add_argument("--procs", type=int, default=2)
    a = ap.parse_args()
    import _hostsim as H
    H.build()
    with mp.Pool(a.procs) as pool:
        rows = sorted(pool.map(one, [(a.name, k) for k in range(-1, a.k)]), key=lambda r: r["k"])
    print(json.dumps({"name": a.name, "runs": rows}))


if __name__ == "__main__":
    main()
