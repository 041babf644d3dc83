"""Device outcome on the one-ulp input neighbours of parity fixtures.

For each fixture: the fixture's instance and its neighbours k = 0..K-1 (tests/_neighbours.py: one init_traj
double moved by one ulp) solved in one batch on the GPU with max_cpu_time off.  Per run: status, iterations,
restoration phases, objective and the largest state difference from the oracle fixture's states; where an
oracle witness for the same neighbour exists (tests/golden/witness/<NAME>_ulp<k>.npz), the oracle's status and
the state difference from the oracle's own end point.

    python tools/neighbour_probe.py E12 E4 D3220 --k 32 > gpurun_out/neighbours.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--gold", default=os.path.join(ROOT, "tests", "golden", "obca_full"))
    ap.add_argument("--witness", default=os.path.join(ROOT, "tests", "golden", "witness"))
    args = ap.parse_args()
    from _fixture_io import load_instance
    from _neighbours import neighbour
    from headland_trajectory_planning_amd import _native
    ctx = _native.Context(0)
    ctx.set_option("max_cpu_time", 0.0)
    out = {}
    for name in args.names:
        g = np.load(os.path.join(args.gold, f"{name}.npz"))
        N = int(g["N"])
        base = load_instance(g)
        insts, cells = [base], [None]
        for k in range(args.k):
            inst, cell = neighbour(base, k)
            insts.append(inst)
            cells.append(cell)
        t = time.time()
        res = ctx.solve(_native.PackedBatch(insts))
        dt = time.time() - t
        rows = []
        for j in range(len(insts)):
            r = {"k": None if j == 0 else j - 1, "cell": cells[j], "status": int(res.status[j]),
                 "iters": int(res.iterations[j]), "n_resto": int(res.n_resto[j]), "f": float(res.objective[j]),
                 "dx_fixture": float(np.max(np.abs(res.x[j, :5 * N] - g["states"])))}
            wp = os.path.join(args.witness, f"{name}_ulp{j - 1}.npz")
            if j > 0 and os.path.exists(wp):
                w = np.load(wp)
                r["oracle"] = {"status": int(w["status_b"]), "iters": int(w["iters_b"]), "n_resto": int(w["n_resto_b"]),
                               "dx_oracle": float(np.max(np.abs(res.x[j, :5 * N] - w["states_b"])))}
            rows.append(r)
        st = np.array([r["status"] for r in rows[1:]])
        near = np.array([r["dx_fixture"] <= 1e-4 for r in rows[1:]])
        out[name] = {"oracle_fixture": {"status": int(g["status"]), "iters": int(g["iters"]), "n_resto": int(g["n_resto"])},
                     "runs": rows, "seconds": dt,
                     "neighbours_status_hist": {int(a): int(b) for a, b in zip(*np.unique(st, return_counts=True))},
                     "neighbours_at_fixture_point": int(near.sum())}
        print(f"{name}: fixture oracle {int(g['status'])}/{int(g['iters'])}/{int(g['n_resto'])} device "
              f"{rows[0]['status']}/{rows[0]['iters']}/{rows[0]['n_resto']} | neighbours {out[name]['neighbours_status_hist']}"
              f" at fixture point {int(near.sum())}/{len(near)} ({dt:.1f} s)", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
