"""Screen the point formulation (optimizer_points.py) for non-success statuses on the CPU.

Runs the solver core's test-only host build (tests/_hostsim.py: the same obca_core.h as the gfx950
kernel) over make_points_instance(pid, N, M) for pids [lo, hi) -- the instances tools/bench_points.py
solves -- and writes the status histogram plus the non-success pids to JSON.

    python tools/screen_points.py LO HI [--N 80] [--M 6] [--procs 4] [--out profiles/r03_screen_points.json]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _one(args):
    pid, N, M = args
    import _hostsim as H
    from headland_trajectory_planning_amd import synth
    r = H.solve_points([synth.make_points_instance(pid, N=N, M=M)])
    return pid, int(r.status[0]), int(r.iterations[0]), int(r.n_resto[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lo", type=int)
    ap.add_argument("hi", type=int)
    ap.add_argument("--N", type=int, default=80)
    ap.add_argument("--M", type=int, default=6)
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_screen_points.json"))
    a = ap.parse_args()
    import _hostsim as H
    H.build()
    rec = {"N": a.N, "M": a.M, "lo": a.lo, "hi": a.hi, "solver": "tests/_hostsim.py solve_points (obca_core.h host build)",
           "status_counts": {}, "failures": []}
    t0 = time.time()
    with mp.get_context("fork").Pool(a.procs) as pool:
        for k, (pid, st, it, nr) in enumerate(pool.imap_unordered(_one, [(p, a.N, a.M) for p in range(a.lo, a.hi)])):
            rec["status_counts"][str(st)] = rec["status_counts"].get(str(st), 0) + 1
            if st not in (0, 1):
                rec["failures"].append({"pid": pid, "status": st, "iters": it, "n_resto": nr})
            if k % 16 == 15:
                rec["seconds"] = time.time() - t0
                print(f"[screen_points] {k + 1}/{a.hi - a.lo}: {rec['status_counts']} ({rec['seconds']:.0f} s)", flush=True)
                with open(a.out, "w") as fh:
                    json.dump(rec, fh, indent=1)
    rec["seconds"] = time.time() - t0
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
