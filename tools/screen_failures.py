"""Screen a config's problems for non-success statuses on the CPU build of the solver core.

Runs libhtp_cpu.so (csrc/obca_core.h compiled for the host, the same source as the gfx950 kernel)
over problem ids [lo, hi) of a BASELINE config with max_cpu_time off, and writes the status
histogram plus every non-success pid (status, iterations, restoration phases) to a JSON file.
The oracle fixtures of tests/golden/make_obca_golden.py are then made for a selection of those pids.

    python tools/screen_failures.py CFG LO HI [--threads 8] [--out profiles/r03_screen_CFG.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from headland_trajectory_planning_amd import _native, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg")
    ap.add_argument("lo", type=int)
    ap.add_argument("hi", type=int)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "headland_trajectory_planning_amd", "libhtp_cpu.so"))
    lib.htp_cpu_obca_solve_range.argtypes = [ctypes.POINTER(_native.ObcaBatch), ctypes.POINTER(_native.ObcaResult),
                                             ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    lib.htp_cpu_obca_solve_range.restype = ctypes.c_int
    out = a.out or os.path.join(ROOT, "profiles", f"r03_screen_{a.cfg}.json")
    rec = {"config": a.cfg, "lo": a.lo, "hi": a.hi, "solver": "libhtp_cpu.so (obca_core.h host build)",
           "max_cpu_time": "off", "status_counts": {}, "failures": [], "iters": []}
    t0 = time.time()
    for c0 in range(a.lo, a.hi, a.chunk):
        pids = list(range(c0, min(a.hi, c0 + a.chunk)))
        pk = _native.PackedBatch([synth.config_instance(a.cfg, p) for p in pids])
        res = _native.HostResults(pk.batch, pk.n_var)
        b, r = pk.struct(), res.struct()
        if lib.htp_cpu_obca_solve_range(ctypes.byref(b), ctypes.byref(r), 0, pk.batch, a.threads) != 0:
            raise RuntimeError("htp_cpu_obca_solve_range failed")
        for k, p in enumerate(pids):
            st = int(res.status[k])
            rec["status_counts"][str(st)] = rec["status_counts"].get(str(st), 0) + 1
            rec["iters"].append(int(res.iterations[k]))
            if st not in (0, 1):
                rec["failures"].append({"pid": p, "status": st, "iters": int(res.iterations[k]),
                                        "n_resto": int(res.n_resto[k])})
        rec["seconds"] = time.time() - t0
        print(f"[screen] {a.cfg} {c0 + len(pids)}/{a.hi}: {rec['status_counts']} ({rec['seconds']:.0f} s)", flush=True)
        with open(out, "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
