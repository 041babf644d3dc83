"""Device-emulation fixtures for the solves where the device and the oracle part ways (tests/test_gpu_obca.py
FAILURE_CLASS_ONLY / DIVERGENT_AFTER_RESTORATION, tests/test_gpu_points.py CHAOTIC): the same instance through
the bit-exact host emulation of the device solver (csrc/htp_emusim.cpp + emu_wave.h: 64 lane threads, the
device's wave-reduction and matrix-core summation order, the device's contraction, the shared correctly
rounded libm).  tests/test_gpu_emulation.py asserts the device returns these doubles bit for bit; the serial
host build (HostLane, the oracle's summation order) ends where the oracle ends -- so the divergence is the
summation order and nothing else.

    python tests/golden/make_emulation.py D347 E84 E6 P19     -> tests/golden/emulation/<name>.npz
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.path.join(ROOT, "tests", "golden", "emulation")


def instance(name):
    """The fixture's instance and its kind ("full" or "points")."""
    from headland_trajectory_planning_amd import synth
    if name.startswith("P"):
        return synth.make_points_instance(int(name[1:]), N=12, M=2), "points"
    from _fixture_io import load_instance
    return load_instance(np.load(os.path.join(ROOT, "tests", "golden", "obca_full", f"{name}.npz"))), "full"


def run(name):
    import _hostsim as H
    t = time.time()
    inst, kind = instance(name)
    r = (H.solve_points_emusim if kind == "points" else H.solve_emusim)([inst])
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"{name}.npz"), x=r.x[0], status=int(r.status[0]), iters=int(r.iterations[0]),
             n_resto=int(r.n_resto[0]), objective=float(r.objective[0]), seconds=time.time() - t)
    return f"{name}: status {r.status[0]} it {r.iterations[0]} resto {r.n_resto[0]} ({time.time() - t:.0f} s)"


if __name__ == "__main__":
    import _hostsim as H
    H.build_emusim()
    import multiprocessing as mp
    with mp.Pool(min(3, len(sys.argv) - 1)) as pool:
        for line in pool.imap_unordered(run, sys.argv[1:]):
            print(line, flush=True)
