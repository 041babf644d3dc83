"""Device-emulation fixtures for the solves where the device and the oracle part ways (tests/test_gpu_obca.py
FAILURE_CLASS_ONLY / DIVERGENT_AFTER_RESTORATION, tests/test_gpu_points.py CHAOTIC): the same instance through
the bit-exact host emulation of the device solver (csrc/htp_emusim.cpp + emu_wave.h: 64 lane threads, the
device's wave-reduction and matrix-core summation order, the device's contraction, the shared correctly
rounded libm).  tests/test_gpu_emulation.py asserts the device returns these doubles bit for bit; the serial
host build (HostLane, the oracle's summation order) ends where the oracle ends -- so the divergence is the
summation order and nothing else.

    python tests/golden/make_emulation.py D347 E84 E6 P19     -> tests/golden/emulation/<name>.npz
    python tests/golden/make_emulation.py short               -> tests/golden/emulation/short_solves.npz
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


def short_groups():
    """tests/test_gpu_emulation.py::test_short_solves_equal_the_emulation's launches (one shape per launch)."""
    from headland_trajectory_planning_amd import synth
    insts = [synth.config_instance("D", p) for p in range(3)] + [synth.config_instance("C", 0),
                                                                  synth.config_instance("A", 1)]
    W = np.diag([10.0, 0.1])
    insts += [synth.make_instance(p, N=12, M=2, implement="mower", W=W) for p in (0, 3)]   # restoration phases
    return [[insts[k] for k in (0, 1, 2)], [insts[3]], [insts[4]], insts[5:]]


def emu_key():
    """Hash of every source the emulation's doubles depend on: the solver core (_native.core_sha) and the
    emulation itself (csrc/emu_wave.h, csrc/htp_emusim.cpp, the MFMA model in csrc/wave_ctx.h)."""
    import hashlib
    from headland_trajectory_planning_amd import _native
    h = hashlib.sha256(_native.core_sha().encode())
    for f in ("emu_wave.h", "htp_emusim.cpp"):
        with open(os.path.join(ROOT, "headland_trajectory_planning_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def group_hash(group):
    from make_oracle_screen import inst_hash
    import hashlib
    return hashlib.sha256("".join(inst_hash(i) for i in group).encode()).hexdigest()[:16]


def run_short():
    """The short solves' emulation, cached (the live run takes minutes of host time on the GPU box):
    tests/golden/emulation/short_solves.npz, keyed by emu_key() and each launch's instance hash."""
    import _hostsim as H
    t = time.time()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    out = {"key": emu_key()}
    for g, group in enumerate(short_groups()):
        r = H.solve_emusim(group)
        out.update({f"g{g}_hash": group_hash(group), f"g{g}_x": r.x, f"g{g}_status": r.status,
                    f"g{g}_iters": r.iterations, f"g{g}_n_resto": r.n_resto, f"g{g}_objective": r.objective})
    out["ngroups"] = len(short_groups())
    out["seconds"] = time.time() - t
    np.savez(os.path.join(OUT, "short_solves.npz"), **out)
    return f"short solves: {out['ngroups']} launches emulated ({time.time() - t:.0f} s), key {out['key']}"


if __name__ == "__main__":
    import _hostsim as H
    H.build_emusim()
    if sys.argv[1:] == ["short"]:
        print(run_short(), flush=True)
        sys.exit(0)
    import multiprocessing as mp
    with mp.Pool(min(3, len(sys.argv) - 1)) as pool:
        for line in pool.imap_unordered(run, sys.argv[1:]):
            print(line, flush=True)
