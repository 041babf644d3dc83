"""Oracle self-divergence witnesses for the fixtures where the device and the oracle fixture part ways
inside long restoration cycles (tests/test_gpu_obca.py FAILURE_CLASS_ONLY / DIVERGENT_AFTER_RESTORATION,
tests/test_gpu_points.py CHAOTIC): the same oracle (oracle/ipm.py, IPOPT 3.14 restated) on the same instance
with a second, equally valid elimination order of the same KKT systems (StructuredKKTLoop for the full-size
fixtures, StructuredPointKKT for the point formulation, whose fixtures use DenseKKT).  Where the two orders
already end at different statuses or points, the reference algorithm itself does not determine the outcome at
rounding level, and the device's different-but-valid ending is the same phenomenon.

    python tests/golden/make_witness.py D347 E84 E6 P19     -> tests/golden/witness/<name>.npz

Libm witnesses (oracle/libm.py): the same oracle, the same KKT elimination (StructuredKKT) and the same
instance, with the transcendental functions taken from glibc (CPython's math module -- the functions CasADi's
SX VM calls in the reference's own solve) instead of numpy's AVX-512 kernels:

    python tests/golden/make_witness.py E12:glibc E54:glibc  -> tests/golden/witness/<name>_libm.npz

Input-rounding witnesses: the same oracle on the fixture's instance with ONE input double moved by one ulp
(init_traj[tests/_neighbours.ulp_cell(K, N)], np.nextafter; each file stores the moved (row, col) as `cell`),
i.e. an instance the reference cannot tell apart from the fixture's after its own float parsing and arithmetic:

    python tests/golden/make_witness.py E12:ulp0 E12:ulp1   -> tests/golden/witness/<name>_ulp<K>.npz
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.environ.get("HTP_WITNESS_OUT", os.path.join(ROOT, "tests", "golden", "witness"))


def run(name):
    try:
        return _run(name)
    except Exception as e:  # noqa: BLE001 -- one run's failure must not end the others (pool)
        return f"{name}: ERROR {type(e).__name__}: {e}"


def _run(name):
    from oracle.ipm import IpoptRestatement
    t = time.time()
    if name.endswith(":glibc"):
        return run_libm(name.split(":")[0], t)
    if ":ulp" in name:
        return run_ulp(name.split(":")[0], int(name.split(":ulp")[1]), t)
    if name.startswith("P"):   # point formulation, tests/test_gpu_points.py small instances (N=12, M=2)
        from headland_trajectory_planning_amd import synth
        from oracle.nlp_points import PointNLP
        from oracle.structured import StructuredPointKKT
        inst = synth.make_points_instance(int(name[1:]), N=12, M=2)
        nlp = PointNLP(inst)
        a = IpoptRestatement(nlp).solve()
        b = IpoptRestatement(nlp, kkt=StructuredPointKKT(nlp)).solve()
        orders = ("DenseKKT", "StructuredPointKKT")
        N = 12
    else:
        from _fixture_io import load_instance
        from oracle.nlp import ObcaNLP
        from oracle.structured import StructuredKKT, StructuredKKTLoop
        g = np.load(os.path.join(ROOT, "tests", "golden", "obca_full", f"{name}.npz"))
        inst = load_instance(g)
        nlp = ObcaNLP(inst)
        a = {"x": np.concatenate([g["states"], np.zeros(1)]), "status": int(g["status"]), "iters": int(g["iters"]),
             "n_resto": int(g["n_resto"]), "f": float(g["f"])}   # the fixture itself (StructuredKKT)
        b = IpoptRestatement(nlp, kkt=StructuredKKTLoop(nlp)).solve()
        orders = ("StructuredKKT", "StructuredKKTLoop")
        N = int(g["N"])
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"{name}.npz"), orders=np.array(orders),
             states_a=a["x"][:5 * N], status_a=a["status"], iters_a=a["iters"], n_resto_a=a["n_resto"],
             states_b=b["x"][:5 * N], status_b=b["status"], iters_b=b["iters"], n_resto_b=b["n_resto"],
             seconds=time.time() - t)
    d = float(np.max(np.abs(a["x"][:5 * N] - b["x"][:5 * N])))
    return (f"{name}: {orders[0]} status {a['status']} it {a['iters']} resto {a['n_resto']} | {orders[1]} status "
            f"{b['status']} it {b['iters']} resto {b['n_resto']} | max state diff {d:.3g} ({time.time() - t:.0f} s)")


def run_libm(name, t):
    from _fixture_io import load_instance
    from oracle import libm
    from oracle.ipm import IpoptRestatement
    from oracle.nlp import ObcaNLP
    from oracle.structured import StructuredKKT
    g = np.load(os.path.join(ROOT, "tests", "golden", "obca_full", f"{name}.npz"))
    nlp = ObcaNLP(load_instance(g))
    N = int(g["N"])
    a = {"x": g["states"], "status": int(g["status"]), "iters": int(g["iters"]), "n_resto": int(g["n_resto"])}
    libm.set_mode("glibc")
    b = IpoptRestatement(nlp, kkt=StructuredKKT(nlp)).solve()
    libm.set_mode("numpy")
    orders = ("StructuredKKT/numpy-libm", "StructuredKKT/glibc-libm")
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"{name}_libm.npz"), orders=np.array(orders),
             states_a=a["x"][:5 * N], status_a=a["status"], iters_a=a["iters"], n_resto_a=a["n_resto"],
             states_b=b["x"][:5 * N], status_b=b["status"], iters_b=b["iters"], n_resto_b=b["n_resto"],
             seconds=time.time() - t)
    d = float(np.max(np.abs(a["x"][:5 * N] - b["x"][:5 * N])))
    return (f"{name} libm: numpy status {a['status']} it {a['iters']} resto {a['n_resto']} | glibc status "
            f"{b['status']} it {b['iters']} resto {b['n_resto']} | max state diff {d:.3g} ({time.time() - t:.0f} s)")


def run_ulp(name, k, t):
    from _fixture_io import load_instance
    from oracle.ipm import IpoptRestatement
    from oracle.nlp import ObcaNLP
    from oracle.structured import StructuredKKT
    g = np.load(os.path.join(ROOT, "tests", "golden", "obca_full", f"{name}.npz"))
    inst = load_instance(g)
    from _neighbours import neighbour
    inst, (row, col) = neighbour(inst, k)
    nlp = ObcaNLP(inst)
    N = int(g["N"])
    a = {"x": g["states"], "status": int(g["status"]), "iters": int(g["iters"]), "n_resto": int(g["n_resto"])}
    b = IpoptRestatement(nlp, kkt=StructuredKKT(nlp)).solve()
    orders = ("StructuredKKT", f"StructuredKKT, init_traj[{row},{col}] + 1 ulp")
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"{name}_ulp{k}.npz"), orders=np.array(orders),
             states_a=a["x"][:5 * N], status_a=a["status"], iters_a=a["iters"], n_resto_a=a["n_resto"],
             states_b=b["x"][:5 * N], status_b=b["status"], iters_b=b["iters"], n_resto_b=b["n_resto"],
             f_b=b["f"], cell=np.array([row, col]), seconds=time.time() - t)
    d = float(np.max(np.abs(a["x"][:5 * N] - b["x"][:5 * N])))
    return (f"{name} ulp{k}: fixture status {a['status']} it {a['iters']} resto {a['n_resto']} | +1 ulp status "
            f"{b['status']} it {b['iters']} resto {b['n_resto']} | max state diff {d:.3g} ({time.time() - t:.0f} s)")


if __name__ == "__main__":
    import multiprocessing as mp
    with mp.Pool(min(int(os.environ.get("HTP_PROCS", "4")), len(sys.argv) - 1)) as pool:
        for line in pool.imap_unordered(run, sys.argv[1:]):
            print(line, flush=True)
