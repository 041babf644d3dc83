"""Generate the full-size OBCA parity fixtures (tests/golden/obca_full/*.npz).

TEST INFRASTRUCTURE: the oracle (oracle/ipm.py IPOPT restatement with the
structured KKT of oracle/structured.py) solves selected problems of the
BASELINE configs A-E (synth.config_instance: shape, implement and turn type --
A fish-tail, B circle-back, C mixed, D/E Dubins -- the same Philox-seeded
workload as bench.py) on the CPU; each fixture stores the state trajectory (5N), the
objective, the status, the iteration count and the number of restoration
phases.  tests/test_gpu_obca.py compares the HIP solver against them (the
oracle needs minutes to hours per full-size problem, too slow to run inside a
GPU test).  Several pids are problems whose line search fails and that need
IPOPT's feasibility restoration (D 33/971, C 47, E 12).  Round 3 adds the problems the
solver does NOT solve -- config-C and config-E pids that end infeasible or at the iteration
limit (picked by tools/screen_failures.py) -- with max_cpu_time off, so the GPU's failure
statuses are pinned against the oracle's.  Every fixture stores its own input (inst_*
arrays, tests/_fixture_io.py), so it stays valid if the synthetic generator changes.

    python tests/golden/make_obca_golden.py [CFG:PID ...]
    python tests/golden/make_obca_golden.py --retrofit     # add inst_* to fixtures that lack them
"""
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.environ.get("HTP_GOLDEN_OUT", os.path.join(ROOT, "tests", "golden", "obca_full"))

CASES = ["A:0", "A:1", "A:2", "B:0", "B:1", "B:9", "D:0", "D:33", "D:971", "C:0", "C:1", "C:2", "C:47", "E:0", "E:1",
         "E:12"]
# Round 3, after configs A-E moved to the reference's scene producers (synth.make_orchard_instance):
# one converged problem per config plus the host-build screen's failures (profiles/r03h_screen_*.json)
CASES_R3 = ["A:3", "B:3", "C:3", "D:3", "E:3", "C:36", "C:59", "A:43", "D:347", "D:946"]


def run(case):
    from _fixture_io import instance_arrays
    from headland_trajectory_planning_amd import synth
    from oracle.ipm import IpoptRestatement
    from oracle.nlp import ObcaNLP
    from oracle.structured import StructuredKKT
    cfg, pid = case.split(":")
    pid = int(pid)
    _, N, M, imp = synth.CONFIGS[cfg]
    inst = synth.config_instance(cfg, pid)
    nlp = ObcaNLP(inst)
    t = time.time()
    r = IpoptRestatement(nlp, kkt=StructuredKKT(nlp)).solve()
    dt = time.time() - t
    np.savez(os.path.join(OUT, f"{cfg}{pid}.npz"), states=r["x"][:5 * N], f=r["f"], status=r["status"],
             iters=r["iters"], n_resto=r["n_resto"], N=N, M=M, implement=imp, turn=inst["meta"]["turn"], seconds=dt,
             status_str=r["status_str"], **instance_arrays(inst))
    return f"{case} {r['status_str']} iters={r['iters']} n_resto={r['n_resto']} f={r['f']:.12g} ({dt:.0f} s)"


def retrofit():
    import glob
    from _fixture_io import has_instance, instance_arrays
    from headland_trajectory_planning_amd import synth
    for f in sorted(glob.glob(os.path.join(OUT, "*.npz"))):
        z = np.load(f)
        if has_instance(z):
            continue
        name = os.path.basename(f)[:-4]
        inst = synth.config_instance(name[0], int(name[1:]))
        data = {k: z[k] for k in z.files}
        data.update(instance_arrays(inst))
        np.savez(f, **data)
        print("retrofit", name, flush=True)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    if sys.argv[1:] == ["--retrofit"]:
        retrofit()
        sys.exit(0)
    cases = sys.argv[1:] or CASES
    with mp.Pool(min(8, len(cases))) as pool:
        for line in pool.imap_unordered(run, cases):
            print(line, flush=True)
