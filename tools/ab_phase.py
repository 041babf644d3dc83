"""A/B of libhtp_<name>.so variants on one config batch (experiments only):
kernel time, solves/s, bit-identity against the first variant, and the
per-phase cycle shares; variants built with -DHTP_KKT_PROF report the KKT
solve's sub-phases (local rhs sweep, stage Riccati solve, local back sweep) in
the last three slots.   python tools/ab_phase.py CFG B name1 name2 ..."""
import sys

import numpy as np

sys.path.insert(0, ".")
from headland_trajectory_planning_amd import _native  # noqa: E402
import bench  # noqa: E402

cfg, B = sys.argv[1], int(sys.argv[2])
names = sys.argv[3:]
pk = _native.PackedBatch(bench.make_batch(list(range(B)), cfg, 16))
ctxs = {}
for n in names:
    path = _native.LIB_PATH if n == "base" else _native.LIB_PATH.replace("libhtp.so", f"libhtp_{n}.so")
    ctxs[n] = _native.Context(0, lib=_native.load(path))
ref = None
for rnd in range(2):
    for k, ctx in ctxs.items():
        r = ctx.solve(pk)
        ms = ctx.last_kernel_ms()
        ok = ""
        if ref is None:
            ref = r
        else:
            ok = f" max|dx|={np.max(np.abs(ref.x - r.x)):.2e} status_eq={np.array_equal(ref.status, r.status)} " \
                 f"iters_eq={np.array_equal(ref.iterations, r.iterations)}"
        line = f"round {rnd} {k}: kernel {ms:.1f} ms {B / (ms / 1e3):.0f} solves/s iters {r.iterations.mean():.2f}{ok}"
        if rnd == 1:
            cyc = ctx.last_cycles(B).astype(float)
            tot = cyc[:, 4].sum()
            tail = ["rhs_sweep", "ric_solve", "back_sweep"] if "kprof" in k else ["errors", "linesearch", "update"]
            head = ["build", "ldlt", "schur"] if "lprof" in k else ["local", "assemble", "chain"]
            nm = head + ["kktsolve", "total"] + tail
            if "kp2" in k:   # HTP_KKT_PROF=2: rhs sweep, stage rhs, Riccati backward, forward, ric+scatter, back sweep, n_kkt
                nm = ["rhs_sweep", "stage_rhs", "ric_bwd", "ric_fwd", "total", "ric+scatter", "back_sweep", "n_kkt"]
                line += " | kkt solves per iteration %.3f" % (cyc[:, 7].sum() / max(1, r.iterations.sum()))
            if "lq" in k.split("_")[0]:   # HTP_LPROF=2: pass 2 split (build, factor, solves)
                nm = ["p2_build", "pass2_cyc", "p2_factor", "p2_solves", "total", "scan_cyc", "n_piv", "n_sweeps"]
                sw = max(1.0, cyc[:, 7].sum())
                line += " | per sweep: pass2 %.0f cyc = build %.0f + factor %.0f + solves %.0f, %.1f pivoted blocks" % (
                        cyc[:, 1].sum() / sw, cyc[:, 0].sum() / sw, cyc[:, 2].sum() / sw, cyc[:, 3].sum() / sw,
                        cyc[:, 6].sum() / sw)
            elif "lp" in k.split("_")[0] and "prof" not in k:   # HTP_LPROF: local factor sweep
                nm = ["pass1_cyc", "pass2_cyc", "pass1_trips", "pass2_trips", "total", "scan_cyc", "n_piv", "n_sweeps"]
                sw = max(1.0, cyc[:, 7].sum())
                line += " | per sweep: pass1 %.0f cyc (%.2f trips), pass2 %.0f cyc (%.2f trips), scan %.0f cyc, %.1f " \
                        "pivoted blocks; sweeps per iteration %.2f" % (cyc[:, 0].sum() / sw, cyc[:, 2].sum() / sw,
                        cyc[:, 1].sum() / sw, cyc[:, 3].sum() / sw, cyc[:, 5].sum() / sw, cyc[:, 6].sum() / sw,
                        sw / max(1, r.iterations.sum()))
            if "prof" in k and "kprof" not in k:   # HTP_PROF_ON: stage-chain sub-steps (factor 1/3/5, solve 6/7)
                nm = ["fac_relax", "fac_mfma", "fac_pn_store", "fac_chol", "total", "fac_sym", "solve_bwd*", "solve_fwd"]
            if "sprof" in k:   # HTP_PROF_ON=2: solve passes split into ring fills and stage steps
                nm = ["bwd_fill", "bwd_stage", "fwd_fill", "fwd_stage", "total", "fac_mfma", "fac_chol", "fac_tail"]
            line += " | " + " ".join(f"{nm[j]} {cyc[:, j].sum() / tot:.3f}" for j in (0, 1, 2, 3, 5, 6, 7))
            line += " | per-iter cycles %.3g" % (cyc[:, 4] / np.maximum(1, r.iterations)).mean()
        print(line, flush=True)
