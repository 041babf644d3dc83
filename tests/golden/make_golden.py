"""Generate golden vectors from the reference's own importable modules.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py
Imports (read-only, no bytecode written) R/path_planner/utils/reeds_shepp.py
and R/path_planner/utils/cubic_spline.py -- both import only math/numpy/scipy/
matplotlib -- and stores inputs + outputs as .npz data fixtures.  No reference
source is copied; the GPU box never reads /root/reference.
"""
import math
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference/path_planner/utils"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import matplotlib
    matplotlib.use("Agg")
    sys.path.insert(0, REF)
    import cubic_spline as ref_spline  # noqa: E402
    import reeds_shepp as ref_rs  # noqa: E402

    rng = np.random.default_rng(20251015)
    # ---- Reeds-Shepp: calc_all_paths over random pose pairs
    maxcs = [math.tan(0.55) / 1.9, math.tan(0.5) / 1.9, 0.5]
    cases, lens, ctyp, Ls, pts, pathoff, ptoff = [], [], [], [], [], [0], [0]
    for k in range(120):
        s = (rng.uniform(-5, 5), rng.uniform(-5, 5), rng.uniform(-math.pi, math.pi))
        g = (rng.uniform(-8, 8), rng.uniform(-8, 8), rng.uniform(-math.pi, math.pi))
        maxc = maxcs[k % 3]
        step = [0.2, 0.1][k % 2]
        paths = ref_rs.calc_all_paths(*s, *g, maxc, step_size=step)
        cases.append(list(s) + list(g) + [maxc, step])
        for p in paths:
            lens.append(np.pad(np.asarray(p.lengths, dtype=np.float64), (0, 5 - len(p.lengths))))
            ctyp.append("".join(p.ctypes).ljust(5, "_"))
            Ls.append(p.L)
            arr = np.stack([p.x, p.y, p.yaw, p.directions, p.cs], axis=1).astype(np.float64)
            pts.append(arr)
            ptoff.append(ptoff[-1] + arr.shape[0])
        pathoff.append(len(Ls))
    np.savez_compressed(os.path.join(HERE, "rs_calc_all_paths.npz"),
                        cases=np.array(cases), path_offsets=np.array(pathoff), lengths=np.array(lens),
                        ctypes=np.array(ctyp), L=np.array(Ls), point_offsets=np.array(ptoff),
                        points=np.concatenate(pts, axis=0))
    # ---- cubic spline: calc_spline_course on random polylines
    sc, sx, sy, soff, out, ooff = [], [], [], [0], [], [0]
    for k in range(40):
        n = int(rng.integers(4, 12))
        t = np.cumsum(rng.uniform(0.3, 1.5, n))
        xs = t * math.cos(rng.uniform(-3, 3)) + rng.normal(0, 0.3, n)
        ys = t * math.sin(rng.uniform(-3, 3)) + rng.normal(0, 0.3, n)
        if k % 5 == 0:  # consecutive duplicate (singular) point
            xs = np.insert(xs, 2, xs[2])
            ys = np.insert(ys, 2, ys[2])
        ds = [0.1, 0.2][k % 2]
        rx, ry, ryaw, rk, s = ref_spline.calc_spline_course(xs, ys, ds=ds)
        sc.append(ds)
        sx.append(xs)
        sy.append(ys)
        soff.append(soff[-1] + len(xs))
        o = np.stack([np.asarray(rx, float), np.asarray(ry, float), np.asarray(ryaw, float),
                      np.asarray(rk, float), np.asarray(s, float)], axis=1)
        out.append(o)
        ooff.append(ooff[-1] + o.shape[0])
    np.savez_compressed(os.path.join(HERE, "spline_course.npz"), ds=np.array(sc), x=np.concatenate(sx),
                        y=np.concatenate(sy), in_offsets=np.array(soff), out=np.concatenate(out),
                        out_offsets=np.array(ooff))
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
