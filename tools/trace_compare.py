"""Iteration-by-iteration comparison of the device solve (its bit-exact host emulation, csrc/emu_wave.h built
with -DHTP_TRACE_ON) against the oracle (oracle/ipm.py) on one parity fixture.

    python tools/trace_compare.py oracle E12 [--ulp K]        -> gpurun_out/trace/E12_oracle.json
    python tools/trace_compare.py emu E12 --max-iter 400      -> gpurun_out/trace/E12_emu.json
    python tools/trace_compare.py host E12 --max-iter 400     -> the serial host build (HostLane)
    python tools/trace_compare.py diff E12                    -> first iteration whose errors differ, and the
                                                                 first whose restoration flag differs

Per iteration: restoration flag, mu and the unscaled dual / complementarity / primal errors at mu = 0 (the
quantities IPOPT prints), each side's own computation.  TEST INFRASTRUCTURE."""
import argparse
import ctypes
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.path.join(ROOT, "gpurun_out", "trace")
TRACE_SO = os.path.join(ROOT, "build", "libhtp_emusim_trace.so")
HOST_TRACE_SO = os.path.join(ROOT, "build", "libhtp_hostsim_trace.so")
CSRC = os.path.join(ROOT, "headland_trajectory_planning_amd", "csrc")


def instance(name, ulp):
    from _fixture_io import load_instance
    from _neighbours import neighbour
    inst = load_instance(np.load(os.path.join(ROOT, "tests", "golden", "obca_full", f"{name}.npz")))
    return neighbour(inst, ulp)[0] if ulp is not None else inst


def tag(name, ulp):
    return name if ulp is None else f"{name}_ulp{ulp}"


def run_oracle(name, ulp, max_iter):
    from oracle.ipm import IpoptRestatement
    from oracle.nlp import ObcaNLP
    from oracle.structured import StructuredKKT
    nlp = ObcaNLP(instance(name, ulp))
    ip = IpoptRestatement(nlp, opts={"max_iter": max_iter} if max_iter else None, kkt=StructuredKKT(nlp))
    r = ip.solve()
    rows = [dict(it=int(e["it"]), resto=bool(e["resto"]), mu=float(e["mu"]), dual=float(e["dual"]),
                 comp=float(e["comp"]), prim=float(e["prim"])) for e in ip.log]
    return {"status": int(r["status"]), "iters": int(r["iters"]), "n_resto": int(r["n_resto"]), "rows": rows}


def _build(kind):
    if kind == "emu":
        if not os.path.exists(TRACE_SO):
            subprocess.check_call(["/opt/rocm/lib/llvm/bin/clang++", "-O2", "-std=c++20", "-ffp-contract=on", "-mfma",
                                   "-shared", "-fPIC", "-DHTP_TRACE_ON", "-o", TRACE_SO,
                                   os.path.join(CSRC, "htp_emusim.cpp"), "-lpthread"])
        return TRACE_SO
    if not os.path.exists(HOST_TRACE_SO):
        subprocess.check_call(["g++", "-O2", "-fno-builtin", "-std=c++17", "-shared", "-fPIC", "-DHTP_TRACE_ON", "-o",
                               HOST_TRACE_SO, os.path.join(CSRC, "htp_hostsim.cpp"),
                               os.path.join(CSRC, "rs_hostsim.cpp"), os.path.join(CSRC, "hastar_hostsim.cpp"),
                               os.path.join(CSRC, "ypark_hostsim.cpp"), os.path.join(CSRC, "refpath_hostsim.cpp"),
                               os.path.join(CSRC, "oge_hostsim.cpp"), os.path.join(CSRC, "classic_hostsim.cpp"),
                               os.path.join(CSRC, "chain_hostsim.cpp")])
    return HOST_TRACE_SO


LINE = re.compile(r"\[trace\] it (\d+)( R)? err dual=(\S+) comp=(\S+) prim=(\S+) mu=(\S+)")


def run_device_model(kind, name, ulp, max_iter):
    """The traced build prints from lane 0 to the process's stdout: run it in a child with stdout to a file."""
    so = _build(kind)
    fd, path = tempfile.mkstemp(suffix=".txt")
    os.close(fd)
    code = (f"import sys, json, ctypes; sys.path[:0] = [{ROOT!r}, {os.path.join(ROOT, 'tests')!r}]\n"
            f"from tools.trace_compare import _child; _child({kind!r}, {name!r}, {ulp!r}, {max_iter!r})")
    with open(path, "w") as f:
        subprocess.check_call([sys.executable, "-c", code], stdout=f)
    rows, summary = [], None
    for ln in open(path):
        m = LINE.search(ln)
        if m:
            rows.append(dict(it=int(m.group(1)), resto=bool(m.group(2)), dual=float(m.group(3)),
                             comp=float(m.group(4)), prim=float(m.group(5)), mu=float(m.group(6))))
        elif "RESULT " in ln:
            summary = json.loads(ln[ln.index("RESULT ") + 7:])
    os.unlink(path)
    return dict(summary, rows=rows)


def _child(kind, name, ulp, max_iter):
    from headland_trajectory_planning_amd import _native
    L = ctypes.CDLL(_build(kind))
    fn = L.htp_emusim_obca_solve if kind == "emu" else L.htp_hostsim_obca_solve
    fn.argtypes = [ctypes.POINTER(_native.ObcaBatch), ctypes.POINTER(_native.ObcaResult), ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    opts = {"max_iter": float(max_iter)} if max_iter else {}
    names = (ctypes.c_char_p * max(1, len(opts)))(*[k.encode() for k in opts])
    vals = (ctypes.c_double * max(1, len(opts)))(*[float(v) for v in opts.values()])
    pk = _native.PackedBatch([instance(name, ulp)])
    res = _native.HostResults(pk.batch, pk.n_var)
    assert fn(ctypes.byref(pk.struct()), ctypes.byref(res.struct()), names, vals, len(opts)) == 0
    sys.stdout.flush()
    ctypes.CDLL(None).fflush(None)   # the traced build's printf lines first
    os.write(1, ("\nRESULT " + json.dumps({"status": int(res.status[0]), "iters": int(res.iterations[0]),
                                         "n_resto": int(res.n_resto[0])}) + "\n").encode())


def diff(a, b):
    ra, rb = a["rows"], b["rows"]
    n = min(len(ra), len(rb))
    first_err, first_flag, out = None, None, []
    for i in range(n):
        x, y = ra[i], rb[i]
        rel = max(abs(x[k] - y[k]) / max(abs(x[k]), abs(y[k]), 1e-300) for k in ("dual", "comp", "prim", "mu"))
        out.append(rel)
        if first_err is None and rel > 1e-6:
            first_err = i
        if first_flag is None and x["resto"] != y["resto"]:
            first_flag = i
    return {"compared": n, "first_rel_gt_1e-6": first_err, "first_resto_flag_differs": first_flag,
            "rel_by_iter": out}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["oracle", "emu", "host", "diff"])
    ap.add_argument("name")
    ap.add_argument("--ulp", type=int, default=None)
    ap.add_argument("--max-iter", type=int, default=0)
    ap.add_argument("--against", default="emu")
    args = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    t = tag(args.name, args.ulp)
    if args.mode == "diff":
        a = json.load(open(os.path.join(OUT, f"{t}_oracle.json")))
        b = json.load(open(os.path.join(OUT, f"{t}_{args.against}.json")))
        d = diff(a, b)
        rel = d.pop("rel_by_iter")
        print(json.dumps(d))
        for i in range(d["compared"]):
            x, y = a["rows"][i], b["rows"][i]
            print(f"{i:5d} {'R' if x['resto'] else ' '}{'R' if y['resto'] else ' '} rel {rel[i]:.2e}  mu {x['mu']:.3e} "
                  f"{y['mu']:.3e}  dual {x['dual']:.6e} {y['dual']:.6e}  prim {x['prim']:.6e} {y['prim']:.6e}")
        return
    r = run_oracle(args.name, args.ulp, args.max_iter) if args.mode == "oracle" else \
        run_device_model(args.mode, args.name, args.ulp, args.max_iter)
    json.dump(r, open(os.path.join(OUT, f"{t}_{args.mode}.json"), "w"))
    print(f"{t} {args.mode}: status {r['status']} iters {r['iters']} n_resto {r['n_resto']} rows {len(r['rows'])}")


if __name__ == "__main__":
    main()
