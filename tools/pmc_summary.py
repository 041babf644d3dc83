"""Summarise the rocprofv3 PMC passes of tools/gpu_pmc.sh into the JSON files
bench.py reads (profiles/<tag>_traffic.json, profiles/<tag>_mfma.json).

    python tools/pmc_summary.py gpurun_out TAG CONFIG [OUT_TAG]

Per pass (fetch / write / sq) the CSV rows of the solver kernel are summed;
the bench JSON line each pass printed gives the launch's problem-iterations.
Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE (kB) is doubled for gfx950 (128-B requests tallied at 64 B; an
upper estimate for the solver's 8-B/lane gathers, raw value kept);
WRITE_SIZE (kB) as is.  GRBM_GUI_ACTIVE is the sum over the 8 XCDs of the
busy clock (MI355X_MICROARCH.md, DVFS item), SQ_VALU_MFMA_BUSY_CYCLES the sum
over the SIMDs, so MFMA busy fraction = MFMA_BUSY / (GUI_ACTIVE / 8 x 1024
SIMDs); it agrees with the FLOP-based utilisation (SQ_INSTS_VALU_MFMA_MOPS_F64
x 512 FLOP / kernel time / the 78.6 TFLOP/s FP64 matrix peak, spec)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from headland_trajectory_planning_amd import _native  # noqa: E402

KERNEL = "obca_"
N_CU = 256
N_XCD = 8
F64_MFMA_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix (spec)


def rows(base, tag, name):
    out = {}
    meta = {}
    for f in glob.glob(os.path.join(base, f"{tag}_pmc_{name}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta = dict(kernel=r["Kernel_Name"], grid=int(r["Grid_Size"]), scratch=int(r["Scratch_Size"]),
                        vgpr=int(r["VGPR_Count"]), agpr=int(r["Accum_VGPR_Count"]), sgpr=int(r["SGPR_Count"]),
                        lds=int(r["LDS_Block_Size"]),
                        ns=int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out, meta


def bench_line(base, tag, name):
    for line in open(os.path.join(base, f"{tag}_pmc_{name}.log")):
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"no bench line in {tag}_pmc_{name}.log")


def main():
    base, tag, cfg = sys.argv[1:4]
    out_tag = sys.argv[4] if len(sys.argv) > 4 else tag
    sha = _native.core_sha()
    fetch, meta = rows(base, tag, "fetch")
    write, _ = rows(base, tag, "write")
    bl_f, bl_w = bench_line(base, tag, "fetch"), bench_line(base, tag, "write")
    it_f = bl_f["solver"]["mean_iters"] * bl_f["config"]["global_batch"] * bl_f["steps"]
    it_w = bl_w["solver"]["mean_iters"] * bl_w["config"]["global_batch"] * bl_w["steps"]
    fkb, wkb = fetch["FETCH_SIZE"], write["WRITE_SIZE"]
    alg = bl_f["roofline"]["bytes_per_iter_per_problem"]
    per_it_x2 = (2 * fkb * 1024) / it_f + (wkb * 1024) / it_w
    per_it_raw = (fkb * 1024) / it_f + (wkb * 1024) / it_w
    from tools.kernel_resources import kernels
    import re
    m = re.search(r"obca_solve_kernel<(\d+), (\d+), (\d+)>", meta.get("kernel", ""))
    want = "obca_solve_kernelILi%sELi%sELi%sE" % m.groups() if m else "obca_solve_kernelILi4ELi4ELi0E"
    co = {k: v for k, v in kernels(_native.LIB_PATH).items() if want in k}
    traffic = {
        "workload": cfg, "batch": bl_f["config"]["global_batch"], "solver_sha": sha, "kernel": meta.get("kernel"),
        "binary": bl_f.get("binary"),
        # from the loaded library's gfx950 code object (tools/kernel_resources.py): VGPR = unified count (arch +
        # accumulation registers), spills, private segment (scratch bytes per lane), LDS bytes per workgroup
        "resources": next(iter(co.values()), None),
        "resources_profiler_csv": {k: meta.get(k) for k in ("grid", "scratch", "vgpr", "agpr", "sgpr", "lds")},
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/gpu_pmc.sh), one "
                  "persistent launch each; counters in kB",
        "FETCH_SIZE_kB": fkb, "WRITE_SIZE_kB": wkb,
        "launch_iterations_fetch_pass": it_f, "launch_iterations_write_pass": it_w,
        "bytes_per_problem_iter": per_it_raw, "bytes_per_problem_iter_raw": per_it_raw,
        "bytes_per_problem_iter_fetch_x2": per_it_x2,
        "algorithmic_bytes_per_problem_iter": alg, "traffic_over_algorithmic": per_it_raw / alg,
        "traffic_over_algorithmic_fetch_x2": per_it_x2 / alg,
        "correction": "primary figure: FETCH_SIZE + WRITE_SIZE as counted.  MI355X_MICROARCH.md's FETCH x2 applies to "
                      "16-B/lane streaming reads (128-B requests tallied at 64 B); the solver's loads are 8-B/lane fp64 "
                      "gathers and sweeps, so the x2 figure is an upper bound, kept as *_fetch_x2",
    }
    sq, smeta = rows(base, tag, "sq")
    bl_s = bench_line(base, tag, "sq")
    it_s = bl_s["solver"]["mean_iters"] * bl_s["config"]["global_batch"] * bl_s["steps"]
    mf = {"workload": cfg, "solver_sha": sha, "kernel": smeta.get("kernel"), "binary": bl_s.get("binary"),
          "counters": sq, "launch_iterations": it_s}
    if sq:
        mf["mfma_f64_per_problem_iter"] = sq.get("SQ_INSTS_VALU_MFMA_F64", 0.0) / it_s
        mf["mfma_mops_f64_per_problem_iter"] = sq.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) / it_s
        mf["valu_per_problem_iter"] = sq.get("SQ_INSTS_VALU", 0.0) / it_s
        if sq.get("GRBM_GUI_ACTIVE"):
            mf["mfma_busy_frac"] = sq.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (sq["GRBM_GUI_ACTIVE"] / N_XCD * N_CU * 4)
            mf["clock_ghz"] = sq["GRBM_GUI_ACTIVE"] / N_XCD / smeta["ns"] if smeta.get("ns") else None
        # MOPS are units of 512 FLOP (one v_mfma_f64_16x16x4f64 = 2*16*16*4 = 2048 FLOP = 4 MOPS)
        if smeta.get("ns"):
            mf["mfma_f64_tflops"] = sq.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512 / (smeta["ns"] * 1e-9) / 1e12
            mf["mfma_f64_frac_of_peak"] = mf["mfma_f64_tflops"] / F64_MFMA_PEAK_TFLOPS
            mf["kernel_ms"] = smeta["ns"] * 1e-6
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for name, obj in (("traffic", traffic), ("mfma", mf)):
        path = os.path.join(ROOT, "profiles", f"{out_tag}_{name}_{cfg}.json")
        json.dump(obj, open(path, "w"), indent=1)
        print(path, json.dumps(obj)[:600])


if __name__ == "__main__":
    main()
