"""Summarise the hybrid A* / Y-park profiles of tools/gpu_evidence.sh (steps `hakt`, `hapmc`, `kernels`): kernel
time from rocprofv3 --kernel-trace --stats, the SQ counter passes of hastar_kernel as shares of its wave-cycles
(SQ cycle counters in quad-cycles, as tools/stall_summary.py), instruction counts per expansion and per pose test,
and the bench lines (searches/s, pose tests/s, CPU baseline).

    python tools/hastar_summary.py gpurun_out/r05i > profiles/r05i_hastar_summary.json
"""
import collections
import csv
import glob
import json
import os
import sys


def pmc(prefix, kernel):
    vals = collections.defaultdict(float)
    regs = {}
    for f in glob.glob(f"{prefix}_hapmc_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]] += float(r["Counter_Value"])
                regs = {k: r[k] for k in ("Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                          "LDS_Block_Size", "Grid_Size")}
    return vals, regs


def kstats(prefix, tag):
    out = {}
    for f in glob.glob(f"{prefix}_{tag}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[r["Name"][:90]] = {"calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                   "avg_ms": float(r["AverageNs"]) / 1e6}
    return out


def bench_line(path):
    try:
        for line in open(path):
            if line.startswith("{"):
                return json.loads(line)
    except OSError:
        pass
    return None


def main():
    prefix = sys.argv[1]
    out = {"prefix": prefix,
           "bench_hastar": bench_line(f"{prefix}_hastar.out"),
           "kernel_stats_hastar": kstats(prefix, "hakt"),
           "kernel_stats_ypark": kstats(prefix, "ypkt")}
    v, regs = pmc(prefix, "hastar_kernel")
    out["hastar_kernel_resources"] = regs
    wc = v.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        out["share_of_wave_cycles"] = {k[3:].lower(): v[k] / wc for k in sorted(v)
                                       if k.startswith("SQ_") and k not in ("SQ_WAVE_CYCLES", "SQ_WAVES")
                                       and ("ACTIVE" in k or "WAIT" in k)}
    prof = bench_line(glob.glob(f"{prefix}_hapmc_*.out")[0]) if glob.glob(f"{prefix}_hapmc_*.out") else None
    if prof and v:
        b = prof["batch"]
        exp = prof["mean_expansions"] * b
        out["per_expansion"] = {k: v[k] / exp for k in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                                                        "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VALU_TRANS_F64",
                                                        "SQ_INSTS_VALU_FMA_F64") if k in v}
        out["per_expansion"]["wave_cycles"] = 4 * wc / exp
        pt = prof.get("pose_tests_per_s", 0) * prof.get("kernel_ms", 0) / 1e3
        if pt:
            out["per_pose_test"] = {"valu": v.get("SQ_INSTS_VALU", 0) / pt, "wave_cycles": 4 * wc / pt}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
