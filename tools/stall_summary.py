"""Summarise tools/gpu_stall.sh's PMC passes for the OBCA solve kernel: share of wave-cycles issuing each
instruction class vs waiting, average VMEM / LDS latency, instruction counts per problem-iteration.

Usage: python tools/stall_summary.py gpurun_out/r03sD [out.json]"""
import collections
import csv
import glob
import json
import os
import sys


def counters(prefix, name):
    vals = collections.defaultdict(float)
    files = glob.glob(os.path.join(f"{prefix}_pmc_{name}", "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            if "obca_solve_kernel" in r["Kernel_Name"]:
                vals[r["Counter_Name"]] += float(r["Counter_Value"])
    return vals


def launch_iterations(prefix, name):
    """IPM iterations of the profiled launch, from the bench JSON line the pass printed."""
    try:
        for line in open(f"{prefix}_pmc_{name}.log"):
            if line.startswith("{") and '"solver"' in line:
                b = json.loads(line)
                return b["solver"]["mean_iters"] * b["config"]["global_batch"] * b["steps"]
    except (OSError, ValueError, KeyError):
        pass
    return None


def main():
    prefix = sys.argv[1]
    act, vm, lds = counters(prefix, "active"), counters(prefix, "vmem"), counters(prefix, "lds")
    out = {"source": "rocprofv3 --pmc, three passes (tools/gpu_stall.sh); SQ cycle counters in quad-cycles"}
    wc = act.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        out["share_of_wave_cycles"] = {k[3:].lower(): act[k] / wc for k in sorted(act) if k != "SQ_WAVE_CYCLES"}
    it = launch_iterations(prefix, "vmem") or launch_iterations(prefix, "lds")
    out["launch_iterations"] = it
    out["vmem_latency_cycles"] = vm.get("VmemLatency")
    out["lds_latency_cycles"] = lds.get("LdsLatency")
    if it:
        per = {k: vm[k] / it for k in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_INSTS_SMEM") if k in vm}
        per.update({k: lds[k] / it for k in ("SQ_INSTS_VALU", "SQ_LDS_BANK_CONFLICT") if k in lds})
        per["wave_cycles"] = 4 * lds.get("SQ_WAVE_CYCLES", 0.0) / it
        out["per_problem_iteration"] = per
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
