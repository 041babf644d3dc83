"""Summarise tools/gpu_diag.sh's PMC passes for the OBCA solve kernel: instruction-cache hit rate and fetch
latency, address-translation (UTCL1) miss rate, L2 hit rate and the share of L2 misses served by DRAM, vector-L1
requests and stalls, per problem-iteration where it applies.

Usage: python tools/diag_summary.py gpurun_out/r04dD [out.json]"""
import json
import sys

from stall_summary import counters, launch_iterations


def main():
    prefix = sys.argv[1]
    c = {}
    for name in ("ic1", "ic2", "tlb", "l2", "tcp"):
        c.update(counters(prefix, name))
    it = launch_iterations(prefix, "ic1") or launch_iterations(prefix, "l2")
    g = lambda k: c.get(k, 0.0)   # noqa: E731
    out = {"source": "rocprofv3 --pmc, five passes (tools/gpu_diag.sh), config D launch", "launch_iterations": it,
           "raw": dict(c)}
    if g("SQC_ICACHE_REQ"):
        out["icache_hit_rate"] = g("SQC_ICACHE_HITS") / g("SQC_ICACHE_REQ")
        out["icache_miss_rate"] = g("SQC_ICACHE_MISSES") / g("SQC_ICACHE_REQ")
    if g("SQ_IFETCH"):
        out["instr_fetch_latency_cycles"] = g("SQ_IFETCH_LEVEL") / g("SQ_IFETCH")
    if g("TCP_UTCL1_REQUEST_sum"):
        out["utcl1_miss_rate"] = g("TCP_UTCL1_TRANSLATION_MISS_sum") / g("TCP_UTCL1_REQUEST_sum")
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"):
        out["l2_hit_rate"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    if g("TCC_EA0_RDREQ_sum"):
        out["l2_miss_reads_to_dram_share"] = g("TCC_EA0_RDREQ_DRAM_sum") / g("TCC_EA0_RDREQ_sum")
    if g("TCP_TCC_READ_REQ_sum"):
        out["l1_to_l2_read_latency_cycles"] = g("TCP_TCC_READ_REQ_LATENCY_sum") / g("TCP_TCC_READ_REQ_sum")
    if it:
        out["per_problem_iteration"] = {k: v / it for k, v in c.items()}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
