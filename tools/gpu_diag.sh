#!/bin/bash
# Memory-system diagnosis of the solver kernel: rocprofv3 PMC passes (one small group per run, gfx950 slot limits)
# over the bench kernel -- instruction cache (SQC_ICACHE_*, SQ_IFETCH), address translation (TCP_UTCL1_*), L2
# (TCC_HIT / MISS, EA reads to DRAM) and the vector L1 (TCP requests, stalls).  Summary: tools/diag_summary.py.
# Usage: tools/gpu_diag.sh TAG [bench args...]   (default: config D, 4096 problems)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r04d}; shift
ARGS=${*:---batch 4096}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
CACHE=/tmp/htp_instcache
timeout -k 10 300 python3 bench.py --gen-only --cache $CACHE $ARGS > gpurun_out/${TAG}_gen.log 2>&1 || exit 1
pass() {  # name, counters
  timeout -s KILL 300 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/${TAG}_pmc_$1 -o $1 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --cache $CACHE $ARGS > gpurun_out/${TAG}_pmc_$1.log 2>&1
  rc=$?; echo "$1 rc=$rc"; return $rc
}
pass ic1 "SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAVES" || exit 1
pass ic2 "SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_INSTS_SALU" || exit 1
pass tlb "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum" || exit 1
pass l2 "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" || exit 1
pass tcp "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" || exit 1
