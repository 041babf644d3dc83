#!/bin/bash
# Where the solver wave's cycles go: rocprofv3 PMC passes (one group per run, gfx950 slot limits) over the
# bench kernel -- issue-active vs waiting (SQ_ACTIVE_INST_* / SQ_WAIT_*), average VMEM and LDS latency
# (VmemLatency / LdsLatency = accumulated in-flight level / instructions), instruction mix, LDS bank conflicts.
# Usage: tools/gpu_stall.sh TAG [bench args...]   (default: config D, 4096 problems); summary: tools/stall_summary.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r03s}; shift
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
pass active "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" || exit 1
pass vmem "VmemLatency SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM" || exit 1
pass lds "LdsLatency SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES" || exit 1
