#!/bin/bash
# Round 6 (p): where a Riccati stage's cycles go.  The stage chain in isolation (tools/micro/ric_micro, 1024 and
# 1 resident wavefronts) against its in-solver cost, and the instruction-cache counters of the solver kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CACHE=/tmp/htp_instcache
( cd tools/micro && timeout -k 5 60 ./ric_micro 1024 20 && timeout -k 5 60 ./ric_micro 1 20 &&
  timeout -k 5 60 ./ric_micro_prof 1024 20 && timeout -k 5 60 ./ric_micro_prof 1 20 ) > gpurun_out/r06p_ric_micro.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/r06p_avail.txt 2>&1
grep -i "icache\|ifetch\|SQC_" gpurun_out/r06p_avail.txt > gpurun_out/r06p_avail_sqc.txt
timeout -k 10 300 python3 bench.py --gen-only --cache $CACHE --batch 4096 > gpurun_out/r06p_gen.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r06p_pmc_ic -o ic -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --cache $CACHE --batch 4096 > gpurun_out/r06p_pmc_ic.log 2>&1
echo "ic rc=$?"
