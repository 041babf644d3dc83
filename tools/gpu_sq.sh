#!/bin/bash
# SQ instruction-mix counters over the bench kernel (one PMC pass, small batch).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/prof_sq -o sq -- python3 bench.py --steps 1 --warmup 0 --batch 1024 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_sq.log 2>&1; rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof_sq2 -o sq2 -- python3 bench.py --steps 1 --warmup 0 --batch 1024 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_sq2.log 2>&1; rc=$?; echo "sq2 rc=$rc"
grep -h obca gpurun_out/prof_sq/sq_counter_collection.csv gpurun_out/prof_sq2/sq2_counter_collection.csv | awk -F'","' '{print $(NF-3), $(NF-2)}'
exit $rc
