#!/bin/bash
# rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) over the bench
# kernel, plus the HA* kernel trace.  A heartbeat file keeps the run visibly alive.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_write.log 2>&1; rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ha -o ha -- python3 tools/bench_hastar.py --batch 2048 --steps 2 --cpu-sample 8 > gpurun_out/prof_ha.log 2>&1; rc=$?; echo "ha rc=$rc"
exit $rc
