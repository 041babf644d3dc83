#!/bin/bash
# Evidence for the current bench kernel: cycle breakdown, kernel-trace stats of bench.py,
# FETCH_SIZE / WRITE_SIZE in separate PMC passes.  A heartbeat keeps the call visibly alive.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python tools/gpu_quick.py D 4096 > gpurun_out/quickD.log 2>&1; rc=$?; echo "quick rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_kt.log 2>&1; rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_write.log 2>&1; rc=$?; echo "write rc=$rc"
exit $rc
