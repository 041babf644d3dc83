#!/bin/bash
# Point-formulation line and config E line, each under its own limit; heartbeat for the long generation.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u tools/bench_points.py > gpurun_out/benchP.json 2> gpurun_out/benchP.err
rc=$?; cat gpurun_out/benchP.json; tail -3 gpurun_out/benchP.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --config E --batch 4096 --steps 1 --warmup 1 --gen-procs 16 --cpu-budget 20 > gpurun_out/benchE.json 2> gpurun_out/benchE.err
rc=$?; cat gpurun_out/benchE.json; tail -3 gpurun_out/benchE.err; exit $rc
