#!/bin/bash
# Config B (256 turns) and config C (4096 turns, mower implement, K=2 bodies) bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u bench.py --config B --batch 256 --steps 3 --warmup 1 --cpu-budget 15 > gpurun_out/benchB.json 2> gpurun_out/benchB.err
rc=$?; cat gpurun_out/benchB.json; tail -3 gpurun_out/benchB.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config C --batch 4096 --steps 2 --warmup 1 --cpu-budget 15 > gpurun_out/benchC.json 2> gpurun_out/benchC.err
rc=$?; cat gpurun_out/benchC.json; tail -3 gpurun_out/benchC.err; exit $rc
