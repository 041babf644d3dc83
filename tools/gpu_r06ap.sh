#!/bin/bash
# Round 6 (ap): config E line of the final binary with its PMC traffic and MFMA
# slice of the 8-GPU share (config D 4096, 20 and 6 steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python3 -u bench.py --config E --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/r06ap_benchE.json 2> gpurun_out/r06ap_benchE.log
