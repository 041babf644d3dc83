#!/bin/bash
# Round 6 (z): the new solver binary on config E (2 steps, the reference's 20 s max_cpu_time) and on the per-GPU
# slice of the 8-GPU share (config D 4096, 20 and 6 steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python3 -u bench.py --batch 4096 --steps 20 --no-cpu-baseline > gpurun_out/r06z_slice4096_s20.json 2> gpurun_out/r06z_slice4096_s20.log &&
timeout -k 10 300 python3 -u bench.py --batch 4096 --steps 6 --no-cpu-baseline > gpurun_out/r06z_slice4096_s6.json 2> gpurun_out/r06z_slice4096_s6.log &&
timeout -k 10 900 python3 -u bench.py --config E --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/r06z_benchE.json 2> gpurun_out/r06z_benchE.log
