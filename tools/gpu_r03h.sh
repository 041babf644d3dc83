#!/bin/bash
# round-3 GPU step h: the reference-producer workload (tests, smoke, default bench) and a compiler-flag A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03h}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/gpu_evidence.sh $T tests bench || exit $?
timeout -k 10 400 python -u tools/ab_phase.py D 4096 base trk pav o2 > gpurun_out/${T}_ab.txt 2>&1 || exit $?
