#!/bin/bash
# round-3: tail share of the persistent launch (config D 32768) and per-stage kernel times of the e2e chain
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03n}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
CACHE=/tmp/htp_instcache
timeout -k 10 300 python3 bench.py --gen-only --cache $CACHE > gpurun_out/${T}_genD.out 2>&1 || exit $?
timeout -k 10 300 python3 -u tools/tail_probe.py D 32768 $CACHE > gpurun_out/${T}_tail.out 2> gpurun_out/${T}_tail.err || exit $?
tail -12 gpurun_out/${T}_tail.out
timeout -k 10 300 python3 bench.py --gen-only --cache $CACHE --config C --batch 4096 > gpurun_out/${T}_genC.out 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_e2ekt -o kt -- python3 bench.py --e2e --config C --batch 4096 --steps 3 --warmup 1 --cache $CACHE > gpurun_out/${T}_e2ekt.out 2>&1 || exit $?
tail -1 gpurun_out/${T}_e2ekt.out | cut -c1-400
