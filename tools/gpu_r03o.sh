#!/bin/bash
# round-3: GPU tests + smoke, default bench, tail probe, e2e per-stage kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03o}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.out 2>&1
rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/${T}_gputest.out
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.out 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.out
CACHE=/tmp/htp_instcache
timeout -k 10 300 python3 bench.py --gen-only --cache $CACHE > gpurun_out/${T}_genD.out 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --cache $CACHE > gpurun_out/${T}_bench.out 2> gpurun_out/${T}_bench.err || exit $?
tail -1 gpurun_out/${T}_bench.out | cut -c1-300
timeout -k 10 200 python3 -u tools/tail_probe.py D 32768 $CACHE > gpurun_out/${T}_tail.out 2> gpurun_out/${T}_tail.err || exit $?
head -12 gpurun_out/${T}_tail.out
timeout -k 10 300 python3 bench.py --gen-only --cache $CACHE --config C --batch 4096 > gpurun_out/${T}_genC.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_e2ekt -o kt -- python3 bench.py --e2e --config C --batch 4096 --steps 3 --warmup 1 --cache $CACHE > gpurun_out/${T}_e2ekt.out 2>&1 || exit $?
tail -1 gpurun_out/${T}_e2ekt.out | cut -c1-400
