#!/bin/bash
# round-3 final evidence: GPU tests + smoke, default bench, kernel trace of the same bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03s}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.out 2>&1
rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/${T}_gputest.out
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.out 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.out
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.out 2> gpurun_out/${T}_bench.err || exit $?
tail -1 gpurun_out/${T}_bench.out | cut -c1-300
timeout -k 10 300 python -u bench.py --gen-only --cache /tmp/htp_instcache > gpurun_out/${T}_ktgen.out 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline --cache /tmp/htp_instcache > gpurun_out/${T}_kt.out 2>&1 || exit $?
tail -1 gpurun_out/${T}_kt.out | cut -c1-200
