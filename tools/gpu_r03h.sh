#!/bin/bash
# round-3 GPU step: all GPU tests, smoke, default bench (reference-producer scenes), the same bench on round 2's
# rectangle scenes, a compiler-flag A/B and the end-to-end device chain bench.  Test failures do not stop the run
# (a fault / timeout does).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03h}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.out 2>&1
rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/${T}_gputest.out
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.out 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.out
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.out 2> gpurun_out/${T}_bench.err || exit $?
tail -1 gpurun_out/${T}_bench.out | cut -c1-300
timeout -k 10 300 python -u bench.py --scene rects --no-cpu-baseline > gpurun_out/${T}_bench_rects.out 2> gpurun_out/${T}_bench_rects.err || exit $?
tail -1 gpurun_out/${T}_bench_rects.out | cut -c1-300
timeout -k 10 400 python -u bench.py --e2e --config C --batch 4096 --steps 2 --warmup 1 > gpurun_out/${T}_e2eC.out 2> gpurun_out/${T}_e2eC.err || exit $?
tail -1 gpurun_out/${T}_e2eC.out | cut -c1-400
if [ -n "$AB" ]; then
  timeout -k 10 400 python -u tools/ab_phase.py D 4096 base $AB > gpurun_out/${T}_ab.txt 2>&1 || exit $?
fi
