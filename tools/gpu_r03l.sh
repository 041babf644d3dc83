#!/bin/bash
# round-3 final evidence: GPU tests, smoke, default bench, rectangle-scene bench, e2e bench, kernel trace of the
# default bench command, PMC passes (D 4096, E 1024).  Test failures do not stop the run (a fault / timeout does).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03l}
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
timeout -k 10 400 python -u bench.py --e2e --config C --batch 4096 --steps 3 --warmup 1 > gpurun_out/${T}_e2eC.out 2> gpurun_out/${T}_e2eC.err || exit $?
tail -1 gpurun_out/${T}_e2eC.out | cut -c1-400
timeout -k 10 300 python -u bench.py --gen-only --cache /tmp/htp_instcache > gpurun_out/${T}_ktgen.out 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline --cache /tmp/htp_instcache > gpurun_out/${T}_kt.out 2>&1 || exit $?
tail -1 gpurun_out/${T}_kt.out | cut -c1-200
bash tools/gpu_pmc.sh ${T}D --batch 4096 || exit $?
bash tools/gpu_pmc.sh ${T}E --config E --batch 1024 || exit $?
