#!/bin/bash
# Config E bench line, hybrid A* (combined kernel) and point-formulation throughput; heartbeat keeps the run visible.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02w}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u tools/bench_hastar.py > gpurun_out/${T}_hastar.json 2> gpurun_out/${T}_hastar.err
rc=$?; echo "hastar rc=$rc"; cut -c1-300 gpurun_out/${T}_hastar.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_points.py > gpurun_out/${T}_points.json 2> gpurun_out/${T}_points.err
rc=$?; echo "points rc=$rc"; cut -c1-300 gpurun_out/${T}_points.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config E --steps 1 --no-cpu-baseline > gpurun_out/${T}_benchE.json 2> gpurun_out/${T}_benchE.err
rc=$?; echo "benchE rc=$rc"; cut -c1-300 gpurun_out/${T}_benchE.json; [ $rc -eq 0 ] || exit $rc
