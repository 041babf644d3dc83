#!/bin/bash
# Config E bench line with the reference's default per-problem time limit (20 s), and config C (mixed, mower).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02aa}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 500 python -u bench.py --config E --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${T}_benchE.json 2> gpurun_out/${T}_benchE.err
rc=$?; echo "benchE rc=$rc"; cut -c1-300 gpurun_out/${T}_benchE.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config C --steps 2 --no-cpu-baseline > gpurun_out/${T}_benchC.json 2> gpurun_out/${T}_benchC.err
rc=$?; echo "benchC rc=$rc"; cut -c1-300 gpurun_out/${T}_benchC.json; exit $rc
