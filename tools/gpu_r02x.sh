#!/bin/bash
# Kernel-trace stats of the default bench command (6 steps) and the throughput-vs-batch sweep (1024 / 4096).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02x}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; grep '^{' gpurun_out/${T}_kt.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
for B in 1024 4096; do
  timeout -k 10 300 python -u bench.py --batch $B --no-cpu-baseline > gpurun_out/${T}_b$B.json 2> gpurun_out/${T}_b$B.err
  rc=$?; echo "b$B rc=$rc"; cut -c1-200 gpurun_out/${T}_b$B.json; [ $rc -eq 0 ] || exit $rc
done
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python -u bench.py --config E --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${T}_benchE.json 2> gpurun_out/${T}_benchE.err
rc=$?; echo "benchE rc=$rc"; cut -c1-300 gpurun_out/${T}_benchE.json; exit $rc
