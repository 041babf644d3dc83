#!/bin/bash
# round-3 GPU step f: point formulation with the 5-column MFMA Sigma pass (probe, parity, bench)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03f}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u tools/points_probe.py 1024 > gpurun_out/${T}_points_probe.txt 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_obca.py -v --timeout 150 --timeout-method thread -k "points or fixtures" > gpurun_out/${T}_tests.txt 2>&1
rc=$?
echo "tests rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u tools/bench_points.py > gpurun_out/${T}_points.json 2> gpurun_out/${T}_points.err || exit 1
