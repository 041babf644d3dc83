#!/bin/bash
# round-3 GPU step d: fixture parity (E failures), point-formulation phase profile, HA* bench, default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03d}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_obca.py -v --timeout 150 --timeout-method thread -k "fixtures" > gpurun_out/${T}_fixtures.txt 2>&1
echo "fixtures rc=$?"
timeout -k 10 300 python -u tools/points_probe.py 1024 > gpurun_out/${T}_points_probe.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_hastar.py > gpurun_out/${T}_hastar.json 2> gpurun_out/${T}_hastar.err || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
