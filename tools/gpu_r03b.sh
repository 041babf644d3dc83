#!/bin/bash
# round-3 GPU step: relaxed-Riccati parity tests, point formulation on the persistent launch, C/E/points benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03b}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_obca.py tests/test_gpu_points.py -x -v --timeout 150 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_points.py > gpurun_out/${T}_points.json 2> gpurun_out/${T}_points.err || exit 1
timeout -k 10 300 python -u bench.py --config C --steps 2 --no-cpu-baseline > gpurun_out/${T}_benchC.json 2> gpurun_out/${T}_benchC.err || exit 1
timeout -k 10 400 python -u bench.py --config E --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${T}_benchE.json 2> gpurun_out/${T}_benchE.err || exit 1
if [ -n "$AB" ]; then
  timeout -k 10 400 python -u tools/ab_phase.py D 4096 $AB > gpurun_out/${T}_ab.txt 2>&1 || exit 1
fi
