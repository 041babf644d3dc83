#!/bin/bash
# GPU check for the hybrid A* kernel: its tests, then the throughput tool.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hastar.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ha_pytest.log 2>&1
rc=$?; tail -12 gpurun_out/ha_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_hastar.py ${HA_ARGS} > gpurun_out/ha_bench.json 2> gpurun_out/ha_bench.err
rc=$?; cat gpurun_out/ha_bench.json; tail -3 gpurun_out/ha_bench.err; exit $rc
