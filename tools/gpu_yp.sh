#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ypark.py tests/test_gpu_notebook.py tests/test_gpu_hastar.py -x -v --timeout 300 --timeout-method thread > gpurun_out/yp_pytest.log 2>&1
rc=$?; tail -8 gpurun_out/yp_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_ypark.py > gpurun_out/yp_bench.json 2> gpurun_out/yp_bench.err
rc=$?; cat gpurun_out/yp_bench.json; tail -3 gpurun_out/yp_bench.err; exit $rc
