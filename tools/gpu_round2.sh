#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_obca.py -x -q -k small > gpurun_out/pytest_small.log 2>&1; echo "pytest small rc=$?"; tail -2 gpurun_out/pytest_small.log
timeout -k 10 400 python tools/gpu_quick.py D 4096 > gpurun_out/quickD.log 2>&1; echo "quickD rc=$?"; cat gpurun_out/quickD.log
