#!/bin/bash
# GPU check for the Reeds-Shepp kernels (+ OBCA small parity after the context refactor).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_rs.py tests/test_gpu_obca.py -x -q -m gpu -k "not full" > gpurun_out/rs_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/rs_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_rs.py --batch 65536 --steps 5 --cpu-budget 10 > gpurun_out/rs_bench.json 2> gpurun_out/rs_bench.err
rc=$?
cat gpurun_out/rs_bench.json
exit $rc
