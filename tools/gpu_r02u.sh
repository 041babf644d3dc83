#!/bin/bash
# Full GPU suite + smoke + default bench (with CPU baseline) + kernel trace + PMC passes (D, C) + config C bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02u}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -2 gpurun_out/${T}_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; grep '^{' gpurun_out/${T}_kt.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh ${T}D --batch 4096 || exit 1
bash tools/gpu_pmc.sh ${T}C --config C --batch 4096 || exit 1
timeout -k 10 300 python -u bench.py --config C --steps 2 --no-cpu-baseline > gpurun_out/${T}_benchC.json 2> gpurun_out/${T}_benchC.err
rc=$?; echo "benchC rc=$rc"; cut -c1-200 gpurun_out/${T}_benchC.json; [ $rc -eq 0 ] || exit $rc
