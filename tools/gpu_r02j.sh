#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02j}
timeout -k 10 300 python -u tools/gpu_quick.py D 4096 > gpurun_out/${T}_quick.log 2>&1; rc=$?; echo "quick rc=$rc"; cat gpurun_out/${T}_quick.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_kt.log 2>&1; rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh ${T} --batch 4096
