#!/bin/bash
# Kernel-trace stats of the default bench line + PMC passes (FETCH, WRITE, SQ/MFMA) for config D
# (4096) and config C (4096, mixed turns, mower) on the committed solver.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02l}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; grep '^{' gpurun_out/${T}_kt.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh ${T}D --batch 4096 || exit 1
bash tools/gpu_pmc.sh ${T}C --config C --batch 4096 || exit 1
timeout -k 10 300 python -u bench.py --config C --steps 2 --no-cpu-baseline > gpurun_out/${T}_benchC.json 2> gpurun_out/${T}_benchC.err
rc=$?; echo "benchC rc=$rc"; cat gpurun_out/${T}_benchC.json; [ $rc -eq 0 ] || exit $rc
