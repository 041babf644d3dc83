#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ/MFMA) for config D and config C (4096 each) on the current solver.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02s}
bash tools/gpu_pmc.sh ${T}D --batch 4096 || exit 1
bash tools/gpu_pmc.sh ${T}C --config C --batch 4096 || exit 1
timeout -k 10 300 python -u bench.py --config C --steps 2 --no-cpu-baseline > gpurun_out/${T}_benchC.json 2> gpurun_out/${T}_benchC.err
rc=$?; echo "benchC rc=$rc"; cut -c1-300 gpurun_out/${T}_benchC.json; [ $rc -eq 0 ] || exit $rc
