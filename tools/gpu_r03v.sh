#!/bin/bash
# round-3 final evidence for the solver with 8-deep sweeps: tests + smoke, bench, kernel trace, PMC (D, E)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r03v}
bash tools/gpu_r03s.sh $T || exit $?
bash tools/gpu_pmc.sh ${T}D --batch 4096 || exit $?
bash tools/gpu_pmc.sh ${T}E --config E --batch 1024 || exit $?
