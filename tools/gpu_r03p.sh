#!/bin/bash
# round-3: PMC traffic / MFMA passes for the current solver (configs D and E)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r03p}
bash tools/gpu_pmc.sh ${T}D --batch 4096 || exit $?
bash tools/gpu_pmc.sh ${T}E --config E --batch 1024 || exit $?
