#!/bin/bash
# Round 6 (af): A/B of the per-sweep binding of build_local invariants
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 hl > gpurun_out/r06af_ab_D.txt 2>&1
