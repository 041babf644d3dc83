#!/bin/bash
# Round 6 (aa): A/B of the pivoted right-hand sides in LDS
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 pvl pvl2 > gpurun_out/r06ab_ab_D.txt 2>&1
