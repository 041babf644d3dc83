#!/bin/bash
# Round 6 (ag): A/B of sweep width and Riccati ring depth on the final kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 sw16 r12 sw12 > gpurun_out/r06ag_ab_D.txt 2>&1
