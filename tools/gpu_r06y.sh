#!/bin/bash
# Round 6 (y): A/B of the pivoted-block right-hand-side register variants on the new kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 selop selmask bkm > gpurun_out/r06y_ab_D.txt 2>&1
