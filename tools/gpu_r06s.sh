#!/bin/bash
# Round 6 (s): A/B of the loop-invariant hoisting in the stage-chain loops on config D 4 096
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 fbkv fbh fbhsprof > gpurun_out/r06s_ab_D.txt 2>&1
