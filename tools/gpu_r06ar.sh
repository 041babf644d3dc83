#!/bin/bash
# Round 6 (ar): which non-default knob breaks bit-identity
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 fs1 r4 pl0 > gpurun_out/r06ar_ab_D.txt 2>&1
