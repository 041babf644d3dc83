#!/bin/bash
# Round 6 (an): A/B of the second-order-correction passes as sweeps
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 soc > gpurun_out/r06an_ab_D.txt 2>&1
