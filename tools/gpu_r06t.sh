#!/bin/bash
# Round 6 (t): A/B of the load-before-store ordering of the constraint evaluation and the KKT scatter
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 fbh fbh2 > gpurun_out/r06t_ab_D.txt 2>&1
