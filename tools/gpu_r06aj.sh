#!/bin/bash
# Round 6 (aj): A/B of the local-sweep trip bound and lane read once
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 ht > gpurun_out/r06aj_ab_D.txt 2>&1
