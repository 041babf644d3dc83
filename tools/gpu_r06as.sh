#!/bin/bash
# Round 6 (as): which round-6 change makes the two-waves build differ
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 w2off w2fb w2ho > gpurun_out/r06as_ab_D.txt 2>&1
