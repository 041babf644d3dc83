#!/bin/bash
# Round 6 (q): A/B of the wave-context and factor-fill variants on config D 4 096 (tools/ab_phase.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 sel reg regsel > gpurun_out/r06q_ab_D.txt 2>&1
