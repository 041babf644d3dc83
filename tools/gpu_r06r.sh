#!/bin/bash
# Round 6 (r): solve-pass fill / stage split in the solver (HTP_PROF_ON=2) and the factor fill batch size
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 fbkv fbh fbhsprof > gpurun_out/r06r_ab_D.txt 2>&1
