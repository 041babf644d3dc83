#!/bin/bash
# Round 6 (aq): one vs two wavefronts per SIMD on the final kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/ab_phase.py D 4096 b44 w2n > gpurun_out/r06aq_ab_D.txt 2>&1
