#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/e_probe.py 512 4 60 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r02y_eprobe.log
