#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/e_probe.py 16 8 20 > gpurun_out/r02z_eprobe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r02z_eprobe.log; exit $rc
