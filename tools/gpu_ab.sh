#!/bin/bash
# A/B of OBCA library variants (tools/build_variants.py) on the GPU: tools/gpu_ab.sh TAG CFG B name...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=$1; shift
timeout -k 10 600 python -u tools/ab_phase.py "$@" > gpurun_out/${T}_ab.log 2>&1
rc=$?; cat gpurun_out/${T}_ab.log | grep -v amdgpu.ids; exit $rc
