#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_check.py > gpurun_out/abc.log 2>&1; echo "abc rc=$?"; cat gpurun_out/abc.log
