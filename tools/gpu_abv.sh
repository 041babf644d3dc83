#!/bin/bash
# A/B timing of libhtp_<name>.so variants (names as arguments) on one config-D batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_variants.py 4096 base "$@" > gpurun_out/abv.log 2>&1; rc=$?; echo "abv rc=$rc"; cat gpurun_out/abv.log; exit $rc
