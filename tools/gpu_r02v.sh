#!/bin/bash
# Default bench line (CPU baseline, PMC traffic/MFMA from profiles/) and configs B, E, A lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02v}
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || exit $rc
for C in B A E; do
  timeout -k 10 400 python -u bench.py --config $C --steps 2 --no-cpu-baseline > gpurun_out/${T}_bench$C.json 2> gpurun_out/${T}_bench$C.err
  rc=$?; echo "bench$C rc=$rc"; cut -c1-200 gpurun_out/${T}_bench$C.json; [ $rc -eq 0 ] || exit $rc
done
