#!/bin/bash
# PC sampling of the OBCA solve (config D, 2048 problems, one timed step): where the wave's cycles go.
# Instances are generated (fork pool) by an unprofiled process first; the profiled one loads the cache.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03i}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 60 rocprofv3 -L > gpurun_out/${T}_pcs_avail.txt 2>&1
echo "list rc=$?"; grep -i -A3 "pc_sampling\|PC Sampling" gpurun_out/${T}_pcs_avail.txt | head -20
timeout -k 10 300 python -u bench.py --gen-only --cache /tmp/htp_pcs --batch 2048 > gpurun_out/${T}_pcs_gen.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 50 --output-format csv -d gpurun_out/${T}_pcs -o pcs -- \
  python3 bench.py --cache /tmp/htp_pcs --batch 2048 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${T}_pcs_run.txt 2>&1
echo "pcs rc=$?"; tail -3 gpurun_out/${T}_pcs_run.txt | cut -c1-300
ls -laR gpurun_out/${T}_pcs | head -20
