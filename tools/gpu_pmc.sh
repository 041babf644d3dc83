#!/bin/bash
# rocprofv3 PMC passes over the bench kernel, one counter group per run (gfx950 slot
# limits): FETCH_SIZE, WRITE_SIZE, and an SQ pass with the FP64 MFMA / VALU counts.
# Usage: tools/gpu_pmc.sh TAG [bench args...]   (default: config D, 4096 problems)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r02}; shift
ARGS=${*:---batch 4096}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
# instances: generated once with the normal parallel (fork-pool) generator, OUTSIDE the profiler
# (rocprofv3's preloaded library brings the GPU up before bench.py starts, so the profiled
# process must not fork); the profiled runs load them from the cache
CACHE=/tmp/htp_instcache
timeout -k 10 300 python3 bench.py --gen-only --cache $CACHE $ARGS > gpurun_out/${TAG}_gen.log 2>&1 || exit 1
pass() {  # name, counters
  timeout -s KILL 300 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/${TAG}_pmc_$1 -o $1 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --cache $CACHE $ARGS > gpurun_out/${TAG}_pmc_$1.log 2>&1
  rc=$?; echo "$1 rc=$rc"; return $rc
}
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
pass sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" || exit 1
