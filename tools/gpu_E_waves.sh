#!/bin/bash
# Config E persistent-launch width A/B: the same 4 096 instances solved with 1 024 (one wavefront per SIMD, the
# default), 768 and 512 wavefronts.  Fewer resident wavefronts share each CU's memory pipeline with fewer
# neighbours, so every solve's iterations run faster; E's step is set by its longest solves (VERDICT r4 item 3:
# 44.5 of 4 096 per step stop at max_cpu_time 20 s under full load).
# Usage: tools/gpu_E_waves.sh TAG [steps] [wave counts...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r05y}; STEPS=${2:-2}; shift; shift
WAVES=${*:-1024 768 512}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
CACHE=/tmp/htp_instcache
timeout -k 10 300 python3 bench.py --config E --gen-only --cache $CACHE > gpurun_out/${TAG}_gen.log 2>&1 || exit 1
for w in $WAVES; do
  timeout -k 10 200 python3 -u bench.py --config E --steps $STEPS --warmup 1 --no-cpu-baseline --cache $CACHE \
    --waves $w > gpurun_out/${TAG}_E_w$w.json 2> gpurun_out/${TAG}_E_w$w.err
  rc=$?; echo "waves=$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
