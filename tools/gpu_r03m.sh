#!/bin/bash
# round-3: per-config bench lines on the reference-producer scenes (A, B, C, E), point formulation, hybrid A*
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03m}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_$name.out 2> gpurun_out/${T}_$name.err
  local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/${T}_$name.out | tail -1 | cut -c1-250
  [ $rc -eq 0 ] || exit $rc
}
run benchA 200 python -u bench.py --config A --steps 2 --no-cpu-baseline
run benchB 200 python -u bench.py --config B --steps 2 --no-cpu-baseline
run benchC 300 python -u bench.py --config C --steps 2 --no-cpu-baseline
run benchE 500 python -u bench.py --config E --steps 1 --warmup 0 --no-cpu-baseline
run points 300 python -u tools/bench_points.py
run hastar 300 python -u tools/bench_hastar.py
