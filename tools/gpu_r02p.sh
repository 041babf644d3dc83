#!/bin/bash
# Local factor-sweep sub-phases, OBCA GPU parity tests on the rebuilt library, bench at 3 and 8 steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02p}
timeout -k 10 300 python -u tools/ab_phase.py D 4096 base ring2lprof > gpurun_out/${T}_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${T}_ab.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_obca.py tests/test_gpu_points.py tests/test_gpu_notebook.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/${T}_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench3.json 2> gpurun_out/${T}_bench3.err
rc=$?; echo "bench3 rc=$rc"; cut -c1-400 gpurun_out/${T}_bench3.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 8 --no-cpu-baseline > gpurun_out/${T}_bench8.json 2> gpurun_out/${T}_bench8.err
rc=$?; echo "bench8 rc=$rc"; cut -c1-400 gpurun_out/${T}_bench8.json; [ $rc -eq 0 ] || exit $rc
