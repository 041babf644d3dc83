#!/bin/bash
# Round GPU check (run through gpurun from the repo root; libraries prebuilt in-tree):
#   1) pytest -m gpu, 2) smoke(), 3) bench.py default line, 4) rocprofv3 kernel trace of the bench.
# Usage: tools/gpu_round.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02}
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
  rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/${TAG}_gputest.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_kt.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -1 gpurun_out/${TAG}_kt.log | cut -c1-400
find gpurun_out/${TAG}_kt -name "*stats*.csv" | head
