#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box):
#  1) kernel trace + stats, 2) FETCH_SIZE pass, 3) WRITE_SIZE pass (separate PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; exit 1; }
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_kt.log 2>&1; echo "kt rc=$?"
tail -2 gpurun_out/prof_kt.log
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_fetch.log 2>&1; echo "fetch rc=$?"
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gen-procs 1 > gpurun_out/prof_write.log 2>&1; echo "write rc=$?"
find gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write -name "*.csv" | head -20
