#!/bin/bash
# Cycle breakdown + rocprofv3 evidence for bench.py's dominant kernel and the HA* kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_quick.py D 4096 > gpurun_out/quickD.log 2>&1 || { echo QUICK FAIL; tail gpurun_out/quickD.log; exit 1; }
cat gpurun_out/quickD.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --gen-procs 8 > gpurun_out/prof_kt.log 2>&1; echo "kt rc=$?"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gen-procs 8 > gpurun_out/prof_fetch.log 2>&1; echo "fetch rc=$?"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gen-procs 8 > gpurun_out/prof_write.log 2>&1; echo "write rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ha -o ha -- python3 tools/bench_hastar.py --batch 2048 --steps 2 --cpu-sample 8 > gpurun_out/prof_ha.log 2>&1; echo "ha rc=$?"
find gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/prof_ha -name "*.csv" | head -30
