#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd headland_trajectory_planning_amd/csrc
timeout -k 10 300 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DHTP_TRACE_ON -include cstdio -o ../libhtp_dbg.so htp_obca.hip > ../../gpurun_out/dbgbuild.log 2>&1 || { echo BUILD FAIL; tail ../../gpurun_out/dbgbuild.log; exit 1; }
cd ../..
timeout -k 10 120 python - > gpurun_out/dbg_run.log 2>&1 <<'PY'
import sys; sys.path.insert(0, '.')
from headland_trajectory_planning_amd import _native, synth
lib = _native.load(_native.LIB_PATH.replace('libhtp.so', 'libhtp_dbg.so'))
ctx = _native.Context(0, lib=lib, options={'max_iter': 3})
insts = [synth.make_instance(0, N=12, M=2, implement='mower')]
try:
    r = ctx.solve(_native.PackedBatch(insts))
    print('status', r.status, r.iterations, r.objective)
except Exception as e:
    print('EXC', e)
PY
echo "rc=$?"
head -60 gpurun_out/dbg_run.log
