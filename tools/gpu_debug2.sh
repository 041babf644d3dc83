#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd headland_trajectory_planning_amd/csrc
timeout -k 10 300 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DHTP_TRACE_ON -include cstdio -o ../libhtp_dbg.so htp_obca.hip > ../../gpurun_out/dbgbuild.log 2>&1 || { echo BUILD FAIL; exit 1; }
cd ../..
for mode in plain1 dbg1 plain3; do
timeout -k 10 120 python - $mode > gpurun_out/dbg_$mode.log 2>&1 <<'PY'
import sys; sys.path.insert(0, '.')
from headland_trajectory_planning_amd import _native, synth
mode = sys.argv[1]
path = _native.LIB_PATH.replace('libhtp.so', 'libhtp_dbg.so') if mode.startswith('dbg') else _native.LIB_PATH
lib = _native.load(path)
ctx = _native.Context(0, lib=lib)
nb = 3 if mode.endswith('3') else 1
insts = [synth.make_instance(pid, N=12, M=2, implement='mower') for pid in range(nb)]
try:
    r = ctx.solve(_native.PackedBatch(insts))
    print('status', r.status, r.iterations, r.objective)
except Exception as e:
    print('EXC', e)
PY
echo "$mode rc=$?"; tail -4 gpurun_out/dbg_$mode.log
done
