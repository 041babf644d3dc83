#!/bin/bash
# persistent-queue launch: GPU tests, bench lines (4096 and default), 2-rank rehearsal on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r02i}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -3 gpurun_out/${T}_gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --batch 4096 --steps 2 --no-cpu-baseline > gpurun_out/${T}_b4096.json 2> gpurun_out/${T}_b4096.err
rc=$?; echo "b4096 rc=$rc"; cat gpurun_out/${T}_b4096.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_b4096.err; exit $rc; }
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.err; exit $rc; }
HTP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --batch 4096 --steps 2 --waves 512 --gen-procs 8 > gpurun_out/${T}_ws2.json 2> gpurun_out/${T}_ws2.err
rc=$?; echo "ws2 rc=$rc"; cat gpurun_out/${T}_ws2.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_ws2.err; exit $rc; }
