#!/bin/bash
# round-3: 2-rank rehearsal of the multi-rank bench path (gloo for the counters: RCCL refuses two ranks on one GPU)
# and a 20-step headline bench (the tail amortised)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r03q}
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
HTP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --batch 4096 --steps 2 --waves 512 --gen-procs 8 \
  > gpurun_out/${T}_ws2.out 2> gpurun_out/${T}_ws2.err || exit $?
grep '^{' gpurun_out/${T}_ws2.out | tail -1 | cut -c1-300
timeout -k 10 500 python -u bench.py --steps 20 --no-cpu-baseline > gpurun_out/${T}_bench20.out 2> gpurun_out/${T}_bench20.err || exit $?
tail -1 gpurun_out/${T}_bench20.out | cut -c1-300
