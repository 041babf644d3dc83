set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for rep in 1 2; do
  for lib in hanew2 haold; do
    tag=${lib:-base}
    timeout -k 10 300 python3 -u tools/bench_hastar.py --batch 2048 --unique 512 --no-cpu ${lib:+--lib $lib} > gpurun_out/r06l_ha2k_${tag}_$rep.json 2>> gpurun_out/r06k.log || exit 1
    timeout -k 10 300 python3 -u tools/bench_hastar.py --batch 16384 --unique 4096 --no-cpu ${lib:+--lib $lib} > gpurun_out/r06l_ha16k_${tag}_$rep.json 2>> gpurun_out/r06k.log || exit 1
  done
done
