set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
CACHE=/tmp/htp_instcache
timeout -k 10 400 python3 -u bench.py --steps 20 --cache $CACHE > gpurun_out/r06al_benchD20.json 2> gpurun_out/r06al_benchD20.log &&
timeout -k 10 300 python3 -u bench.py --cache $CACHE > gpurun_out/r06al_bench_D.json 2> gpurun_out/r06al_bench_D.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06al_kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --cache $CACHE > gpurun_out/r06al_kt_bench.json 2> gpurun_out/r06al_kt.log &&
timeout -k 10 300 python3 -u bench.py --config C --cache $CACHE > gpurun_out/r06al_benchC.json 2> gpurun_out/r06al_benchC.log
