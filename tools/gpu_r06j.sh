set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python3 -u tools/bench_hastar.py --batch 2048 --unique 512 > gpurun_out/r06j_hastar_r05workload.json 2> gpurun_out/r06j_hastar_r05workload.log &&
timeout -k 10 300 python3 -u tools/bench_ypark.py > gpurun_out/r06j_ypark.json 2> gpurun_out/r06j_ypark.log &&
timeout -k 10 300 python3 -u tools/bench_points.py > gpurun_out/r06j_points.json 2> gpurun_out/r06j_points.log &&
timeout -k 10 600 python3 -u bench.py --e2e --planner ypark_hastar --batch 16384 --steps 2 --no-cpu-baseline > gpurun_out/r06j_ychain16k.json 2> gpurun_out/r06j_ychain16k.log
