set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=25 -p no:cacheprovider > gpurun_out/r06n_gputest.txt 2>&1; echo "pytest rc=$?" >> gpurun_out/r06n_gputest.txt
grep -q "pytest rc=0\|pytest rc=1" gpurun_out/r06n_gputest.txt && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06n_smoke.txt 2>&1
