set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/neighbour_probe.py E12 E4 E54 D347 D946 --k 32 > gpurun_out/r06a_neighbours.json 2> gpurun_out/r06a_neighbours.log &&
timeout -k 10 300 python -u bench.py --batch 4096 --steps 6 --no-cpu-baseline > gpurun_out/r06a_slice4096_s6.json 2> gpurun_out/r06a_slice4096_s6.log &&
timeout -k 10 300 python -u bench.py --batch 4096 --steps 20 --no-cpu-baseline > gpurun_out/r06a_slice4096_s20.json 2> gpurun_out/r06a_slice4096_s20.log &&
timeout -k 10 300 python -u tools/bench_hastar.py --batch 16384 --unique 4096 --cpu-sample 1024 > gpurun_out/r06a_hastar16k.json 2> gpurun_out/r06a_hastar16k.log
