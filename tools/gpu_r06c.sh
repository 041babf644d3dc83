set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_phase.py D 4096 b44 ub l16 w2 > gpurun_out/r06c_ab_D.txt 2>&1 &&
timeout -k 10 300 python -u tools/neighbour_probe.py E12 D9730 D15734 D15863 D16412 D9252 --k 26 > gpurun_out/r06c_neighbours.json 2> gpurun_out/r06c_neighbours.log
