set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/neighbour_probe.py D9730 D15734 D3220 D17294 D8593 --k 26 > gpurun_out/r06b_neighbours_D.json 2> gpurun_out/r06b_neighbours_D.log &&
timeout -k 10 400 python -u tools/tail_probe.py D 32768 "" gpurun_out/r06b_tail_D.npz > gpurun_out/r06b_tail_D.json 2> gpurun_out/r06b_tail_D.log
