set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/neighbour_probe.py D15863 D16412 D9252 D18559 D20233 D21025 D22403 --k 26 > gpurun_out/r06d_neighbours.json 2> gpurun_out/r06d_neighbours.log
