set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CACHE=/tmp/htp_instcache
timeout -k 10 300 python3 -u tools/neighbour_probe.py D24406 D25337 D27105 D24682 --k 26 > gpurun_out/r06h_neighbours.json 2> gpurun_out/r06h_neighbours.log &&
timeout -k 10 300 python3 bench.py --gen-only --cache $CACHE --batch 4096 > gpurun_out/r06h_gen.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/r06h_pmc_tlb -o tlb -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --cache $CACHE --batch 4096 > gpurun_out/r06h_pmc_tlb.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r06h_pmc_l2 -o l2 -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --cache $CACHE --batch 4096 > gpurun_out/r06h_pmc_l2.log 2>&1
