#!/bin/bash
# GPU evidence runs (through gpurun, from the repo root; libraries prebuilt in-tree).
#   tools/gpu_evidence.sh TAG STEP...      STEP in:
#     tests    pytest -m gpu + smoke()
#     bench    default bench line (config D 32768, 6 steps, CPU baseline)
#     kt       rocprofv3 --kernel-trace --stats of the default bench command
#     pmc      FETCH / WRITE / SQ passes for configs D and C (then: python tools/pmc_summary.py gpurun_out TAG{D,C} {D,C} r02)
#     configs  bench lines of configs A, B, C, E and the batch sweep 1024 / 4096
#     kernels  hybrid A* and point-formulation throughput
#     ws2      2-rank rehearsal of the multi-GPU bench on one GPU (gloo: RCCL refuses two ranks on one device)
#     pytest:FILE[,FILE...]   only these GPU test files (tests/FILE)
#     pytestk:FILE[,...]      the same, every test (no -x, output shown) and the script goes on after test failures
#     benchC / benchE / benchD20   config C at 6 steps, config E, config D at 20 steps
#     ychain16k  notebook planner chain e2e at 16 384 scenes (cached draws), then its rocprofv3 kernel stats
#     pmcC / pmcE    PMC passes for configs C / E only
#     stall    the three SQ stall passes (tools/gpu_stall.sh) on config D
#     diag     I-cache / TLB / L2 / L1 passes (tools/gpu_diag.sh) on config D
#     ab:CFG:B:name,name...   A/B of libhtp_<name>.so variants (tools/build_variants.py; "base" = libhtp.so)
#     slow:CFG:MAXIT:PID,..:name,..  tools/slow_probe.py (per-problem kernel time / factorizations under variants)
#     fx:NAME,..:variant,..   tools/fixture_probe.py (oracle fixtures under A/B variants)
#     counters  rocprofv3 --list-avail (the PMC counter names of this box)
#     tail      tools/tail_probe.py on config D 32768 (per-problem cycles -> TAG_tail_D.npz for scale_projection.py)
#     tailE     the same on config E 4096 (which solves reach the 20 s limit, at what cost per iteration)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=$1; shift
( while true; do date >> gpurun_out/heartbeat.log; sleep 20; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > gpurun_out/${T}_$name.out 2> gpurun_out/${T}_$name.err
  local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids gpurun_out/${T}_$name.out | tail -3 | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
for S in "$@"; do
  case $S in
    tests) run gputest 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
           run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python -u bench.py ;;
    kt) run ktgen 300 python -u bench.py --gen-only --cache /tmp/htp_instcache
        run kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline --cache /tmp/htp_instcache ;;
    pmc) bash tools/gpu_pmc.sh ${T}D --batch 4096 || exit 1
         bash tools/gpu_pmc.sh ${T}C --config C --batch 4096 || exit 1 ;;
    configs) run benchA 200 python -u bench.py --config A --steps 2 --no-cpu-baseline
             run benchB 200 python -u bench.py --config B --steps 2 --no-cpu-baseline
             run benchC 300 python -u bench.py --config C --steps 2 --no-cpu-baseline
             run benchE 500 python -u bench.py --config E --steps 1 --warmup 0 --no-cpu-baseline
             run b1024 200 python -u bench.py --batch 1024 --no-cpu-baseline
             run b4096 200 python -u bench.py --batch 4096 --no-cpu-baseline ;;
    kernels) run hastar 300 python -u tools/bench_hastar.py
             run points 300 python -u tools/bench_points.py ;;
    ws2) HTP_DIST_BACKEND=gloo run ws2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
           --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --batch 4096 --steps 2 --waves 512 --gen-procs 8 ;;
    pytestk:*) files=$(echo "${S#pytestk:}" | tr ',' ' ' | sed 's|\([^ ]*\)|tests/\1|g')
               timeout -k 10 900 python -u -m pytest $files -m gpu -v -s --timeout 600 --timeout-method thread \
                 > gpurun_out/${T}_pytestk.out 2> gpurun_out/${T}_pytestk.err
               rc=$?; echo "pytestk rc=$rc"; grep -E "PASS|FAIL|ERROR|SKIP|model\]" gpurun_out/${T}_pytestk.out | cut -c1-300
               [ $rc -le 1 ] || exit $rc ;;   # test failures (1) go on; a crash, abort or time limit stops
    pytest:*) files=$(echo "${S#pytest:}" | tr ',' ' ' | sed 's|\([^ ]*\)|tests/\1|g')
              run pytest_sel 900 python -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread ;;
    benchAB) run benchA 200 python -u bench.py --config A --steps 2 --no-cpu-baseline
             run benchB 200 python -u bench.py --config B --steps 6 --no-cpu-baseline ;;
    e2eC) run e2eC 600 python -u bench.py --e2e --config C --steps 3 --warmup 1 ;;
    ychain) run ychain 600 python -u bench.py --e2e --planner ypark_hastar --steps 3 --warmup 1 ;;
    ychain16k) run ychaingen 300 python -u bench.py --e2e --planner ypark_hastar --batch 16384 --gen-only --cache /tmp/htp_ycache
           run ychain16k 600 python -u bench.py --e2e --planner ypark_hastar --batch 16384 --steps 2 --warmup 1 --cache /tmp/htp_ycache
           run ychainkt 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_ychainkt -o ykt -- \
               python3 -u bench.py --e2e --planner ypark_hastar --batch 16384 --steps 1 --warmup 0 --cache /tmp/htp_ycache ;;
    benchC) run benchC 600 python -u bench.py --config C --steps 6 --no-cpu-baseline ;;
    benchE) run benchE 900 python -u bench.py --config E --steps 2 --warmup 0 --no-cpu-baseline ;;
    benchE512) run benchE512 900 python -u bench.py --config E --steps 1 --warmup 0 --no-cpu-baseline --waves 512 ;;
    benchD20) run benchD20 900 python -u bench.py --steps 20 --no-cpu-baseline ;;
    pmcC) bash tools/gpu_pmc.sh ${T}C --config C --batch 4096 || exit 1 ;;
    pmcE) bash tools/gpu_pmc.sh ${T}E --config E --batch 1024 || exit 1 ;;
    stall) bash tools/gpu_stall.sh ${T}D || exit 1 ;;
    diag) bash tools/gpu_diag.sh ${T}D || exit 1 ;;
    ab:*) IFS=: read -r _ cfg nb names <<< "$S"
          run ab_$cfg 900 python -u tools/ab_phase.py $cfg $nb $(echo $names | tr ',' ' ') ;;
    slow:*) IFS=: read -r _ cfg mi pids names <<< "$S"
            run slow_$cfg 600 python -u tools/slow_probe.py $cfg $mi $pids $names ;;
    fx:*) IFS=: read -r _ names vars <<< "$S"
          run fx 900 python -u tools/fixture_probe.py $names $vars ;;
    counters) run counters 120 rocprofv3 --list-avail ;;
    hakt) run hakt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_hakt -o hakt -- python3 tools/bench_hastar.py --no-cpu
          run ypkt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_ypkt -o ypkt -- python3 tools/bench_ypark.py ;;
    hapmc) for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" \
                      "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_VALU_FMA_F64"; do
             n=$(echo $grp | cut -c1-12 | tr ' ' '_')
             run hapmc_$n 180 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${T}_hapmc_$n -o pmc -- python3 tools/bench_hastar.py --no-cpu --steps 1 --warmup 0
           done ;;
    tailE) run tailgenE 300 python -u bench.py --config E --batch 4096 --gen-only --cache /tmp/htp_instcache
           run tailE 600 python -u tools/tail_probe.py E 4096 /tmp/htp_instcache gpurun_out/${T}_tail_E.npz ;;
    tail) run tailgen 300 python -u bench.py --gen-only --cache /tmp/htp_instcache
          run tail 600 python -u tools/tail_probe.py D 32768 /tmp/htp_instcache gpurun_out/${T}_tail_D.npz ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
