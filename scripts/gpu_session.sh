#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Stops at the first step that faults / aborts / times out (rc not in {0,1}).
# usage: bash scripts/gpu_session.sh [steps...]   (default: smoke tests bench prof)
# (no LOMPC_* run-time knobs exist in the product library: variants are -D builds, scripts/build_variant.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${*:-smoke tests bench prof}
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  # a failed step whose log shows a GPU fault ends the session too (no second faulting run)
  if [ $rc -eq 1 ] && grep -q -e "illegal memory access" -e "hipErrorIllegalAddress" -e "Memory access fault" "gpurun_out/$name.log"; then
    echo "stopping after $name (GPU fault in its log)"; exit 1
  fi
  return 0
}
PYT="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 $PYT tests -m gpu ;;
    quick) run pytest_quick 600 $PYT tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -m gpu ;;
    pipetest) run pipetest 600 $PYT tests/test_gpu_pipeline.py -m gpu -k run_steps ;;
    comm) run comm 600 $PYT tests/test_gpu_comm.py -m gpu ;;
    c5test) run c5test 600 $PYT tests/test_gpu_example.py -m gpu -k config5 ;;
    loop) run loop 600 $PYT tests/test_gpu_price_solver.py tests/test_gpu_station.py -m gpu ;;
    qnew) run qnew 600 $PYT tests/test_gpu_example.py tests/test_gpu_station.py -m gpu ;;
    bench) run bench 600 python bench.py ;;
    bench20) run bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench20q) run bench20q 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-station ;;
    bench100q) run bench100q 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    # the N > 1 code path on one GPU: two rank processes started by bench.py itself (gloo: RCCL refuses
    # two ranks on one device), and the RCCL path as a world-size-1 group
    bdist2) run bdist2 600 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-cpu-baseline --no-direct --no-contracts --station-evs-per-gpu 65536 --station-steps 3 --station-warmup 1 --station-prof-steps 0 ;;
    bdist) run bdist 600 python bench.py --force-dist --no-cpu-baseline --no-direct ;;
    bdistq) run bdistq 300 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline --no-direct --no-station ;;
    station) run station 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-direct --no-contracts ;;
    sprofk) run sprofk 600 rocprofv3 --kernel-trace --stats -d gpurun_out/sprofk -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-direct --no-contracts --station-steps 5 --station-warmup 1 --station-prof-steps 0 ;;
    sprof) run sprof 300 python scripts/station_profile.py ;;
    bimpc) run bimpc 300 python scripts/bimpc_timing.py ;;
    benchdirect) run bench_direct 600 python bench.py --mode direct --no-cpu-baseline ;;
    stamps) run stamps 300 python scripts/kstamps.py ;;
    lstamps) run lstamps 300 python scripts/loop_stamps.py station ;;
    lstamps32) run lstamps32 300 python scripts/loop_stamps.py station --cells 32 ;;
    lstamps8) run lstamps8 300 python scripts/loop_stamps.py station --cells 8 ;;
    stampsrt) run stampsrt 300 env KS_RT=1 KS_VARIANT=rt python scripts/kstamps.py 24 ;;
    # the driver's exact command under the kernel trace: where the wall time per step goes
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-station --no-direct ;;
    r5new) run r5new 600 $PYT tests/test_gpu_chain.py tests/test_gpu_price_loop_c5.py tests/test_gpu_levels.py -m gpu ;;
    stationt) run stationt 600 $PYT tests/test_gpu_station.py tests/test_gpu_example.py -m gpu ;;
    benchq) run benchq 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-station --no-direct ;;
    # round 6
    syncmodes) P="python -u scripts/step_probe.py --cells 4 --steps 20 --reps 8 --warmup 5 --gpu-span"
               run sync_default 200 $P; run sync_spin 200 $P --spin
               run sync_active 200 env ROC_ACTIVE_WAIT_TIMEOUT=100000 $P ;;
    cells100) run cells100 300 python -u scripts/step_probe.py --cells 4 8 12 --steps 100 --reps 5 --warmup 10 ;;
    stationt6) run stationt6 600 $PYT tests/test_gpu_station.py tests/test_gpu_levels.py -m gpu ;;
    bdistst) run bdistst 600 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline --no-direct --no-contracts ;;
    bst) run bst 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-direct --no-contracts ;;
    bprofh) run bprofh 300 python scripts/bimpc_prof.py ;;
    pipetests) run pipetests 600 $PYT tests/test_gpu_pipeline.py tests/test_gpu_parity.py -m gpu ;;
    contracts) run contracts 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-station --no-direct ;;
    looptests) run looptests 600 $PYT tests/test_gpu_price_loop_c5.py tests/test_gpu_price_loop_long.py tests/test_gpu_price_solver.py tests/test_gpu_chain.py tests/test_gpu_comm.py tests/test_gpu_station.py -m gpu ;;
    *) echo "unknown step $s" ;;
  esac
done
