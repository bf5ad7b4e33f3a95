#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Stops at the first step that faults / aborts / times out (rc not in {0,1}).
# usage: bash scripts/gpu_session.sh [steps...]   (default: smoke tests bench prof)
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
  return 0
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    quick) run pytest_quick 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    testsall) run pytest_gpu_all 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    bdist) run bdist 600 python bench.py --force-dist --no-cpu-baseline --no-direct ;;
    bdistq) run bdistq 300 python bench.py --force-dist --steps 100 --warmup 10 --no-cpu-baseline --no-direct --no-station ;;
    c5test) run c5test 600 python -u -m pytest tests/test_gpu_example.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k config5 ;;
    station) run station 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-direct --no-contracts ;;
    stationh) LOMPC_HOST_LOOP=1 run stationh 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-direct --no-contracts ;;
    stationd) run stationd 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-direct --no-contracts --force-dist ;;
    sprofk) run sprofk 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/sprofk -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-direct --no-contracts --station-steps 5 --station-warmup 1 --station-prof-steps 0 ;;
    comm) run comm 600 python -u -m pytest tests/test_gpu_comm.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench20) run bench20 300 python bench.py --steps 20 --warmup 5 ;;
    bench20q) run bench20q 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-station ;;
    bqtag) run "bq_${TAG}" 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --no-direct ;;
    bclose) LOMPC_CLOSE=1 run bclose 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --no-direct ;;
    qclose) LOMPC_CLOSE=1 run qclose 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sclose) LOMPC_CLOSE=1 run stamps_close 300 python scripts/kstamps.py ;;
    pipetest) run pipetest 600 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k run_steps ;;
    bench100q) run bench100q 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bsplit) run bsplit 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --split-types ;;
    bsplitset) run bsplitset 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --split-types --outputs set ;;
    bnoev) run bnoev 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --no-kernel-events ;;
    bev8) LOMPC_LIB=liblompc_amd_ev8.so run bev8 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bev4) LOMPC_LIB=liblompc_amd_ev4.so run bev4 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    qev8) LOMPC_LIB=liblompc_amd_ev8.so run qev8 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_baseline_configs.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    station5) run station5 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-direct --station-evs-per-gpu 2097152 --station-steps 5 --station-warmup 1 ;;
    qnew) run qnew 600 python -u -m pytest tests/test_gpu_example.py tests/test_gpu_station.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sprof) run sprof 300 python scripts/station_profile.py ;;
    bimpc) run bimpc 300 python scripts/bimpc_timing.py ;;
    stampsvar) for v in ${KS_VARIANTS}; do KS_VARIANT=$v run stamps_$v 300 python scripts/kstamps.py || exit $?; done ;;
    sproftrace) run sproftrace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/sproft -o run --output-format csv -- python scripts/station_profile.py ;;
    bcost) run bcost 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --outputs cost ;;
    bset) run bset 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --outputs set ;;
    bwarm) run bwarm 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --warm ;;
    bwarmset) run bwarmset 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station --warm --outputs set ;;
    stampsw) KS_WARM=1 run stampsw 300 python scripts/kstamps.py && KS_WARM=1 KS_OUTPUTS=set run stampsw_set 300 python scripts/kstamps.py ;;
    bg8) LOMPC_CELLS=8 run bg8 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg12) LOMPC_CELLS=12 run bg12 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg20) LOMPC_CELLS=20 run bg20 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg24) LOMPC_CELLS=24 run bg24 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg16) LOMPC_CELLS=16 run bg16 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg48) LOMPC_CELLS=48 run bg48 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg64) LOMPC_CELLS=64 run bg64 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg32) LOMPC_CELLS=32 run bg32 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg128) LOMPC_CELLS=128 run bg128 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    bg256) LOMPC_CELLS=256 run bg256 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-station ;;
    benchdirect) run bench_direct 600 python bench.py --mode direct --no-cpu-baseline ;;
    sweep) run sweep 600 python scripts/sweep_eval.py ;;
    host) run host 300 python scripts/host_overhead.py ;;
    stamps) run stamps 300 python scripts/kstamps.py && KS_OUTPUTS=set run stamps_set 300 python scripts/kstamps.py && run stamps48 300 python scripts/kstamps.py 48 ;;
    fail) run fail 600 python scripts/find_failures.py ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-station --no-direct ;;
    profsplit) run profsplit 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profsplit -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-station --split-types ;;
    *) echo "unknown step $s" ;;
  esac
done
