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
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    testsall) run pytest_gpu_all 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    benchdirect) run bench_direct 600 python bench.py --mode direct --no-cpu-baseline ;;
    sweep) run sweep 600 python scripts/sweep_eval.py ;;
    k1) run k1 300 python scripts/k1_stats.py ;;
    host) run host 300 python scripts/host_overhead.py ;;
    fail) run fail 600 python scripts/find_failures.py ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-station ;;
    *) echo "unknown step $s" ;;
  esac
done
