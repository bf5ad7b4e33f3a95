#!/bin/bash
# Path-cell count sweep (LQ_G compile-time variants built in-tree by build.build(defines=("LQ_G=..",)))
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" g32 g128; do
  lib=${v:+liblompc_amd_$v.so}
  LOMPC_LIB=$lib timeout -k 10 300 python bench.py --no-station --no-cpu-baseline > gpurun_out/bench_cells_${v:-g64}.log 2>&1
  rc=$?; echo "${v:-g64} rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
