#!/bin/bash
# k_solve variant sweep on the GPU box (diagnostics): bench.py's QP/s leg for every built
# lompc_amd/liblompc_amd_<W>_<P>.so, full outputs and reductions only, optional cell counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for so in incentive-design-mpc_amd/lompc_amd/liblompc_amd_[0-9]*_[0-9]*.so; do
  v=$(basename "$so" .so); v=${v#liblompc_amd_}
  for cells in ${CELLS:-default}; do
    for out in full set; do
      if [ "$cells" = default ]; then unset LOMPC_CELLS; else export LOMPC_CELLS=$cells; fi
      LOMPC_LIB=$(basename "$so") timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline \
        --no-station --outputs $out > "gpurun_out/bv_${v}_g${cells}_${out}.log" 2>&1
      rc=$?
      echo "variant $v cells $cells $out rc=$rc"
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
