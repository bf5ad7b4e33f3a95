#!/bin/bash
# Bench compile-time variants of the library (built in-tree as lompc_amd/liblompc_amd_<tag>.so)
# usage: bash scripts/sweep_variants.sh tag1 tag2 ...   ("" = product library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=liblompc_amd_$v.so
  LOMPC_LIB=$lib timeout -k 10 300 python bench.py --no-station --no-cpu-baseline > gpurun_out/bench_var_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
