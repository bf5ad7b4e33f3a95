#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only; never combined with sys/runtime traces)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 3 --no-cpu-baseline --no-station --no-direct --no-contracts"}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc/p$i -o run --output-format csv -- python bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc" | tee -a gpurun_out/pmc/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS
GROUPS
