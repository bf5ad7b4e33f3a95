#!/bin/bash
# World-size-2 rehearsal of bench.py's N>1 path (EV shards, all-reduces, sharded station leg)
# on ONE GPU: both ranks on cuda:0, gloo instead of RCCL (RCCL refuses two ranks on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --station-evs-per-gpu 65536 \
  > gpurun_out/dist2.log 2>&1
rc=$?; echo "dist2 rc=$rc"; exit $rc
