#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box (NOT a measurement):
# 2 ranks on device 0, gradients all-reduced over gloo (RCCL takes one rank
# per device).  Weak-scaling default line, then a strong-scaling one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rehearse}; mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1
for mode in weak strong; do
  extra=""; [ $mode = strong ] && extra="--global-batch 1024"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --comm torch --dist-backend gloo \
    --all-ranks-on-device 0 $extra > "$OUT/$mode.json" 2> "$OUT/$mode.err"
  rc=$?; echo "$mode rc=$rc"; tail -1 "$OUT/$mode.json"
  [ $rc -eq 0 ] || exit $rc
done
