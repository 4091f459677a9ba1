#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box (NOT a measurement):
# 2 ranks on device 0, gradients all-reduced over gloo (RCCL takes one rank
# per device).  bench.py launches the ranks itself (no torch.distributed.run
# on the command line); the weak line carries the strong-scaling sub-record.
# A WORLD_SIZE that disagrees with --gpus must exit non-zero.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rehearse}; mkdir -p "$OUT"
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --comm torch --dist-backend gloo \
  --all-ranks-on-device 0 --no-wide > "$OUT/n2.json" 2> "$OUT/n2.err"
rc=$?; echo "n2 rc=$rc"; tail -1 "$OUT/n2.json"
[ $rc -eq 0 ] || exit $rc
WORLD_SIZE=3 timeout -k 10 60 python bench.py --gpus 2 --steps 1 > "$OUT/mismatch.json" 2> "$OUT/mismatch.err"
rc=$?; echo "mismatch rc=$rc (expected non-zero)"; tail -1 "$OUT/mismatch.err"
[ $rc -ne 0 ] || exit 1
exit 0
