#!/bin/bash
# Round-5 session b: GPU tests; the l3r split at 512 / 1024 / 4096 tiles
# (SRCNN_L3R_SPLIT_BELOW moves the switch point); the 4K forward A/B against
# the previous commit's library (lib/variants/libsrcnn_hip_head.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/${1:-r05_b}
mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
  SRCNN_PARITY_LOG=$ROOT/$OUT/parity_checks.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
  [ -s "$OUT/parity_checks.jsonl" ] && python3 tools/parity_summary.py "$OUT/parity_checks.jsonl" > "$OUT/parity_summary.json"
fi
for b in 512 1024; do
  timeout -k 10 300 python tools/strong_shard.py --batch $b --modes lazy,step > "$OUT/split_$b.jsonl" 2> "$OUT/split_$b.err" || exit $?
  echo "split b=$b"; cat "$OUT/split_$b.jsonl"
  SRCNN_L3R_SPLIT_BELOW=0 timeout -k 10 300 python tools/strong_shard.py --batch $b --modes lazy,step > "$OUT/whole_$b.jsonl" 2> "$OUT/whole_$b.err" || exit $?
  echo "whole b=$b"; cat "$OUT/whole_$b.jsonl"
done
SRCNN_L3R_SPLIT_BELOW=100000 timeout -k 10 300 python tools/strong_shard.py --batch 4096 --steps 100 --warmup 20 --modes step > "$OUT/split_4096.jsonl" 2> "$OUT/split_4096.err" || exit $?
echo "split b=4096"; cat "$OUT/split_4096.jsonl"
timeout -k 10 300 python tools/strong_shard.py --batch 4096 --steps 100 --warmup 20 --modes step > "$OUT/whole_4096.jsonl" 2> "$OUT/whole_4096.err" || exit $?
echo "whole b=4096"; cat "$OUT/whole_4096.jsonl"
for rep in 1 2; do
  for v in head cur; do
    lib=cnn-super-resolution_amd/lib/variants/libsrcnn_hip_head.so
    [ $v = cur ] && lib=cnn-super-resolution_amd/lib/libsrcnn_hip.so
    SRCNN_HIP_LIB=$ROOT/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-wide --steps 20 --warmup 5 \
      > "$OUT/fwd_${v}_$rep.json" 2> "$OUT/fwd_${v}_$rep.err" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/fwd_${v}_$rep.json')); f=d['forward']; print('$v', $rep, 'frame', f['ms_per_frame'], {k: v['ms_per_frame'] for k, v in f['kernels'].items()}, 'step', d['ms_per_step'])"
  done
done
