#!/bin/bash
# l3r half-sample items: GPU tests, then the strong-scaling shard with and
# without the split (SRCNN_L3R_SPLIT_BELOW=0 turns it off), at 512 and 1024
# tiles, and the driver's headline command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/${1:-r05_split}
mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
  SRCNN_PARITY_LOG=$ROOT/$OUT/parity_checks.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -x \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
for b in 512 1024; do
  timeout -k 10 300 python tools/strong_shard.py --batch $b --modes ${MODES:-lazy,step} > "$OUT/split_$b.jsonl" 2> "$OUT/split_$b.err" || exit $?
  echo "split b=$b"; cat "$OUT/split_$b.jsonl"
  SRCNN_L3R_SPLIT_BELOW=0 timeout -k 10 300 python tools/strong_shard.py --batch $b --modes ${MODES:-lazy,step} > "$OUT/whole_$b.jsonl" 2> "$OUT/whole_$b.err" || exit $?
  echo "whole b=$b"; cat "$OUT/whole_$b.jsonl"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/d20.json" 2> "$OUT/d20.err" || exit $?
python3 -c "import json; d=json.load(open('$OUT/d20.json')); print('d20', d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
