#!/bin/bash
# A/B of library variants on the default training step at batch 4096 and at
# the 512-tile strong-scaling shard:
#   tools/ab_step.sh <tag> <lib1.so> [lib2.so ...]
# Each variant first passes the fused train-step parity tests; then two
# interleaved reps of bench.py (4096 and 512 tiles, no side lines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab}; shift
mkdir -p "$OUT"
i=0
for lib in "$@"; do
  i=$((i+1))
  SRCNN_HIP_LIB=$PWD/$lib SRCNN_PARITY_LOG=$OUT/parity_$i.jsonl timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "train_step or full_batch or sq_err" > "$OUT/pytest_$i.log" 2>&1
  rc=$?; echo "variant $i ($lib) pytest rc=$rc: $(tail -1 $OUT/pytest_$i.log)"
  [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for b in 4096 512; do
    i=0
    for lib in "$@"; do
      i=$((i+1))
      f=$OUT/bench_${i}_b${b}_$rep
      SRCNN_HIP_LIB=$PWD/$lib timeout -k 10 180 python bench.py --batch $b --no-cpu-baseline --no-wide --no-forward \
        --steps $((b == 512 ? 300 : 100)) --warmup 30 > $f.json 2> $f.err || exit $?
      python3 -c "import json; d=json.load(open('$f.json')); print('variant $i b$b rep $rep', round(d['value']), d['ms_per_step'], {k:round(v['ms_per_step'],4) for k,v in d['kernels'].items()})"
    done
  done
done
