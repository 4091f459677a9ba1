#!/bin/bash
# Same-box A/B of library builds on the training step only (no side legs):
#   tools/ab_train.sh <tag> <lib1.so> [lib2.so ...]   (paths relative to the repo)
# two interleaved reps of bench.py --steps 30 --warmup 5 per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab_train}; shift
mkdir -p "$OUT"
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    SRCNN_HIP_LIB=$PWD/$lib timeout -k 10 180 python bench.py --no-cpu-baseline --no-wide --no-forward --steps 30 --warmup 5 \
      > "$OUT/bench_${i}_$rep.json" 2> "$OUT/bench_${i}_$rep.err" || { tail -5 "$OUT/bench_${i}_$rep.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${i}_$rep.json')); print('variant $i rep $rep', round(d['value']), d['ms_per_step'], {k: round(v['ms_per_step'], 4) for k, v in d['kernels'].items()})"
  done
done
