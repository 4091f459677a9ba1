#!/bin/bash
# Bench-only A/B of library variants (no parity; for diagnostic builds whose
# results are invalid): tools/ab_bench.sh <tag> <lib1.so> [lib2.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abb}; shift
mkdir -p "$OUT"
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    f=$OUT/bench_${i}_$rep
    SRCNN_HIP_LIB=$PWD/$lib timeout -k 10 180 python bench.py --no-cpu-baseline --no-wide --no-forward > $f.json 2> $f.err || exit $?
    python3 -c "import json; d=json.load(open('$f.json')); print('variant $i ($lib) rep $rep', round(d['value']), d['ms_per_step'], {k:round(v['ms_per_step'],4) for k,v in d['kernels'].items()})"
  done
done
