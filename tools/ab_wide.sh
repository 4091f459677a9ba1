#!/bin/bash
# A/B of library variants on the wide net: tools/ab_wide.sh <tag> <lib1.so> [lib2.so ...]
# Each variant first passes the wide-net GPU parity tests, then the bench's
# wide line runs twice per variant (interleaved, short headline, no 4K line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abw}; shift
mkdir -p "$OUT"
i=0
for lib in "$@"; do
  i=$((i+1))
  SRCNN_HIP_LIB=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_wide_gpu.py -m gpu -q -x -p no:cacheprovider > "$OUT/pytest_$i.log" 2>&1
  rc=$?; echo "variant $i ($lib) pytest rc=$rc: $(tail -1 $OUT/pytest_$i.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    SRCNN_HIP_LIB=$PWD/$lib timeout -k 10 180 python bench.py --no-cpu-baseline --no-forward --steps 20 --warmup 5 > "$OUT/bench_${i}_$rep.json" 2>"$OUT/bench_${i}_$rep.err" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/bench_${i}_$rep.json')); print('variant $i rep $rep', 'wide', d.get('wide',{}).get('ms_per_step'), {k:round(v['ms_per_step'],4) for k,v in d.get('wide',{}).get('kernels',{}).items()})"
  done
done
