#!/bin/bash
# A/B bench of library variants: tools/ab_libs.sh <tag> <lib1.so> [lib2.so ...]
# Each variant first passes the fused train-step parity tests, then is benched
# twice (interleaved) to expose run-to-run noise.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab}; shift
mkdir -p "$OUT"
i=0
for lib in "$@"; do
  i=$((i+1))
  SRCNN_HIP_LIB=$PWD/$lib timeout -k 10 300 python -m pytest tests/test_parity_gpu.py -m gpu -q -x -p no:cacheprovider -k "train_step or full_batch" > "$OUT/pytest_$i.log" 2>&1
  rc=$?; echo "variant $i ($lib) pytest rc=$rc: $(tail -1 $OUT/pytest_$i.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    SRCNN_HIP_LIB=$PWD/$lib timeout -k 10 180 python bench.py --no-cpu-baseline > "$OUT/bench_${i}_$rep.json" 2>"$OUT/bench_${i}_$rep.err" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/bench_${i}_$rep.json')); print('variant $i rep $rep', round(d['value']), d['ms_per_step'], {k:round(v['ms_per_step'],4) for k,v in d['kernels'].items()}, 'wide', d.get('wide',{}).get('ms_per_step'), {k:round(v['ms_per_step'],4) for k,v in d.get('wide',{}).get('kernels',{}).items()})"
  done
done
