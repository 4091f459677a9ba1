#!/bin/bash
# Bench-only comparison of library variants (no parity tests: for diagnostic
# builds whose results are deliberately invalid).  tools/bench_variants.sh <tag> <lib>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-bv}; shift
mkdir -p "$OUT"
i=0
for lib in "$@"; do
  i=$((i+1))
  SRCNN_HIP_LIB=$PWD/$lib timeout -k 10 180 python bench.py --no-cpu-baseline ${BV_ARGS:-} > "$OUT/bench_$i.json" 2>"$OUT/bench_$i.err" || exit $?
  python3 -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('$(basename $lib)', round(d['value']), d['ms_per_step'], {k:round(v['ms_per_step'],4) for k,v in d['kernels'].items()}, 'fwd', d.get('forward',{}).get('ms_per_frame'), 'wide', d.get('wide',{}).get('ms_per_step'), {k:v['ms_per_step'] for k,v in d.get('wide',{}).get('kernels',{}).items()})"
done
