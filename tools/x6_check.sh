#!/bin/bash
# GPU check of the split-bf16 kernels: the GPU suite, then a short bench
# (split and fp32 arithmetic, same box).   tools/x6_check.sh <tag> [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-x6}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1
else
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
fi
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" "$OUT/pytest.log" | head -30; exit $rc; }
for a in split f32 split; do
  env_a=""; [ $a = f32 ] && env_a="SRCNN_ARITH=f32"
  env $env_a timeout -k 10 300 python bench.py --no-cpu-baseline --no-wide --no-forward --steps 20 --warmup 5 \
    > "$OUT/bench_$a.json" 2> "$OUT/bench_$a.err" || { cat "$OUT/bench_$a.err" | tail; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$a.json')); print('$a', d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
done
