#!/bin/bash
# Same-box A/B of the l3 kernels: unit-stream l3s (SRCNN_L3=stream) vs the
# whole-tile l3_delta (SRCNN_L3=tile), headline bench and the 512-tile shard.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab_l3}; mkdir -p "$OUT"
for rep in 1 2; do
  for v in stream tile; do
    env_="SRCNN_L3=$v"
    env $env_ timeout -k 10 200 python bench.py --no-cpu-baseline --no-wide --no-forward > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || exit $?
    env $env_ timeout -k 10 200 python bench.py --batch 512 --no-cpu-baseline --no-wide --no-forward --steps 200 --warmup 50 > "$OUT/$v.b512.$rep.json" 2> "$OUT/$v.b512.$rep.err" || exit $?
    python3 -c "
import json
for f in ['$OUT/$v.$rep.json', '$OUT/$v.b512.$rep.json']:
    d = json.load(open(f)); print(f, d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
  done
done
