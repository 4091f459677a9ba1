#!/bin/bash
# Same-box A/B of the 4K forward's Q layout: transposed (default) vs rows
# (SRCNN_FWD_Q=rows); bench.py's 4K line only, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ab_fwdq}; mkdir -p "$OUT"
for rep in 1 2; do
  for v in qt rows; do
    env_=""; [ $v = rows ] && env_="SRCNN_FWD_Q=rows"
    env $env_ timeout -k 10 200 python bench.py --no-cpu-baseline --no-wide --steps 5 --warmup 2 > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err" || exit $?
    python3 -c "
import json
d = json.load(open('$OUT/$v.$rep.json'))['forward']; print('$v', $rep, d['ms_per_frame'], d['kernels'])"
  done
done
