#!/bin/bash
# Round-4 GPU session: the standard session (tests, smoke, bench, rocprofv3),
# then the N = 2 launcher rehearsal and the 512-tile strong-scaling shard.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NAME=${1:-r04}
bash tools/gpu_session.sh "$NAME" || exit $?
bash tools/rehearse_n2.sh "$NAME/rehearse" || exit $?
OUT=gpurun_out/$NAME/strong; mkdir -p "$OUT"
timeout -k 10 200 python bench.py --batch 512 --no-cpu-baseline --no-wide --no-forward --steps 200 --warmup 50 \
  > "$OUT/b512.json" 2> "$OUT/b512.err" || exit $?
python3 -c "import json; d=json.load(open('$OUT/b512.json')); print(512, d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/rocprof" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --batch 512 --no-cpu-baseline --no-wide --no-forward --steps 200 --warmup 50 \
  > "$GRAFT_REPO_ROOT/$OUT/rocprof.log" 2>&1
