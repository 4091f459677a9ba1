#!/bin/bash
# Round-5 session: the driver's exact bench command next to the 30 + 100
# default on one box, and a rocprofv3 kernel trace of the driver's command
# (per-launch durations of every headline kernel across the whole run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r05_clock}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
rocm-smi --showproductname > "$OUT/smi.txt" 2>&1 || true
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/d20a.json" 2> "$OUT/d20a.err" || exit $?
echo "d20a"; python3 -c "import json; d=json.load(open('$OUT/d20a.json')); print(d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/d100.json" 2> "$OUT/d100.err" || exit $?
echo "d100"; python3 -c "import json; d=json.load(open('$OUT/d100.json')); print(d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/d20b.json" 2> "$OUT/d20b.err" || exit $?
echo "d20b"; python3 -c "import json; d=json.load(open('$OUT/d20b.json')); print(d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/rocprof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$ROOT/$OUT/rocprof_d20.log" 2>&1 || exit $?
echo "rocprof ok"
