#!/bin/bash
# Round-5 verification session: GPU tests + smoke, the bench at its defaults
# and at the driver's flags (twice), a rocprofv3 kernel trace of the driver's
# command, the strong-scaling shard, the N = 2 launcher rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/${1:-r05_c}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocm-smi --showproductname > "$OUT/smi.txt" 2>&1 || true
rm -f "$OUT/parity_checks.jsonl"
SRCNN_PARITY_LOG=$ROOT/$OUT/parity_checks.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ -s "$OUT/parity_checks.jsonl" ] && python3 tools/parity_summary.py "$OUT/parity_checks.jsonl" > "$OUT/parity_summary.json"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json; d=json.load(open('$1')); print('$2', d['value'], d['ms_per_step'], d['config'].get('settle_steps'), {k: v['ms_per_step'] for k, v in d['kernels'].items()}, 'wide', d.get('wide', {}).get('ms_per_step'), 'fwd', d.get('forward', {}).get('ms_per_frame'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; }
timeout -k 10 400 python bench.py > "$OUT/d100.json" 2> "$OUT/d100.err" || exit $?
summ "$OUT/d100.json" d100
for r in a b; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/d20$r.json" 2> "$OUT/d20$r.err" || exit $?
  summ "$OUT/d20$r.json" d20$r
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/rocprof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$ROOT/$OUT/rocprof_d20.log" 2>&1 || exit $?
cd "$ROOT"; echo "rocprof ok"
timeout -k 10 300 python tools/strong_shard.py --modes lazy,separate,step > "$OUT/strong.jsonl" 2> "$OUT/strong.err" || exit $?
cat "$OUT/strong.jsonl"
bash tools/rehearse_n2.sh "${1:-r05_c}/rehearse" || exit $?
