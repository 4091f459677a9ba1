#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step runs under its own time limit; any fault / abort / timeout
# ends the session (exit codes >= 124 or signals), plain test failures do not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

echo "== rocm-smi" && (rocm-smi --showproductname > "$OUT/smi.txt" 2>&1 || true)
# every parity check logs its achieved errors (tests/hip_util.py); the raw log
# and its summary go under profiles/ with the session
rm -f "$OUT/parity_checks.jsonl"
SRCNN_PARITY_LOG=$PWD/$OUT/parity_checks.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
[ -s "$OUT/parity_checks.jsonl" ] && python3 tools/parity_summary.py "$OUT/parity_checks.jsonl" > "$OUT/parity_summary.json"
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/rocprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" ${BENCH_ARGS:-} --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/rocprof_bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
