#!/bin/bash
# GPU iteration: the -m gpu tests (optionally a -k filter), then one bench
# line without the CPU baselines and a rocprofv3 kernel-stats pass of it.
#   tools/gpu_iter.sh TAG ["pytest -k expr"]
# Output: gpurun_out/TAG/{pytest.log,bench.json,rocprof/...}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-iter}; mkdir -p "$OUT"
export TMPDIR=/tmp
K=${2:-}
if [ -n "$K" ]; then
  SRCNN_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
else
  SRCNN_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.err"
[ $rc -eq 0 ] || exit $rc
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("default", d["value"], "tiles/s", d["ms_per_step"], "ms", "step_roof", d["step_roofline"]["frac"])
for k, v in d["kernels"].items(): print("  ", k, v["ms_per_step"])
if "forward" in d: print("forward", d["forward"]["mpix_s"], "Mpix/s", d["forward"]["ms_per_frame"], "ms")
if "wide" in d:
    w = d["wide"]; print("wide", w["tiles_s"], "tiles/s", w["ms_per_step"], "ms", "step_roof", w["step_roofline"]["frac"])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/rocprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-wide --no-forward > "$GRAFT_REPO_ROOT/$OUT/rocprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
