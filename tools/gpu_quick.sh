#!/bin/bash
# Quick GPU iteration: every -m gpu parity test, then one bench line
# (no CPU baseline).  Output: gpurun_out/<tag>/{pytest.log,bench.json}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-q}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.err"
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("default", d["value"], "tiles/s", d["ms_per_step"], "ms", "step_roof", d["step_roofline"]["frac"])
for k, v in d["kernels"].items(): print("  ", k, v["ms_per_step"])
if "forward" in d: print("forward", d["forward"]["mpix_s"], "Mpix/s", d["forward"]["ms_per_frame"], "ms")
if "wide" in d:
    w = d["wide"]; print("wide", w["tiles_s"], "tiles/s", w["ms_per_step"], "ms", "step_roof", w["step_roofline"]["frac"])
    for k, v in w["kernels"].items(): print("  ", k, v["ms_per_step"])
PY
exit $rc
