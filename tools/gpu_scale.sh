#!/bin/bash
# GPU session: all -m gpu tests, the default bench line, then the per-rank
# workload of strong scaling (global batch 4096 over N GPUs = 4096/N tiles per
# rank) measured on one GPU at batch 512 / 1024 / 2048 / 4096, and a
# rocprofv3 kernel trace of the batch-512 step (the 8-GPU per-rank step).
# Every GPU step has its own time limit; a fault / timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-scale}
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; head -c 1500 "$OUT/bench.json"; echo; tail -3 "$OUT/bench.err"
[ $rc -eq 0 ] || exit $rc
for gb in 512 1024 2048 4096; do
  timeout -k 10 300 python bench.py --global-batch $gb --steps 200 --warmup 50 --no-cpu-baseline \
      --no-forward --no-wide > "$OUT/strong_$gb.json" 2> "$OUT/strong_$gb.err"
  rc=$?; echo "strong gb=$gb rc=$rc"; head -c 400 "$OUT/strong_$gb.json"; echo
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/rocprof512" \
    -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --global-batch 512 --steps 200 \
    --warmup 50 --no-cpu-baseline --no-forward --no-wide > "$GRAFT_REPO_ROOT/$OUT/rocprof512.log" 2>&1
rc=$?; echo "rocprof512 rc=$rc"
exit $rc
