#!/bin/bash
# Same-box A/B of the working tree's library against lib/variants/libsrcnn_hip_head.so
# (tools/build_rev_variant.sh head <rev>): the training-step parity tests with
# each, then bench.py (no side legs) and the 512-tile shard, interleaved twice.
#   tools/ab_head.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${1:-ab_head}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
HEAD=$ROOT/cnn-super-resolution_amd/lib/variants/libsrcnn_hip_head.so
CUR=$ROOT/cnn-super-resolution_amd/lib/libsrcnn_hip.so
for v in head cur; do
  lib=$HEAD; [ $v = cur ] && lib=$CUR
  SRCNN_HIP_LIB=$lib timeout -k 10 300 python -m pytest tests/test_parity_gpu.py tests/test_dp_gpu.py -m gpu -q -x \
    -p no:cacheprovider -k "train_step or lazy or full_batch" > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "$v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in head cur; do
    lib=$HEAD; [ $v = cur ] && lib=$CUR
    SRCNN_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-wide --no-forward "$@" \
      > "$OUT/bench_${v}_$rep.json" 2> "$OUT/bench_${v}_$rep.err" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/bench_${v}_$rep.json')); print('$v', $rep, d['value'], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
    SRCNN_HIP_LIB=$lib timeout -k 10 300 python tools/strong_shard.py --modes lazy,step \
      > "$OUT/strong_${v}_$rep.jsonl" 2> "$OUT/strong_${v}_$rep.err" || exit $?
    sed "s/^/$v $rep /" "$OUT/strong_${v}_$rep.jsonl"
  done
done
