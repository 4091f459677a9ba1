#!/bin/bash
# Diagnostic (results invalid in the diag build): the wide step with and
# without the conv kernels' next-chunk LDS-DMA (SRCNN_WIDE_DIAG=4), twice each.
#   tools/build_variant.sh base && tools/build_variant.sh diag4 -DSRCNN_WIDE_DIAG=4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-diag}; mkdir -p "$OUT"
V=cnn-super-resolution_amd/lib/variants
for rep in 1 2; do
  for v in base diag4; do
    SRCNN_HIP_LIB=$PWD/$V/libsrcnn_hip_$v.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-forward \
      --steps 20 --warmup 5 > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v', $rep, d['wide']['ms_per_step'], {k:round(x['ms_per_step'],4) for k,x in d['wide']['kernels'].items()})"
  done
done
