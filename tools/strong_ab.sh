#!/bin/bash
# Per-rank strong-scaling workloads (bench.py --global-batch G on one GPU) for
# library variants: tools/strong_ab.sh <tag> <lib.so|default>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-strong}; shift
mkdir -p "$OUT"
for lib in "$@"; do
  for gb in ${GBS:-512 1024 2048}; do
    tag=$(basename "$lib" .so)_$gb
    if [ "$lib" = default ]; then unset SRCNN_HIP_LIB; else export SRCNN_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --global-batch $gb --steps 200 --warmup 50 --no-cpu-baseline \
        --no-forward --no-wide > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})" "$OUT/$tag.json" "$tag"
  done
done
