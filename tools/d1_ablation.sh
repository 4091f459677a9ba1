#!/bin/bash
# d1_grad12 ablation: bench-only variants with one part of the chunk removed
# (results invalid; timing only).  Bits of SRCNN_D1_DIAG: 1 no delta1 MFMAs,
# 2 no gW2 MFMAs, 4 no relu' mask, 8 no gW1 MFMAs, 16 no operand DMA.
# Build:  for d in 0 1 2 4 8 16; do tools/build_variant.sh diag$d -DSRCNN_D1_DIAG=$d; done
# Run:    gpurun -- tools/d1_ablation.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=cnn-super-resolution_amd/lib/variants
BV_ARGS="--no-wide --no-forward" tools/bench_variants.sh d1abl $V/libsrcnn_hip_diag0.so $V/libsrcnn_hip_diag1.so \
  $V/libsrcnn_hip_diag2.so $V/libsrcnn_hip_diag4.so $V/libsrcnn_hip_diag8.so $V/libsrcnn_hip_diag16.so $V/libsrcnn_hip_diag0.so
