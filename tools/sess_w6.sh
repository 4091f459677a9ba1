#!/bin/bash
# wl2x6 (split-bf16 wide L2 forward): parity, then same-box wide A/B vs HEAD
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/w6; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_split_arith_gpu.py -k wide -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/split_wide.log 2>&1
rc=$?; tail -15 $OUT/split_wide.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_wide.sh w6/ab cnn-super-resolution_amd/lib/variants/libsrcnn_hip_head.so cnn-super-resolution_amd/lib/variants/libsrcnn_hip_w6.so
