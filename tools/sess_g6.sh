#!/bin/bash
# wgrad2x6 (split-bf16 wide gW2): parity, then same-box wide A/B vs the wl2x6 tree
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/g6; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_split_arith_gpu.py -k wide -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/split_wide.log 2>&1
rc=$?; grep -E "W2|B2|PASS|FAIL|Error|error" $OUT/split_wide.log | tail -30; [ $rc -eq 0 ] || exit $rc
bash tools/ab_wide.sh g6/ab cnn-super-resolution_amd/lib/variants/libsrcnn_hip_w6.so cnn-super-resolution_amd/lib/variants/libsrcnn_hip_g6.so
