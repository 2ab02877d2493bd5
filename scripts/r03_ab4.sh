#!/bin/bash
# A/B: (1) BN backward unfused for the deep pointwise layers (DORKNET_BNBWD_UNFUSE_K), (2) image runs
# in the fused depthwise backward (knob 7: 0 = one image per block); then the affected GPU tests.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_bn_on_load.py -x -q -k "depthwise_bwd_bnbwd" --timeout 100 \
    --timeout-method thread -p no:cacheprovider > "$OUT/tests_r03g_dwb.log" 2>&1
rc=$?; tail -2 "$OUT/tests_r03g_dwb.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/ab_step.py --knob env:DORKNET_BNBWD_UNFUSE_K=100000 --knob env:DORKNET_BNBWD_UNFUSE_K=512 \
    --knob env:DORKNET_BNBWD_UNFUSE_K=256 --knob env:DORKNET_BNBWD_UNFUSE_K=128 --knob 7:0 --knob 7:768 --knob 7:1024 \
    --rounds 3 --steps 10 > "$OUT/ab_r03g.txt" 2>&1
rc=$?; grep knob "$OUT/ab_r03g.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_network.py tests/test_gpu_fullsize.py tests/test_gpu_fold.py \
    tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests_r03g.log" 2>&1
rc=$?; tail -3 "$OUT/tests_r03g.log"; exit $rc
