#!/bin/bash
# A/B: depthwise forward row segments (knob 8: 0 = always 8 rows, -1 = adaptive), then the affected GPU tests.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_bn_on_load.py -x -q -k "depthwise" \
    --timeout 100 --timeout-method thread -p no:cacheprovider > "$OUT/tests_r03h_dw.log" 2>&1
rc=$?; tail -2 "$OUT/tests_r03h_dw.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/ab_step.py --knob 8:0 --knob 8:-1 --knob 8:2048 --rounds 3 --steps 10 > "$OUT/ab_r03h.txt" 2>&1
rc=$?; grep knob "$OUT/ab_r03h.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_r03h.log" 2>&1
rc=$?; tail -3 "$OUT/tests_r03h.log"; exit $rc
