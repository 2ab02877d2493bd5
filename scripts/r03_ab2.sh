#!/bin/bash
# Round-3 A/B: the streaming fused pointwise backward with / without operand prefetch (knob 5),
# nontemporal stores (knob 4), then the config-2 row tiles and the DP tests.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 400 python scripts/ab_step.py --knob 5:1 --knob 5:0 --knob 4:1 --knob 4:0 --rounds 4 --steps 10 \
    > "$OUT/ab_r03b.txt" 2>&1
rc=$?; cat "$OUT/ab_r03b.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/cfg2_ab.py -1,6,8,14 > "$OUT/cfg2_ab_r03.txt" 2>&1
rc=$?; cat "$OUT/cfg2_ab_r03.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_pw_bwd_fused.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > "$OUT/dp_r03.log" 2>&1
rc=$?; tail -5 "$OUT/dp_r03.log"; exit $rc
