#!/bin/bash
# strided dw dgrad with the input BN's partials: tests, cross-build A/B (configs 5 and 3), config 5 shapes.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 700 python -u -m pytest tests/test_gpu_bn_on_load.py tests/test_gpu_bf16.py tests/test_gpu_bf16_fullsize.py \
    tests/test_gpu_layers.py tests/test_gpu_network.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_r03o.log" 2>&1
rc=$?; tail -3 "$OUT/tests_r03o.log"; step tests $rc
BASE_ENV=DORKNET_DW_STRIDED_BN=0 bash scripts/ab_builds.sh 5 2 > "$OUT/abb5_r03o.txt" 2>&1
rc=$?; cat "$OUT/abb5_r03o.txt"; step abb5 $rc
BASE_ENV=DORKNET_DW_STRIDED_BN=0 bash scripts/ab_builds.sh 3 2 > "$OUT/abb3_r03o.txt" 2>&1
rc=$?; cat "$OUT/abb3_r03o.txt"; step abb3 $rc
timeout -k 10 120 python scripts/call_shapes.py --config 5 --min-us 10 > "$OUT/call_shapes_c5_r03o.txt" 2>&1
step shapes $?
timeout -k 10 300 python scripts/ab_step.py --config 5 --knob env:DORKNET_DW_STRIDED_BN=0 --knob env:DORKNET_DW_STRIDED_BN=1 \
    --rounds 3 --steps 8 > "$OUT/ab5_r03o.txt" 2>&1
rc=$?; grep knob "$OUT/ab5_r03o.txt"; step ab5 $rc
