#!/bin/bash
# sub-pixel dgrad operands as pipelined buffer loads: tests, per-call shapes (configs 3 and 5), cross-build A/B.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_bn_on_load.py tests/test_gpu_layers.py tests/test_gpu_network.py \
    tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_r03p.log" 2>&1
rc=$?; tail -3 "$OUT/tests_r03p.log"; step tests $rc
timeout -k 10 120 python scripts/call_shapes.py --config 5 --min-us 10 > "$OUT/call_shapes_c5_r03p.txt" 2>&1
step shapes5 $?
timeout -k 10 120 python scripts/call_shapes.py --config 3 --min-us 10 > "$OUT/call_shapes_c3_r03p.txt" 2>&1
step shapes3 $?
grep -E "dwconv_dgrad" "$OUT/call_shapes_c5_r03p.txt" "$OUT/call_shapes_c3_r03p.txt"
BASE_ENV=DORKNET_DW_STRIDED_BN=0 bash scripts/ab_builds.sh 5 2 > "$OUT/abb5_r03p.txt" 2>&1
rc=$?; cat "$OUT/abb5_r03p.txt"; step abb5 $rc
bash scripts/ab_builds.sh 3 3 > "$OUT/abb3_r03p.txt" 2>&1
rc=$?; cat "$OUT/abb3_r03p.txt"; step abb3 $rc
