#!/bin/bash
# bf16 streaming pointwise kernels: their bitwise tests, the bf16 suite, config 5 A/B (knob 9) and bench line.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_pw_stream_bf16.py -x -q --timeout 100 --timeout-method thread \
    -p no:cacheprovider > "$OUT/tests_pwsh.log" 2>&1
rc=$?; tail -3 "$OUT/tests_pwsh.log"; step pwsh $rc
timeout -k 10 120 python scripts/call_shapes.py --config 5 --min-us 10 > "$OUT/call_shapes_c5.txt" 2>&1
step shapes $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_bf16_fullsize.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/tests_bf16_r03j.log" 2>&1
rc=$?; tail -3 "$OUT/tests_bf16_r03j.log"; step bf16 $rc
timeout -k 10 300 python bench.py --config 5 --batch 512 --steps 10 --warmup 3 > "$OUT/bench5_r03j.json" 2> "$OUT/bench5_r03j.err"
rc=$?; cut -c1-300 "$OUT/bench5_r03j.json"; step bench5 $rc
