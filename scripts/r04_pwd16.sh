#!/bin/bash
# Round-4 pass over the deep pointwise kernels: the fp32 deep tests, the bf16 streaming/deep tests,
# and scripts/pwd16_bench.py.  Each step under its own time limit; stops at the first failure.
set -u
TAG=$1
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_pw_deep.py tests/test_gpu_pw_stream_bf16.py -x -q -rf --timeout 200 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pwd16_tests_$TAG.log" 2>&1
rc=$?; grep -E "^FAILED|assert|Error" "$OUT/pwd16_tests_$TAG.log" | head -20; tail -2 "$OUT/pwd16_tests_$TAG.log"; step tests $rc
timeout -k 10 300 python -u scripts/pwd16_bench.py > "$OUT/pwd16_bench_$TAG.txt" 2>&1
rc=$?; cat "$OUT/pwd16_bench_$TAG.txt"; step bench $rc
