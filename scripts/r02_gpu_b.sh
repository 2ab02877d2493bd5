#!/bin/bash
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r02c}
timeout -k 10 300 python -u -m pytest tests/test_gpu_pw_stream.py tests/test_gpu_bn_on_load.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_pws_$TAG.log" 2>&1
rc=$?; tail -4 "$OUT/tests_pws_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/pws_bench.py > "$OUT/pws_$TAG.txt" 2>&1
rc=$?; cat "$OUT/pws_$TAG.txt" | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s --timeout 280 --timeout-method thread -p no:cacheprovider > "$OUT/tests_full_$TAG.log" 2>&1
rc=$?; grep -E "PASS|FAIL|errors|^  " "$OUT/tests_full_$TAG.log" | head -80; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-sample 0 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cat "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
