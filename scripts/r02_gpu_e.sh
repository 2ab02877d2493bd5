#!/bin/bash
# Usage (gpurun): bash scripts/r02_gpu_e.sh TAG "test files..." [bench]
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-x}; TESTS=${2:-}; BENCH=${3:-}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
  rc=$?; tail -4 "$OUT/tests_$TAG.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python -u scripts/pws_bench.py > "$OUT/pws_$TAG.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/pws_$TAG.txt"; [ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --cpu-sample 0 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; cat "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
fi
