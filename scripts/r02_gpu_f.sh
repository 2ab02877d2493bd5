#!/bin/bash
# Usage (gpurun): bash scripts/r02_gpu_f.sh TAG "test files..." [bench] [prof]
# tests (stop on failure) -> optional bench line -> optional rocprofv3 kernel stats of the bench.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-x}; TESTS=${2:-}; BENCH=${3:-}; PROF=${4:-}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
  rc=$?; tail -15 "$OUT/tests_$TAG.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --cpu-sample 0 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; cat "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o bench -- \
      python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
