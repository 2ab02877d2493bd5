#!/bin/bash
# Round-4 GPU pass: an optional kernel micro-bench (scripts/<name>.py), the -m gpu suite (or a
# selection), and a bench line.  Each step under its own time limit; stops at the first failure.
# Usage (gpurun): bash scripts/r04_gpu.sh TAG [--kbench NAME] [--tests "pytest args" | --no-tests] [--no-bench] [--config N]
set -u
TAG=$1; shift
KB=""; TESTS="tests -m gpu"; BENCH=1; CFG=3
while [ $# -gt 0 ]; do
  case $1 in
    --kbench) KB=$2; shift;;
    --tests) TESTS=$2; shift;;
    --no-tests) TESTS="";;
    --no-bench) BENCH=0;;
    --config) CFG=$2; shift;;
  esac
  shift
done
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
if [ -n "$KB" ]; then
  timeout -k 10 300 python -u scripts/$KB.py > "$OUT/${KB}_$TAG.txt" 2>&1
  rc=$?; cat "$OUT/${KB}_$TAG.txt"; step kbench $rc
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      > "$OUT/tests_$TAG.log" 2>&1
  rc=$?; tail -4 "$OUT/tests_$TAG.log"; step tests $rc
fi
if [ $BENCH = 1 ]; then
  timeout -k 10 400 python bench.py --config $CFG --cpu-sample 0 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; cut -c1-600 "$OUT/bench_$TAG.json"; step bench $rc
fi
