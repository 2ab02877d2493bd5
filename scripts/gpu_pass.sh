#!/bin/bash
# One GPU pass: an optional kernel micro-bench (scripts/<name>.py), the -m gpu suite (or a selection),
# and bench lines.  Each step under its own time limit; stops at the first failure.
# Usage (gpurun): bash scripts/gpu_pass.sh TAG [--kbench NAME] [--tests "pytest args" | --no-tests]
#                 [--configs "3 5 2" | --no-bench] [--smoke]
set -u
TAG=$1; shift
KB=""; TESTS="tests -m gpu"; CFGS="3"; SMOKE=0
while [ $# -gt 0 ]; do
  case $1 in
    --kbench) KB=$2; shift;;
    --tests) TESTS=$2; shift;;
    --no-tests) TESTS="";;
    --configs) CFGS=$2; shift;;
    --no-bench) CFGS="";;
    --smoke) SMOKE=1;;
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
if [ $SMOKE = 1 ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  rc=$?; tail -1 "$OUT/smoke_$TAG.log"; step smoke $rc
fi
for c in $CFGS; do
  timeout -k 10 400 python bench.py --config $c --cpu-sample 0 > "$OUT/bench${c}_$TAG.json" 2> "$OUT/bench${c}_$TAG.err"
  rc=$?; cut -c1-500 "$OUT/bench${c}_$TAG.json"; step bench$c $rc
done
