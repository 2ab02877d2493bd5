#!/bin/bash
# Round-2 GPU check A: full GPU test suite, the default bench line (with CPU baseline),
# and the 2-rank launch test of bench.py --gpus 2 (ranks share the one GPU: gloo).
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r02a}
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
rc=$?; tail -6 "$OUT/tests_$TAG.log"; step tests $rc
timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cat "$OUT/bench_$TAG.json"; step bench $rc
timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-roofline > "$OUT/bench2_$TAG.json" 2> "$OUT/bench2_$TAG.err"
rc=$?; cat "$OUT/bench2_$TAG.json"; tail -3 "$OUT/bench2_$TAG.err"; step bench2 $rc
