#!/bin/bash
# Round-3 bf16 MFMA check: the bf16 tests (kernel contracts, stack vs oracle, config 5 at batch 512)
# and a config-5 bench line.  Usage (gpurun): bash scripts/r03_bf16.sh TAG
set -u
TAG=${1:-b}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_bf16_fullsize.py -v -s --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/bf16_tests_$TAG.log" 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" "$OUT/bf16_tests_$TAG.log" | tail -30; step tests $rc
timeout -k 10 300 python bench.py --config 5 --batch 512 --steps 10 --warmup 3 > "$OUT/bench5_$TAG.json" 2> "$OUT/bench5_$TAG.err"
rc=$?; cut -c1-3000 "$OUT/bench5_$TAG.json"; step bench5 $rc
