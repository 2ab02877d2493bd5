#!/bin/bash
# bf16: streaming + tuned tiles + in-launch folds; bf16 / fold tests, config 5 A/B and bench line.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_pw_stream_bf16.py tests/test_gpu_bf16.py tests/test_gpu_bf16_fullsize.py \
    tests/test_gpu_fold.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/tests_bf16_r03l.log" 2>&1
rc=$?; tail -3 "$OUT/tests_bf16_r03l.log"; step tests $rc
timeout -k 10 400 python scripts/ab_step.py --config 5 --knob 9:0 --knob 9:1 --knob env:DORKNET_INLAUNCH_FOLD=0 \
    --rounds 3 --steps 8 > "$OUT/ab_r03l.txt" 2>&1
rc=$?; grep knob "$OUT/ab_r03l.txt"; step ab $rc
timeout -k 10 300 python bench.py --config 5 --batch 512 --steps 10 --warmup 3 > "$OUT/bench5_r03l.json" 2> "$OUT/bench5_r03l.err"
rc=$?; cut -c1-300 "$OUT/bench5_r03l.json"; step bench5 $rc
