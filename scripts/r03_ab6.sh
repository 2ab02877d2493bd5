#!/bin/bash
# config 5 A/B: bf16 streaming pointwise (knob 9) and row / split-K tiles for the deep bf16 GEMMs.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 600 python scripts/ab_step.py --config 5 --knob 9:0 --knob 9:1 --knob 0:10 --knob 0:11 --knob 0:5 \
    --knob 0:16 --knob 0:2 --knob 1:2 --knob 1:4 --knob 1:5 --rounds 3 --steps 8 > "$OUT/ab_r03k.txt" 2>&1
rc=$?; grep knob "$OUT/ab_r03k.txt"; exit $rc
