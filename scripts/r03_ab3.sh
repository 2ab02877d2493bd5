#!/bin/bash
# A/B of nontemporal output stores (knob 4) on the step, then the full GPU suite.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 400 python scripts/ab_step.py --knob 4:0 --knob 4:1 --rounds 5 --steps 10 > "$OUT/ab_r03c.txt" 2>&1
rc=$?; cat "$OUT/ab_r03c.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_r03c.log" 2>&1
rc=$?; tail -4 "$OUT/tests_r03c.log"; exit $rc
