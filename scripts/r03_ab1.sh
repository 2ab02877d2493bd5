#!/bin/bash
# Round-3 A/B: nontemporal output stores (knob 4) on the config-3 step; config-2 row tiles.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 300 python scripts/ab_step.py --knob 4:0 --knob 4:1 --rounds 4 --steps 10 > "$OUT/ab_nt_r03.txt" 2>&1
rc=$?; cat "$OUT/ab_nt_r03.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/cfg2_ab.py -1,6,8,14 > "$OUT/cfg2_ab_r03.txt" 2>&1
rc=$?; cat "$OUT/cfg2_ab_r03.txt"; exit $rc
