#!/bin/bash
# Round-4 last pass: scripts/r03_final.sh (the -m gpu suite, smoke, config-3 line + CPU baseline,
# rocprof, PMC, config-5 and config-2 lines), the bf16 depthwise forward per shape, and the config-5
# A/B of the strided-dgrad nontemporal family.  Usage (gpurun): bash scripts/r04_last.sh TAG
set -u
TAG=${1:-last}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
bash scripts/r03_final.sh "$TAG" || exit $?
DW_SEGS=-1 timeout -k 10 120 python scripts/dw_fwd_seg.py --bf16 > "$OUT/dwfwd16_$TAG.txt" 2>/dev/null || exit 1
bash scripts/env_ab.sh 5 2 DORKNET_NT_STORES 2431 3455 > "$OUT/ab_nt5_$TAG.txt" || exit 1
cat "$OUT/dwfwd16_$TAG.txt" "$OUT/ab_nt5_$TAG.txt"
