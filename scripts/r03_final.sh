#!/bin/bash
# Round-3 end-of-session GPU pass: scripts/r02_final.sh (the -m gpu suite, smoke, the config-3 bench
# line with the CPU baseline, rocprof kernel stats, PMC traffic), then the config-5 and config-2 lines.
# Usage (gpurun): bash scripts/r03_final.sh TAG
set -u
TAG=${1:-final}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
bash scripts/r02_final.sh "$TAG" || exit $?
timeout -k 10 300 python bench.py --config 5 > "$OUT/bench5_$TAG.json" 2> "$OUT/bench5_$TAG.err"
rc=$?; cut -c1-300 "$OUT/bench5_$TAG.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 2 > "$OUT/bench2_$TAG.json" 2> "$OUT/bench2_$TAG.err"
rc=$?; cut -c1-300 "$OUT/bench2_$TAG.json"; exit $rc
