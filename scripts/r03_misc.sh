#!/bin/bash
# Diagnostics: torch-side copies/fills of a step; BASELINE config 2 bench line + rocprof kernel stats.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 200 python scripts/find_copies.py > "$OUT/copies_r03i.txt" 2>&1
step copies $?
timeout -k 10 300 python bench.py --config 2 > "$OUT/bench2_r03i.json" 2> "$OUT/bench2_r03i.err"
step bench2 $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof2_r03i" -o c2 -- \
    python "$ROOT/bench.py" --config 2 --steps 10 --warmup 3 --cpu-sample 0 --no-roofline > "$OUT/prof2_r03i.log" 2>&1
step rocprof2 $?
