#!/bin/bash
# Round-4 end-of-session GPU pass: scripts/r03_final.sh (the -m gpu suite, smoke, the config-3 bench
# line, rocprof kernel stats, config-3 PMC traffic, the config-5 and config-2 lines), then the two
# HBM-traffic passes over the config-5 (bf16) step for its roofline `traffic`.
# Usage (gpurun): bash scripts/r04_final.sh TAG [--skip-base]
set -u
TAG=${1:-final}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
if [ "${2:-}" != "--skip-base" ]; then bash scripts/r03_final.sh "$TAG" || exit $?; fi
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --config 5 --steps 3 --warmup 1 --cpu-sample 0 --no-roofline"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/pmc5_$TAG/fetch" -o run -- python $BENCH \
    > "$OUT/pmc5_${TAG}_fetch.log" 2>&1
step fetch5 $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/pmc5_$TAG/write" -o run -- python $BENCH \
    > "$OUT/pmc5_${TAG}_write.log" 2>&1
step write5 $?
cd "$ROOT"
python scripts/pmc_summary.py "$OUT/pmc5_$TAG/fetch" "$OUT/pmc5_$TAG/write" --out "$OUT/${TAG}_config5_pmc.json" \
    > "$OUT/${TAG}_config5_pmc_summary.txt" 2>&1
step summary5 $?
