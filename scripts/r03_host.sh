#!/bin/bash
# host-side issue cost after the raw stream / device lookups: full GPU suite, host overhead, cross-build A/B.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_r03n.log" 2>&1
rc=$?; tail -3 "$OUT/tests_r03n.log"; step tests $rc
timeout -k 10 200 python scripts/host_overhead.py --config 3 --steps 10 > "$OUT/host3_r03n.txt" 2>&1
rc=$?; head -3 "$OUT/host3_r03n.txt"; step host3 $rc
timeout -k 10 200 python scripts/host_overhead.py --config 5 --steps 10 --profile > "$OUT/host5_r03n.txt" 2>&1
rc=$?; grep "host issue" "$OUT/host5_r03n.txt"; step host5 $rc
timeout -k 10 300 python scripts/ab_step.py --config 3 --knob 2:-1 --rounds 3 --steps 10 > "$OUT/ab3_r03n.txt" 2>&1
rc=$?; grep knob "$OUT/ab3_r03n.txt"; step ab3 $rc
timeout -k 10 300 python scripts/ab_step.py --config 5 --knob 2:-1 --rounds 3 --steps 10 > "$OUT/ab5_r03n.txt" 2>&1
rc=$?; grep knob "$OUT/ab5_r03n.txt"; step ab5 $rc
