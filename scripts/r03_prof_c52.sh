#!/bin/bash
# rocprofv3 kernel statistics for BASELINE configs 5 and 2 and the two HBM-traffic counter passes for
# config 5.  Usage (gpurun): bash scripts/r03_prof_c52.sh TAG
set -u
TAG=${1:-c52}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof5_$TAG" -o bench -- \
    python "$ROOT/bench.py" --config 5 --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$OUT/prof5_$TAG.log" 2>&1
step prof5 $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof2_$TAG" -o bench -- \
    python "$ROOT/bench.py" --config 2 --steps 10 --warmup 3 --cpu-sample 0 --no-roofline > "$OUT/prof2_$TAG.log" 2>&1
step prof2 $?
B5="$ROOT/bench.py --config 5 --steps 3 --warmup 1 --cpu-sample 0 --no-roofline"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/pmc5_$TAG/fetch" -o run -- python $B5 \
    > "$OUT/pmc5_${TAG}_fetch.log" 2>&1
step fetch5 $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/pmc5_$TAG/write" -o run -- python $B5 \
    > "$OUT/pmc5_${TAG}_write.log" 2>&1
step write5 $?
