#!/bin/bash
# One GPU-box session: parity tests, a 1-GPU bench line, a rocprofv3 kernel-stats profile and
# the two PMC passes (FETCH_SIZE, WRITE_SIZE) that give the dominant kernel's HBM traffic.
# Usage (from the repo root, via gpurun): bash scripts/gpu_session.sh [tag]
# Each GPU step has its own time limit; a crash / timeout (rc > 1) ends the session.
set -u
TAG=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -gt 1 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }

timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
rc=$?; tail -15 "$OUT/tests_$TAG.log"; step tests $rc

cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o bench -- \
    python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
rc=$?; step rocprof $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -f csv -d "$OUT/pmc_${TAG}_$c" -o run -- \
      python "$ROOT/bench.py" --steps 2 --warmup 1 --cpu-sample 0 --no-roofline > "$OUT/pmc_${TAG}_$c.json" \
      2> "$OUT/pmc_${TAG}_$c.err"
  rc=$?; step "pmc $c" $rc
done
cd "$ROOT"
python scripts/pmc_summary.py "$OUT/pmc_${TAG}_FETCH_SIZE" "$OUT/pmc_${TAG}_WRITE_SIZE" --out "$OUT/${TAG}_pmc.json" \
    > "$OUT/pmc_$TAG.txt" 2>&1; cat "$OUT/pmc_$TAG.txt"
cp "$OUT/${TAG}_pmc.json" "$ROOT/profiles/" 2>/dev/null

timeout -k 10 900 python bench.py --steps 10 --warmup 3 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cat "$OUT/bench_$TAG.json"; tail -5 "$OUT/bench_$TAG.err"; step bench $rc

timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-roofline > "$OUT/bench2_$TAG.json" 2> "$OUT/bench2_$TAG.err"
rc=$?; cat "$OUT/bench2_$TAG.json"; tail -3 "$OUT/bench2_$TAG.err"; step bench2 $rc
