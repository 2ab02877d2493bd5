#!/bin/bash
# Quick GPU check: parity tests, a bench line, and a rocprofv3 kernel-stats run.
# Usage (via gpurun): bash scripts/quick_gpu.sh TAG [--no-tests] [--no-prof]
set -u
TAG=${1:-q}; shift || true
TESTS=1; PROF=1
for a in "$@"; do case $a in --no-tests) TESTS=0;; --no-prof) PROF=0;; esac; done
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
if [ $TESTS = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
  rc=$?; tail -4 "$OUT/tests_$TAG.log"; step tests $rc
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-sample 0 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cat "$OUT/bench_$TAG.json"; step bench $rc
if [ $PROF = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o bench -- \
      python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
  rc=$?; step rocprof $rc
  cd "$ROOT" && python scripts/prof_summary.py "$OUT/prof_$TAG" --steps 8 > "$OUT/kstats_$TAG.md" && head -45 "$OUT/kstats_$TAG.md"
fi
