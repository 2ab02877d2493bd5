#!/bin/bash
# End-of-session GPU pass: the whole -m gpu suite, smoke(), the config-3 bench line with the CPU
# baseline, a rocprofv3 kernel-stats run, the FETCH_SIZE / WRITE_SIZE counter passes of configs 3 and 5
# (each in its own run), and the config-5 and config-2 lines.  Each step under its own time limit;
# stops at the first failure.  Usage (gpurun): bash scripts/final_pass.sh TAG [--skip-tests]
set -u
TAG=${1:-final}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
if [ "${2:-}" != "--skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      > "$OUT/tests_$TAG.log" 2>&1
  rc=$?; tail -3 "$OUT/tests_$TAG.log"; step tests $rc
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; tail -1 "$OUT/smoke_$TAG.log"; step smoke $rc
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cut -c1-400 "$OUT/bench_$TAG.json"; step bench $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o bench -- \
    python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
step rocprof $?
for c in 3 5; do
  BENCH="$ROOT/bench.py --config $c --steps 3 --warmup 1 --cpu-sample 0 --no-roofline"
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/pmc${c}_$TAG/fetch" -o run -- python $BENCH \
      > "$OUT/pmc${c}_${TAG}_fetch.log" 2>&1
  step fetch$c $?
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/pmc${c}_$TAG/write" -o run -- python $BENCH \
      > "$OUT/pmc${c}_${TAG}_write.log" 2>&1
  step write$c $?
done
cd "$ROOT"
python scripts/prof_summary.py "$OUT/prof_$TAG" --steps 6 > "$OUT/kstats_$TAG.md" && head -12 "$OUT/kstats_$TAG.md"
python scripts/pmc_summary.py "$OUT/pmc3_$TAG/fetch" "$OUT/pmc3_$TAG/write" --out "$OUT/${TAG}_pmc.json" \
    > "$OUT/${TAG}_pmc_summary.txt" 2>&1
step summary3 $?
python scripts/pmc_summary.py "$OUT/pmc5_$TAG/fetch" "$OUT/pmc5_$TAG/write" --out "$OUT/${TAG}_config5_pmc.json" \
    > "$OUT/${TAG}_config5_pmc_summary.txt" 2>&1
step summary5 $?
timeout -k 10 300 python bench.py --config 5 > "$OUT/bench5_$TAG.json" 2> "$OUT/bench5_$TAG.err"
rc=$?; cut -c1-300 "$OUT/bench5_$TAG.json"; step bench5 $rc
timeout -k 10 300 python bench.py --config 2 > "$OUT/bench2_$TAG.json" 2> "$OUT/bench2_$TAG.err"
rc=$?; cut -c1-300 "$OUT/bench2_$TAG.json"; step bench2 $rc
