#!/bin/bash
# Round-2 end-of-session GPU pass: the whole -m gpu suite, smoke(), the default bench line (with the
# CPU baseline), a rocprofv3 kernel-stats run and the two HBM-traffic counter passes.
# Usage (gpurun): bash scripts/r02_final.sh TAG
set -u
TAG=${1:-final}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_$TAG.log" 2>&1
rc=$?; tail -3 "$OUT/tests_$TAG.log"; step tests $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; tail -1 "$OUT/smoke_$TAG.log"; step smoke $rc
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cut -c1-400 "$OUT/bench_$TAG.json"; step bench $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o bench -- \
    python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
step rocprof $?
BENCH="$ROOT/bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-roofline"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/pmc_$TAG/fetch" -o run -- python $BENCH \
    > "$OUT/pmc_${TAG}_fetch.log" 2>&1
step fetch $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/pmc_$TAG/write" -o run -- python $BENCH \
    > "$OUT/pmc_${TAG}_write.log" 2>&1
step write $?
cd "$ROOT"
python scripts/prof_summary.py "$OUT/prof_$TAG" --steps 6 > "$OUT/kstats_$TAG.md" && head -12 "$OUT/kstats_$TAG.md"
python scripts/pmc_summary.py "$OUT/pmc_$TAG/fetch" "$OUT/pmc_$TAG/write" --out "$OUT/${TAG}_pmc.json" \
    > "$OUT/${TAG}_pmc_summary.txt" 2>&1
step summary $?
