#!/bin/bash
# Round-6 GPU pass: named steps, each under its own time limit, stopping at the first failure.
# Usage (gpurun): bash scripts/r06_pass.sh TAG step [step ...]
#   deep      tests/test_gpu_pw_deep.py            net    whole-network training tests (-v -s: tie report)
#   pwdbench  scripts/pwd_bench.py --only dgrad    smoke  __graft_entry__.smoke()
#   bench     config 3 bench line                  bench5 / bench2   the config 5 / 2 lines
#   prof      rocprofv3 kernel stats of config 3   suite  the whole -m gpu suite
#   sq        SQ counter passes of config 3 (scripts/sq_passes.sh)
#   file      the test file(s) in $TESTFILE
#   ab        config-3 bench lines alternating the knob settings in $AB (e.g. AB="21=2 21=1"), 2 rounds
#   prof0     as prof with the knob settings in $KNOBS (e.g. KNOBS="--knob 21=1")
#   abenv     config-3 bench lines alternating the environment settings in $ABENV (e.g. ABENV="A=0 A=1")
set -u
AB=${AB:-}; KNOBS=${KNOBS:-}; ABENV=${ABENV:-}; TESTFILE=${TESTFILE:-}
TAG=$1; shift
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
for s in "$@"; do
  case $s in
    deep) timeout -k 10 300 $PYT tests/test_gpu_pw_deep.py > "$OUT/tests_${TAG}_deep.log" 2>&1
          rc=$?; tail -2 "$OUT/tests_${TAG}_deep.log"; step deep $rc;;
    net) timeout -k 10 600 $PYT -v -s tests/test_gpu_network.py -k training_steps > "$OUT/tests_${TAG}_net.log" 2>&1
          rc=$?; tail -2 "$OUT/tests_${TAG}_net.log"; step net $rc;;
    pwdbench) timeout -k 10 300 python -u scripts/pwd_bench.py --only ${PWD_ONLY:-dgrad} --modes ${PWD_MODES:-0,1} > "$OUT/pwd_bench_${TAG}.txt" 2>&1
          rc=$?; cat "$OUT/pwd_bench_${TAG}.txt"; step pwdbench $rc;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_${TAG}.log" 2>&1
          rc=$?; tail -1 "$OUT/smoke_${TAG}.log"; step smoke $rc;;
    bench) timeout -k 10 400 python bench.py --cpu-sample 0 > "$OUT/bench3_${TAG}.json" 2> "$OUT/bench3_${TAG}.err"
          rc=$?; cut -c1-300 "$OUT/bench3_${TAG}.json"; step bench $rc;;
    bench5) timeout -k 10 300 python bench.py --config 5 > "$OUT/bench5_${TAG}.json" 2> "$OUT/bench5_${TAG}.err"
          rc=$?; cut -c1-300 "$OUT/bench5_${TAG}.json"; step bench5 $rc;;
    bench2) timeout -k 10 300 python bench.py --config 2 > "$OUT/bench2_${TAG}.json" 2> "$OUT/bench2_${TAG}.err"
          rc=$?; cut -c1-300 "$OUT/bench2_${TAG}.json"; step bench2 $rc;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o bench -- \
              python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err")
          rc=$?; step prof $rc
          python scripts/prof_summary.py "$OUT/prof_$TAG" --steps 6 > "$OUT/kstats_$TAG.md"; head -24 "$OUT/kstats_$TAG.md";;
    prof0) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof0_$TAG" -o bench -- \
              python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline $KNOBS > "$OUT/prof0_bench_$TAG.json" 2> "$OUT/prof0_$TAG.err")
          rc=$?; step prof0 $rc
          python scripts/prof_summary.py "$OUT/prof0_$TAG" --steps 6 > "$OUT/kstats0_$TAG.md"; head -24 "$OUT/kstats0_$TAG.md";;
    ab) for round in 1 2; do for kv in $AB; do
          timeout -k 10 300 python bench.py --cpu-sample 0 --no-roofline --knob $kv > "$OUT/ab_${TAG}_${kv}_$round.json" 2>/dev/null
          rc=$?; echo "knob $kv: $(grep -o 'ms_per_step": [0-9.]*' "$OUT/ab_${TAG}_${kv}_$round.json")"; step ab $rc
        done; done;;
    abenv) for round in 1 2; do for kv in $ABENV; do
          timeout -k 10 300 env $kv python bench.py --cpu-sample 0 --no-roofline > "$OUT/abenv_${TAG}_${kv}_$round.json" 2>/dev/null
          rc=$?; echo "$kv: $(grep -o 'ms_per_step": [0-9.]*' "$OUT/abenv_${TAG}_${kv}_$round.json")"; step abenv $rc
        done; done;;
    sq) bash scripts/sq_passes.sh "$TAG" > "$OUT/sq_$TAG.log" 2>&1; rc=$?; tail -3 "$OUT/sq_$TAG.log"; step sq $rc
          python scripts/sq_ratios.py "$OUT/pmc_$TAG" --top 30 > "$OUT/sq_ratios_$TAG.md"; head -32 "$OUT/sq_ratios_$TAG.md";;
    file) timeout -k 10 300 $PYT $TESTFILE > "$OUT/tests_${TAG}_file.log" 2>&1
          rc=$?; tail -2 "$OUT/tests_${TAG}_file.log"; step file $rc;;
    suite) timeout -k 10 900 $PYT tests -m gpu > "$OUT/tests_${TAG}.log" 2>&1
          rc=$?; tail -2 "$OUT/tests_${TAG}.log"; step suite $rc;;
    *) echo "unknown step $s"; exit 2;;
  esac
done
