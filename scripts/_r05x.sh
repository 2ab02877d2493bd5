set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
CFG=${1:-3}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$ROOT/$OUT/prof_r05y_c$CFG" -o bench -- \
    python "$ROOT/bench.py" --config $CFG --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$ROOT/$OUT/prof_r05y_c$CFG.json" 2> "$ROOT/$OUT/prof_r05y_c$CFG.err"
rc=$?; echo rocprof $rc; [ $rc -eq 0 ] || exit $rc
cd "$ROOT" && python scripts/gap_summary.py $OUT/prof_r05y_c$CFG --list > $OUT/gaps_r05y_c$CFG.txt; rc=$?; cat $OUT/gaps_r05y_c$CFG.txt; exit $rc
