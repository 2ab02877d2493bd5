set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 300 python -u scripts/ab_step.py --config 5 --knob 21:1 --knob 21:2 --rounds 3 --steps 20 > $OUT/ab_r05l_c5.txt 2>&1; rc=$?; tail -3 $OUT/ab_r05l_c5.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/prof5_r05l" -o bench -- \
    python "$ROOT/bench.py" --config 5 --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$ROOT/$OUT/prof5_r05l.json" 2> "$ROOT/$OUT/prof5_r05l.err"
rc=$?; echo rocprof $rc; [ $rc -eq 0 ] || exit $rc
cd "$ROOT" && python scripts/prof_summary.py $OUT/prof5_r05l --steps 5 > $OUT/r05l_config5_kernel_stats.md; head -40 $OUT/r05l_config5_kernel_stats.md
