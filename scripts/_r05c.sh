set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05c.log 2>&1; rc=$?; tail -3 $OUT/tests_r05c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/pwd_bench.py --only bwd > $OUT/pwd_bench_r05c.txt 2>&1; rc=$?; cat $OUT/pwd_bench_r05c.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/prof_r05c" -o bench -- python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$ROOT/$OUT/prof_bench_r05c.json" 2> "$ROOT/$OUT/prof_r05c.err"; rc=$?; [ $rc -eq 0 ] || exit $rc
cd $ROOT; python scripts/prof_summary.py $OUT/prof_r05c --steps 6 > $OUT/kstats_r05c.md; head -30 $OUT/kstats_r05c.md
timeout -k 10 400 python bench.py --cpu-sample 0 > $OUT/bench_r05c.json 2> $OUT/bench_r05c.err; rc=$?; cut -c1-600 $OUT/bench_r05c.json; exit $rc
