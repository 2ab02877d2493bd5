set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 200 python -u scripts/join_bench.py > $OUT/join_bench_r05e.txt 2>&1; rc=$?; cat $OUT/join_bench_r05e.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/join_bench.py --stride 2 > $OUT/join_bench2_r05e.txt 2>&1; rc=$?; cat $OUT/join_bench2_r05e.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/pwd_bench.py --only bwd > $OUT/pwd_bench_r05e.txt 2>&1; rc=$?; cat $OUT/pwd_bench_r05e.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/prof_r05e" -o bench -- python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$ROOT/$OUT/prof_bench_r05e.json" 2> "$ROOT/$OUT/prof_r05e.err"; rc=$?; [ $rc -eq 0 ] || exit $rc
cd $ROOT; python scripts/prof_summary.py $OUT/prof_r05e --steps 6 > $OUT/kstats_r05e.md; head -50 $OUT/kstats_r05e.md
