set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_join_fwd.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05d_join.log 2>&1; rc=$?; tail -15 $OUT/tests_r05d_join.log; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 3 DORKNET_FUSE_JOIN_FWD 1 0 > $OUT/ab_r05d_joinfwd.txt 2>&1; rc=$?; cat $OUT/ab_r05d_joinfwd.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05d.log 2>&1; rc=$?; tail -3 $OUT/tests_r05d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/pwd_bench.py --only bwd > $OUT/pwd_bench_r05d.txt 2>&1; rc=$?; cat $OUT/pwd_bench_r05d.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/prof_r05d" -o bench -- python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$ROOT/$OUT/prof_bench_r05d.json" 2> "$ROOT/$OUT/prof_r05d.err"; rc=$?; [ $rc -eq 0 ] || exit $rc
cd $ROOT; python scripts/prof_summary.py $OUT/prof_r05d --steps 6 > $OUT/kstats_r05d.md; head -45 $OUT/kstats_r05d.md
timeout -k 10 400 python bench.py --cpu-sample 0 > $OUT/bench_r05d.json 2> $OUT/bench_r05d.err; rc=$?; cut -c1-600 $OUT/bench_r05d.json; exit $rc
