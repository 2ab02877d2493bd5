set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
bash scripts/sq_passes.sh r05h_c5 --config 5 --steps 2 --warmup 1 --no-roofline --cpu-sample 0 || exit $?
python scripts/sq_ratios.py gpurun_out/pmc_r05h_c5 --top 30 > $OUT/r05h_sq_ratios_c5.md 2>&1; head -34 $OUT/r05h_sq_ratios_c5.md
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/prof5_r05h" -o bench -- python "$ROOT/bench.py" --config 5 --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$ROOT/$OUT/prof5_bench_r05h.json" 2> "$ROOT/$OUT/prof5_r05h.err" || exit $?
cd $ROOT; python scripts/prof_summary.py $OUT/prof5_r05h --steps 6 > $OUT/kstats5_r05h.md; head -40 $OUT/kstats5_r05h.md
timeout -k 10 400 python bench.py --config 5 > $OUT/bench5_r05h.json 2> $OUT/bench5_r05h.err; rc=$?; cut -c1-800 $OUT/bench5_r05h.json; exit $rc
