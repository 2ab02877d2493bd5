set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
bash scripts/sq_passes.sh r05g_c3 || exit $?
python scripts/sq_ratios.py gpurun_out/pmc_r05g_c3 --top 30 > $OUT/r05g_sq_ratios_c3.md 2>&1; head -40 $OUT/r05g_sq_ratios_c3.md
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-roofline"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$ROOT/$OUT/pmc3_r05g/fetch" -o run -- python $BENCH > "$ROOT/$OUT/pmc3_r05g_fetch.log" 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$ROOT/$OUT/pmc3_r05g/write" -o run -- python $BENCH > "$ROOT/$OUT/pmc3_r05g_write.log" 2>&1 || exit $?
cd $ROOT; python scripts/pmc_summary.py $OUT/pmc3_r05g/fetch $OUT/pmc3_r05g/write --out $OUT/r05g_pmc.json > $OUT/r05g_pmc_summary.txt 2>&1; head -20 $OUT/r05g_pmc_summary.txt
