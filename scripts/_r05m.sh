set -u
OUT=gpurun_out; mkdir -p $OUT
bash scripts/sq_cmd.sh r05m scripts/dwb_bench.py --hw 56 > $OUT/sq_r05m.txt 2>&1; rc=$?; tail -8 $OUT/sq_r05m.txt; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_table.py gpurun_out/pmc_r05m > $OUT/sq_r05m_table.txt 2>&1; grep -A2 "dw_bwd" $OUT/sq_r05m_table.txt | head -20
