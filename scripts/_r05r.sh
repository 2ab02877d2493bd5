set -u
OUT=gpurun_out; mkdir -p $OUT
bash scripts/env_ab.sh 3 3 DORKNET_WGRAD_MAIN_K 0 512 256 > $OUT/ab_r05r_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05r_c3.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 5 2 DORKNET_WGRAD_MAIN_K 0 512 > $OUT/ab_r05r_c5.txt 2>&1; rc=$?; cat $OUT/ab_r05r_c5.txt; exit $rc
