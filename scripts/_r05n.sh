set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dw_bwd_s2.py tests/test_gpu_dw_bwd_cols.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05n.log 2>&1; rc=$?; tail -3 $OUT/tests_r05n.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_fullsize.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05n_full.log 2>&1; rc=$?; tail -2 $OUT/tests_r05n_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/dwb_bench.py --f32 > $OUT/dwb_r05n_f32.txt 2>&1; rc=$?; cat $OUT/dwb_r05n_f32.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 5 3 DORKNET_DW_S2_FUSED 0 1 > $OUT/ab_r05n_c5.txt 2>&1; rc=$?; cat $OUT/ab_r05n_c5.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 2 DORKNET_DW_S2_FUSED 0 1 > $OUT/ab_r05n_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05n_c3.txt; exit $rc
