set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dw_bwd_s2.py tests/test_gpu_network.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05p.log 2>&1; rc=$?; tail -3 $OUT/tests_r05p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "joins or res4_res6" > $OUT/tests_r05p_full.log 2>&1; rc=$?; tail -3 $OUT/tests_r05p_full.log; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 3 DORKNET_DW_S2_FUSED 0 1 > $OUT/ab_r05p_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05p_c3.txt; exit $rc
