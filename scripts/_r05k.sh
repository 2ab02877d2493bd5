set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dw_bwd_cols.py tests/test_gpu_bf16.py tests/test_gpu_bn_on_load.py tests/test_gpu_fold.py tests/test_gpu_join_fwd.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05k.log 2>&1; rc=$?; tail -3 $OUT/tests_r05k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/dwb_bench.py > $OUT/dwb_r05k.txt 2>&1; rc=$?; cat $OUT/dwb_r05k.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/dwb_bench.py --f32 > $OUT/dwb_r05k_f32.txt 2>&1; rc=$?; cat $OUT/dwb_r05k_f32.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05k_full.log 2>&1; rc=$?; tail -2 $OUT/tests_r05k_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_step.py --config 5 --knob 21:1 --knob 21:2 --rounds 3 --steps 20 > $OUT/ab_r05k_c5.txt 2>&1; rc=$?; tail -3 $OUT/ab_r05k_c5.txt; exit $rc
