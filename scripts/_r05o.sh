set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dw_bwd_cols.py tests/test_gpu_dw_bwd_s2.py tests/test_gpu_bn_on_load.py tests/test_gpu_fold.py tests/test_gpu_join_fwd.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05o.log 2>&1; rc=$?; tail -3 $OUT/tests_r05o.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05o_full.log 2>&1; rc=$?; tail -3 $OUT/tests_r05o_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_step.py --config 3 --knob 21:1 --knob 21:2 --rounds 3 --steps 20 > $OUT/ab_r05o_c3.txt 2>&1; rc=$?; tail -3 $OUT/ab_r05o_c3.txt; exit $rc
