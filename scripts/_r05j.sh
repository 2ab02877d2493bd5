set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pw_stream_bf16.py tests/test_gpu_pw_bwd_fused.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "fused" > $OUT/tests_r05j_bf16f.log 2>&1; rc=$?; tail -15 $OUT/tests_r05j_bf16f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_fullsize.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05j_bf16.log 2>&1; rc=$?; tail -15 $OUT/tests_r05j_bf16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_step.py --config 5 --knob 20:2 --knob 20:1 --rounds 3 --steps 20 > $OUT/ab_r05j_c5.txt 2>&1; rc=$?; tail -4 $OUT/ab_r05j_c5.txt; exit $rc
