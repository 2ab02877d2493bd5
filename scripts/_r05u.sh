set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_dp.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05u.log 2>&1; rc=$?; tail -3 $OUT/tests_r05u.log; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 2 DORKNET_WGRAD_FLUSH_EVERY 1 4 8 60 > $OUT/ab_r05u2_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05u2_c3.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 5 2 DORKNET_WGRAD_FLUSH_EVERY 1 4 8 60 > $OUT/ab_r05u2_c5.txt 2>&1; rc=$?; cat $OUT/ab_r05u2_c5.txt; exit $rc
