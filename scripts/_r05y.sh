set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_dp.py tests/test_gpu_network.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05y.log 2>&1; rc=$?; tail -3 $OUT/tests_r05y.log; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 2 DORKNET_WGRAD_FLUSH_LAST 0 1 2 > $OUT/ab_r05y_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05y_c3.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 5 2 DORKNET_WGRAD_FLUSH_LAST 0 1 2 > $OUT/ab_r05y_c5.txt 2>&1; rc=$?; cat $OUT/ab_r05y_c5.txt; exit $rc
