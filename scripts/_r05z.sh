set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_dp.py tests/test_gpu_network.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05z.log 2>&1; rc=$?; tail -3 $OUT/tests_r05z.log; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 3 DORKNET_WGRAD_INLINE_LAST 0 1 > $OUT/ab_r05z_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05z_c3.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 5 3 DORKNET_WGRAD_INLINE_LAST 0 1 > $OUT/ab_r05z_c5.txt 2>&1; rc=$?; cat $OUT/ab_r05z_c5.txt; [ $rc -eq 0 ] || exit $rc
sed -i 's/prof_r05y_c/prof_r05z_c/g; s/gaps_r05y_c/gaps_r05z_c/g' scripts/_r05x.sh
bash scripts/_r05x.sh 5 > /dev/null && bash scripts/_r05x.sh 3 > /dev/null
