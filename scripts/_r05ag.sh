set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 700 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_bf16_fullsize.py tests/test_gpu_join_fwd.py tests/test_gpu_layers.py tests/test_gpu_fold.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05ag.log 2>&1; rc=$?; tail -3 $OUT/tests_r05ag.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_builds.sh 5 4 > $OUT/ab_r05ag_c5.txt 2>&1; rc=$?; cat $OUT/ab_r05ag_c5.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_builds.sh 3 3 > $OUT/ab_r05ag_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05ag_c3.txt; exit $rc
