set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_join_fwd.py tests/test_gpu_pw_bwd_fused.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05f_join.log 2>&1; rc=$?; tail -4 $OUT/tests_r05f_join.log; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 4 DORKNET_FUSE_JOIN_FWD 1 0 > $OUT/ab_r05f_joinfwd.txt 2>&1; rc=$?; cat $OUT/ab_r05f_joinfwd.txt; exit $rc
