set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_pw_stream.py tests/test_gpu_pw_bwd_fused.py tests/test_gpu_pw_lattice_fused.py tests/test_gpu_network.py tests/test_gpu_fold.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05ae.log 2>&1; rc=$?; tail -3 $OUT/tests_r05ae.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_builds.sh 3 3 > $OUT/ab_r05ae_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05ae_c3.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 3 DORKNET_PWS_BWD_PF 0 1 > $OUT/ab_r05ae_pf_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05ae_pf_c3.txt; exit $rc
