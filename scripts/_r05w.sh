set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_pw_lattice_fused.py tests/test_gpu_network.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05w.log 2>&1; rc=$?; tail -3 $OUT/tests_r05w.log; [ $rc -eq 0 ] || exit $rc
bash scripts/env_ab.sh 3 3 DORKNET_PW_LATTICE_FUSED 0 1 > $OUT/ab_r05w_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05w_c3.txt; exit $rc
