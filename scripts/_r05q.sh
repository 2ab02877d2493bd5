set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05q.log 2>&1; rc=$?; tail -4 $OUT/tests_r05q.log; exit $rc
