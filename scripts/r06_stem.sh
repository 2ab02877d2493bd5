#!/bin/bash
# stem kernels: their GPU tests, then the config-3 profile and bench (round 6)
set -u
OUT=gpurun_out; mkdir -p $OUT; TAG=$1
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_fullsize.py tests/test_gpu_bn_on_load.py tests/test_gpu_fold.py -x -q -k "narrow or stem or conv0 or conv" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_${TAG}_stem.log 2>&1
rc=$?; tail -2 $OUT/tests_${TAG}_stem.log; step stemtests $rc
bash scripts/r06_pass.sh $TAG prof bench
