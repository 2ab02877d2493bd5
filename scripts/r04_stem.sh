#!/bin/bash
# Round-4 stem + deep-wgrad pass: the narrow-stem tests, scripts/stem_bench.py, and a kernel trace of
# the deep pointwise weight gradient (pwd_bench --only wgrad).  Each step under its own limit.
set -u
TAG=$1
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn_on_load.py tests/test_gpu_fold.py tests/test_gpu_fullsize.py \
    tests/test_gpu_layers.py -k "narrow or stem" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/stem_tests_$TAG.log" 2>&1
rc=$?; tail -3 "$OUT/stem_tests_$TAG.log"; step tests $rc
timeout -k 10 200 python -u scripts/stem_bench.py --only narrow > "$OUT/stem_bench_$TAG.txt" 2>&1
rc=$?; cat "$OUT/stem_bench_$TAG.txt"; step stem_bench $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_wg_$TAG" -o run -- python3 "$OLDPWD/scripts/pwd_bench.py" --only wgrad \
    > "$OUT/prof_wg_$TAG.log" 2>&1
rc=$?; tail -12 "$OUT/prof_wg_$TAG.log"; step prof $rc
