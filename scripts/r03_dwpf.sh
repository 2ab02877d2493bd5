#!/bin/bash
# bf16 fused depthwise backward with packed two-row prefetch: tests, cross-build A/B on configs 5 and 3,
# host overhead, config 1 bench line.
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_bn_on_load.py tests/test_gpu_bf16.py tests/test_gpu_bf16_fullsize.py \
    tests/test_gpu_network.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_r03m.log" 2>&1
rc=$?; tail -3 "$OUT/tests_r03m.log"; step tests $rc
bash scripts/ab_builds.sh 5 3 > "$OUT/abb5_r03m.txt" 2>&1
rc=$?; cat "$OUT/abb5_r03m.txt"; step abb5 $rc
bash scripts/ab_builds.sh 3 3 > "$OUT/abb3_r03m.txt" 2>&1
rc=$?; cat "$OUT/abb3_r03m.txt"; step abb3 $rc
timeout -k 10 200 python scripts/host_overhead.py --config 5 --steps 10 --profile > "$OUT/host5_r03m.txt" 2>&1
step host5 $?
timeout -k 10 200 python scripts/host_overhead.py --config 3 --steps 10 > "$OUT/host3_r03m.txt" 2>&1
rc=$?; head -3 "$OUT/host3_r03m.txt"; step host3 $rc
timeout -k 10 200 python bench.py --config 1 > "$OUT/bench1_r03m.json" 2> "$OUT/bench1_r03m.err"
rc=$?; cut -c1-300 "$OUT/bench1_r03m.json"; step bench1 $rc
