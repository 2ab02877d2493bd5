#!/bin/bash
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r02f}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pw_stream.py tests/test_gpu_pw_bwd_fused.py tests/test_gpu_network.py tests/test_gpu_layers.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > "$OUT/tests_pws_$TAG.log" 2>&1
rc=$?; tail -4 "$OUT/tests_pws_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/pws_bench.py > "$OUT/pws_$TAG.txt" 2>&1
rc=$?; grep -v amdgpu.ids "$OUT/pws_$TAG.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-sample 0 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cat "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
