#!/bin/bash
# Host-issue check: the -m gpu suite, then scripts/host_overhead.py for configs 3 and 5 (with
# cProfile for config 3) and the config-3 bench line.  Usage (gpurun): bash scripts/r03_host.sh TAG
set -u
TAG=${1:-host}
OUT=gpurun_out; mkdir -p $OUT
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $OUT/tests_$TAG.log 2>&1
rc=$?; tail -2 $OUT/tests_$TAG.log; step tests $rc
timeout -k 10 240 python scripts/host_overhead.py --config 3 --profile > $OUT/host3_$TAG.txt 2>&1
rc=$?; sed -n 2p $OUT/host3_$TAG.txt; step host3 $rc
timeout -k 10 240 python scripts/host_overhead.py --config 5 > $OUT/host5_$TAG.txt 2>&1
rc=$?; tail -1 $OUT/host5_$TAG.txt; step host5 $rc
timeout -k 10 300 python bench.py --cpu-sample 0 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; cut -c1-300 $OUT/bench_$TAG.json; step bench $rc
