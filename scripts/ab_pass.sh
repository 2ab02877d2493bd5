#!/bin/bash
# GPU check of a library change: the given GPU test files, then scripts/ab_builds.sh (the baseline build
# dorknet_amd/lib/libdorknet_hip_base.so against the current one) for each config, ROUNDS rounds.
# Usage (gpurun): bash scripts/ab_pass.sh TAG ROUNDS "CONFIGS" test_file ...
set -u
TAG=$1; ROUNDS=$2; CONFIGS=$3; shift 3
OUT=gpurun_out; mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > $OUT/tests_$TAG.log 2>&1
  rc=$?; tail -3 $OUT/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for c in $CONFIGS; do
  bash scripts/ab_builds.sh "$c" "$ROUNDS" > $OUT/ab_${TAG}_c$c.txt 2>&1; rc=$?; cat $OUT/ab_${TAG}_c$c.txt
  [ $rc -eq 0 ] || exit $rc
done
