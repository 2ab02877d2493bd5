#!/bin/bash
# bench.py A/B of two library builds on one box (libdorknet_hip_base.so vs libdorknet_hip.so),
# alternating.  Usage: bash scripts/ab_bench.sh CONFIG ROUNDS
set -u
CFG=${1:-5}; ROUNDS=${2:-2}
L=$(pwd)/dorknet_amd/lib
for r in $(seq 1 "$ROUNDS"); do
  for V in base new; do
    if [ $V = new ]; then P=$L/libdorknet_hip.so; else P=$L/libdorknet_hip_base.so; fi
    DORKNET_HIP_LIB=$P timeout -k 10 300 python bench.py --config "$CFG" --cpu-sample 0 --no-roofline 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('config $CFG $V', d['ms_per_step'], d['value'])"
    rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || exit "$rc"
  done
done
