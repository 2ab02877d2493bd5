#!/bin/bash
# A/B of two builds of the library on one box: dorknet_amd/lib/libdorknet_hip_base.so (the baseline)
# against dorknet_amd/lib/libdorknet_hip.so, alternating, for a config.  Usage: bash scripts/ab_builds.sh CONFIG ROUNDS
set -u
CFG=${1:-3}; ROUNDS=${2:-3}
ROOT=$(pwd); BASE=$ROOT/dorknet_amd/lib/libdorknet_hip_base.so; NEW=$ROOT/dorknet_amd/lib/libdorknet_hip.so
for r in $(seq 1 "$ROUNDS"); do
  for L in base new; do
    if [ $L = base ]; then P=$BASE; else P=$NEW; fi
    DORKNET_HIP_LIB=$P timeout -k 10 200 python scripts/ab_step.py --config "$CFG" --knob 2:-1 --rounds 1 --steps 10 \
        2>/dev/null | grep knob | sed "s/^/config $CFG $L: /"
    rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || exit "$rc"
  done
done
