#!/bin/bash
# A/B/C of three library builds on one box (libdorknet_hip_base.so, libdorknet_hip_mid.so,
# libdorknet_hip.so), alternating, for a config.  Usage: bash scripts/ab3_builds.sh CONFIG ROUNDS
set -u
CFG=${1:-3}; ROUNDS=${2:-2}
ROOT=$(pwd); L=$ROOT/dorknet_amd/lib
for r in $(seq 1 "$ROUNDS"); do
  for V in base mid new; do
    if [ $V = new ]; then P=$L/libdorknet_hip.so; else P=$L/libdorknet_hip_$V.so; fi
    DORKNET_HIP_LIB=$P timeout -k 10 200 python scripts/ab_step.py --config "$CFG" --knob 2:-1 --rounds 1 --steps 10 \
        2>/dev/null | grep knob | sed "s/^/config $CFG $V: /"
    rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || exit "$rc"
  done
done
