#!/bin/bash
# A/B of two builds of the library on one box: dorknet_amd/lib/libdorknet_hip_base.so (the baseline)
# against dorknet_amd/lib/libdorknet_hip.so, alternating, for a config.  Usage: bash scripts/ab_builds.sh CONFIG ROUNDS
# BASE_ENV (optional, e.g. "DORKNET_DW_STRIDED_BN=0"): environment for the baseline runs, for Python paths the
# baseline build lacks.
set -u
CFG=${1:-3}; ROUNDS=${2:-3}
ROOT=$(pwd); BASE=$ROOT/dorknet_amd/lib/libdorknet_hip_base.so; NEW=$ROOT/dorknet_amd/lib/libdorknet_hip.so
for r in $(seq 1 "$ROUNDS"); do
  for L in base new; do
    if [ $L = base ]; then P=$BASE; E=${BASE_ENV:-DORKNET_AB_BASE=1}; else P=$NEW; E=DORKNET_AB_BASE=0; fi
    env "$E" DORKNET_HIP_LIB=$P timeout -k 10 200 python scripts/ab_step.py --config "$CFG" --knob 2:-1 --rounds 1 --steps 10 \
        2>/dev/null | grep knob | sed "s/^/config $CFG $L: /"
    rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || exit "$rc"
  done
done
