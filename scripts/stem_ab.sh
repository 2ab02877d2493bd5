#!/bin/bash
# A/B of the stem kernels (scripts/stem_bench.py --only narrow) between dorknet_amd/lib/libdorknet_hip_base.so and
# the current build, alternating.  Usage (gpurun): bash scripts/stem_ab.sh [ROUNDS]
set -u
for r in $(seq 1 "${1:-2}"); do for L in base new; do
  if [ $L = base ]; then P=dorknet_amd/lib/libdorknet_hip_base.so; else P=dorknet_amd/lib/libdorknet_hip.so; fi
  DORKNET_HIP_LIB=$(pwd)/$P timeout -k 10 120 python scripts/stem_bench.py --only narrow 2>/dev/null | sed "s/^/$L: /"
  rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || exit "$rc"
done; done
