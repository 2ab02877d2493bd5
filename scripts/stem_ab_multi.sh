#!/bin/bash
# A/B of the stem kernels (scripts/stem_bench.py --only narrow) across builds dorknet_amd/lib/libdorknet_hip_<TAG>.so,
# alternating.  Usage (gpurun): bash scripts/stem_ab_multi.sh ROUNDS TAG1 TAG2 ...
set -u
ROUNDS=$1; shift
for r in $(seq 1 "$ROUNDS"); do for L in "$@"; do
  DORKNET_HIP_LIB=$(pwd)/dorknet_amd/lib/libdorknet_hip_$L.so timeout -k 10 120 python scripts/stem_bench.py --only narrow \
      2>/dev/null | sed "s/^/$L: /"
  rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || exit "$rc"
done; done
