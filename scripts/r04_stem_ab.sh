#!/bin/bash
# Same-box A/B of the narrow stem kernels: dorknet_amd/lib/libdorknet_hip_base.so (baseline build)
# against libdorknet_hip.so, scripts/stem_bench.py alternating ROUNDS times; then a FETCH_SIZE and a
# WRITE_SIZE pass (one counter each) per build.  Usage: bash scripts/r04_stem_ab.sh TAG [ROUNDS]
set -u
TAG=$1; ROUNDS=${2:-3}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
B=$ROOT/dorknet_amd/lib/libdorknet_hip_base.so; N=$ROOT/dorknet_amd/lib/libdorknet_hip.so
for r in $(seq 1 "$ROUNDS"); do
  for L in base new; do
    if [ $L = base ]; then P=$B; else P=$N; fi
    DORKNET_HIP_LIB=$P timeout -k 10 120 python -u scripts/stem_bench.py --only narrow 2>/dev/null | sed "s/^/$L: /"
    rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || { echo "rc=$rc"; exit "$rc"; }
  done
done | tee "$OUT/stem_ab_$TAG.txt"
cd /tmp && export TMPDIR=/tmp
for L in base new; do
  if [ $L = base ]; then P=$B; else P=$N; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    DORKNET_HIP_LIB=$P timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -f csv -d "$OUT/stem_pmc_${L}_${C}_$TAG" -o run \
        -- python3 "$ROOT/scripts/stem_bench.py" --only narrow > "$OUT/stem_pmc_${L}_${C}_$TAG.log" 2>&1
    rc=$?; echo "pmc $L $C rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"
  done
done
