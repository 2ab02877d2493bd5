#!/bin/bash
# Depthwise-forward ring window A/B: the -m gpu suite on the new build, then the forward per shape
# (scripts/dw_fwd_seg.py, fp32 config 3 / bf16 config 5 shapes) for the baseline and the new build,
# then step A/Bs (scripts/ab_builds.sh) for configs 5 and 3.
# Usage (gpurun): bash scripts/r04_dw.sh TAG [--skip-tests]
set -u
TAG=${1:-dw}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
if [ "${2:-}" != "--skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
      > "$OUT/tests_$TAG.log" 2>&1
  rc=$?; tail -3 "$OUT/tests_$TAG.log"; step tests $rc
fi
for L in base new; do
  if [ $L = base ]; then P=$ROOT/dorknet_amd/lib/libdorknet_hip_base.so; else P=$ROOT/dorknet_amd/lib/libdorknet_hip.so; fi
  for H in "" --bf16; do
    DW_SEGS=-1 DORKNET_HIP_LIB=$P timeout -k 10 120 python scripts/dw_fwd_seg.py $H 2>/dev/null | sed "s/^/$L /" \
        | tee -a "$OUT/dwfwd_$TAG.txt"
    step "dwfwd $L $H" ${PIPESTATUS[0]}
  done
done
bash scripts/ab_builds.sh 5 2 | tee -a "$OUT/ab_$TAG.txt"; step ab5 ${PIPESTATUS[0]}
bash scripts/ab_builds.sh 3 2 | tee -a "$OUT/ab_$TAG.txt"; step ab3 ${PIPESTATUS[0]}
