#!/bin/bash
# SQ counter passes (each its own rocprofv3 run, <= 8 SQ counters) over any python command, then the
# per-kernel ratio table (scripts/sq_ratios.py).
# Usage (gpurun): bash scripts/sq_cmd.sh TAG script.py [args...]
set -u
TAG=$1; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace -f csv -d "$OUT/p$i" -o p -- python "$ROOT/$@" \
      > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$ROOT" && python scripts/sq_ratios.py "$OUT" > "$OUT/ratios.md" && cat "$OUT/ratios.md"
