#!/bin/bash
# Stem kernel timings + SQ counters (scripts/stem_bench.py).  Usage (gpurun): bash scripts/stem_pmc.sh TAG
set -u
TAG=${1:-stem}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_$TAG; mkdir -p "$OUT"
timeout -k 10 120 python scripts/stem_bench.py > "$OUT/times.txt" 2>&1; rc=$?; cat "$OUT/times.txt"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -f csv -d "$OUT/p1" -o p -- \
    python "$ROOT/scripts/stem_bench.py" > "$OUT/p1.log" 2>&1; rc=$?; echo "pmc1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD \
    SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_WAVES --kernel-trace -f csv -d "$OUT/p2" -o p -- \
    python "$ROOT/scripts/stem_bench.py" > "$OUT/p2.log" 2>&1; rc=$?; echo "pmc2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT" && python scripts/pmc_table.py "$OUT" > "$OUT/table.txt" 2>&1 && grep -A1 "nar::\|igemm" "$OUT/table.txt" | cut -c1-600
