#!/bin/bash
set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 400 python -u scripts/diag_fullsize.py 16 256 > "$OUT/diag_fullsize.txt" 2>&1
rc=$?; cat "$OUT/diag_fullsize.txt" | grep -v Warn; echo "diag rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_probe.sh r02a
