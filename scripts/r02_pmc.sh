#!/bin/bash
# Round-2 counter evidence for the config-3 step, plus config 2 / 5 profiles.
# Usage (gpurun): bash scripts/r02_pmc.sh TAG
#   p1: FETCH_SIZE, p2: WRITE_SIZE (HBM traffic, scripts/pmc_summary.py)
#   p3: SQ instruction / MFMA-busy / LDS counters (scripts/pmc_table.py)
#   config 2: bench line + rocprofv3 kernel stats; config 5: bench line
set -u
TAG=${1:-pmc}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT/pmc_$TAG"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
BENCH="$ROOT/bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-roofline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d "$OUT/pmc_$TAG/fetch" -o run -- python $BENCH \
    > "$OUT/pmc_$TAG/fetch.log" 2>&1
step fetch $?
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$OUT/pmc_$TAG/write" -o run -- python $BENCH \
    > "$OUT/pmc_$TAG/write.log" 2>&1
step write $?
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace -f csv -d "$OUT/pmc_$TAG/p3" -o p -- python $BENCH > "$OUT/pmc_$TAG/p3.log" 2>&1
step sq $?
cd "$ROOT"
python scripts/pmc_summary.py "$OUT/pmc_$TAG/fetch" "$OUT/pmc_$TAG/write" --out "$OUT/${TAG}_pmc.json" \
    > "$OUT/${TAG}_pmc_summary.txt" 2>&1
step summary $?
python scripts/pmc_table.py "$OUT/pmc_$TAG" > "$OUT/${TAG}_sq_table.txt" 2>&1
step table $?
timeout -k 10 200 python bench.py --config 2 --steps 20 --warmup 5 --cpu-sample 0 > "$OUT/${TAG}_config2_bench.json" \
    2> "$OUT/${TAG}_config2.err"
step config2 $?
timeout -k 10 200 python bench.py --config 5 --steps 10 --warmup 3 --cpu-sample 0 > "$OUT/${TAG}_config5_bench.json" \
    2> "$OUT/${TAG}_config5.err"
step config5 $?
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_${TAG}_c2" -o c2 -- \
    python "$ROOT/bench.py" --config 2 --steps 10 --warmup 3 --cpu-sample 0 --no-roofline > "$OUT/${TAG}_c2_prof.log" 2>&1
step c2prof $?
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace -f csv -d "$OUT/pmc_${TAG}_c2/p1" -o p -- python "$ROOT/bench.py" --config 2 --steps 3 --warmup 1 \
    --cpu-sample 0 --no-roofline > "$OUT/${TAG}_c2_pmc.log" 2>&1
step c2pmc $?
cd "$ROOT" && python scripts/pmc_table.py "$OUT/pmc_${TAG}_c2" > "$OUT/${TAG}_c2_sq_table.txt" 2>&1
cat "$OUT/${TAG}_config2_bench.json" "$OUT/${TAG}_config5_bench.json"
