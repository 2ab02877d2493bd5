#!/bin/bash
# Round-4 experiments (each under its own time limit): the deep weight gradient on a subset of the CUs
# (config 3 step A/B, knob 12 off / on, DORKNET_PWD_WGRAD_CUS), and fewer deep walkers for small pixel
# counts (DORKNET_PWD_MIN_TILES, standalone kernels).  Usage: bash scripts/r04_exp.sh TAG
set -u
TAG=$1
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
for cus in 128 64; do
  DORKNET_PWD_WGRAD_CUS=$cus timeout -k 10 300 python -u scripts/ab_step.py --knob 12:0 --knob 12:1 --rounds 3 --steps 10 \
      2>/dev/null | grep knob | sed "s/^/wgrad_cus=$cus /" | tee -a "$OUT/exp_$TAG.txt"
  rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || { echo "rc=$rc"; exit "$rc"; }
done
for mt in 0 10; do
  DORKNET_PWD_MIN_TILES=$mt timeout -k 10 200 python -u scripts/pwd16_bench.py --only fwd 2>/dev/null \
      | sed "s/^/min_tiles=$mt bf16 /" | tee -a "$OUT/exp_$TAG.txt"
  rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || { echo "rc=$rc"; exit "$rc"; }
  DORKNET_PWD_MIN_TILES=$mt timeout -k 10 200 python -u scripts/pwd_bench.py --deep 1 --only fwd 2>/dev/null \
      | sed "s/^/min_tiles=$mt fp32 /" | tee -a "$OUT/exp_$TAG.txt"
  rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || { echo "rc=$rc"; exit "$rc"; }
done
