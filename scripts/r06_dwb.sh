#!/bin/bash
# fused depthwise backward block-target sweep at the small images (round 6)
set -u
OUT=gpurun_out; mkdir -p $OUT; TAG=$1
timeout -k 10 300 python -u scripts/dwb_bench.py --f32 --batch 256 --blocks 768,256,384,512,1024,1536,3072 > $OUT/dwb_${TAG}.txt 2>&1
rc=$?; cat $OUT/dwb_${TAG}.txt; echo "== dwb rc=$rc"; exit $rc
