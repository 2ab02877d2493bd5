#!/bin/bash
# Host-issue A/B of a Python change on one box: a copy of the tree under /tmp with the files 
# scripts/_ab_old/ (the baseline versions, placed by name under dorknet_amd/layers/) against this
# tree, alternating.  Usage (gpurun): bash scripts/host_ab.sh CONFIG ROUNDS
set -u
CFG=${1:-3}; ROUNDS=${2:-3}
ROOT=$(pwd); OLD=/tmp/host_ab_old
rm -rf "$OLD"; mkdir -p "$OLD"
cp -r "$ROOT/dorknet_amd" "$ROOT/examples" "$ROOT/scripts" "$ROOT/include" "$OLD/"
for f in "$ROOT"/scripts/_ab_old/*.py; do cp "$f" "$OLD/dorknet_amd/layers/$(basename "$f")"; done
for r in $(seq 1 "$ROUNDS"); do
  for L in old new; do
    if [ $L = old ]; then D=$OLD; else D=$ROOT; fi
    timeout -k 10 200 python "$D/scripts/host_overhead.py" --config "$CFG" --steps 30 2>/dev/null | grep "host issue" | sed "s/^/$L: /"
    rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || exit "$rc"
  done
done
