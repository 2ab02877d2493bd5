#!/bin/bash
# A/B of a process-level environment knob (read once per process, so one process per setting), alternating.
# Usage (gpurun): bash scripts/env_ab.sh CONFIG ROUNDS NAME VALUE1 VALUE2 ...
set -u
CFG=$1; ROUNDS=$2; NAME=$3; shift 3
for r in $(seq 1 "$ROUNDS"); do
  for V in "$@"; do
    env "$NAME=$V" timeout -k 10 200 python scripts/ab_step.py --config "$CFG" --knob 2:-1 --rounds 1 --steps 20 \
        2>/dev/null | grep knob | sed "s/^/config $CFG $NAME=$V: /"
    rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || exit "$rc"
  done
done
