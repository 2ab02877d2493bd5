#!/bin/bash
# bench.py itself under two settings of an environment switch, alternating (one process per run).
# Usage (gpurun): bash scripts/bench_env_ab.sh CONFIG ROUNDS NAME VALUE1 VALUE2 ...
set -u
CFG=$1; ROUNDS=$2; NAME=$3; shift 3
for r in $(seq 1 "$ROUNDS"); do
  for V in "$@"; do
    out=$(env "$NAME=$V" timeout -k 10 300 python bench.py --config "$CFG" --cpu-sample 0 --no-roofline 2>/dev/null) || exit 1
    echo "config $CFG $NAME=$V: $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", d["value"], d["unit"])')"
  done
done
