#!/bin/bash
# Round-4 closing check on the final library: the -m gpu suite, smoke(), the config-5 line (value
# over uninstrumented steps) and config 3 with and without the in-region event records.
# Usage (gpurun): bash scripts/r04_check.sh TAG
set -u
TAG=${1:-check}
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_$TAG.log" 2>&1
rc=$?; tail -2 "$OUT/tests_$TAG.log"; step tests $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; tail -1 "$OUT/smoke_$TAG.log"; step smoke $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --config 5 > "$OUT/bench5_${TAG}_$i.json" 2>/dev/null; step bench5 $?
  timeout -k 10 300 python bench.py --cpu-sample 0 > "$OUT/bench_${TAG}_$i.json" 2>/dev/null; step bench3 $?
  timeout -k 10 300 python bench.py --cpu-sample 0 --no-roofline > "$OUT/bench_${TAG}_plain_$i.json" 2>/dev/null; step bench3p $?
done
for f in "$OUT"/bench*_"$TAG"_*.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['value'], r.get('kernel'), r.get('frac'))" "$f"
done
