set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
DORKNET_WGRAD_FLUSH_EVERY=60 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$ROOT/$OUT/prof_r05v" -o bench -- \
    python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$ROOT/$OUT/prof_r05v.json" 2> "$ROOT/$OUT/prof_r05v.err"
rc=$?; echo rocprof $rc; [ $rc -eq 0 ] || exit $rc
cd "$ROOT" && python scripts/gap_summary.py $OUT/prof_r05v
