set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
DORKNET_ASYNC_WGRAD=0 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$ROOT/$OUT/prof_r05t_sync" -o bench -- \
    python "$ROOT/bench.py" --steps 5 --warmup 2 --cpu-sample 0 --no-roofline > "$ROOT/$OUT/prof_r05t_sync.json" 2> "$ROOT/$OUT/prof_r05t_sync.err"
rc=$?; echo rocprof $rc; [ $rc -eq 0 ] || exit $rc
cd "$ROOT" && python scripts/gap_summary.py $OUT/prof_r05t_sync
bash scripts/env_ab.sh 3 2 DORKNET_ASYNC_WGRAD 1 0 > $OUT/ab_r05t_c3.txt 2>&1; rc=$?; cat $OUT/ab_r05t_c3.txt; exit $rc
