set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u scripts/host_overhead.py --config 3 --steps 20 --profile > $OUT/host_r05s_c3.txt 2>&1; rc=$?; head -30 $OUT/host_r05s_c3.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/host_overhead.py --config 5 --steps 20 > $OUT/host_r05s_c5.txt 2>&1; rc=$?; head -3 $OUT/host_r05s_c5.txt; exit $rc
