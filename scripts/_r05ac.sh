set -u
OUT=gpurun_out; mkdir -p $OUT; ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_dw_bwd_cols.py tests/test_gpu_bf16.py tests/test_gpu_bf16_fullsize.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_r05ac.log 2>&1; rc=$?; tail -3 $OUT/tests_r05ac.log; [ $rc -eq 0 ] || exit $rc
for L in base new; do
  if [ $L = base ]; then P=$ROOT/dorknet_amd/lib/libdorknet_hip_base.so; else P=$ROOT/dorknet_amd/lib/libdorknet_hip.so; fi
  DORKNET_HIP_LIB=$P timeout -k 10 200 python scripts/dwb_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/bf16 $L: /"
done > $OUT/dwb_r05ac.txt; rc=$?; cat $OUT/dwb_r05ac.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_builds.sh 5 4 > $OUT/ab_r05ac_c5.txt 2>&1; rc=$?; cat $OUT/ab_r05ac_c5.txt; exit $rc
