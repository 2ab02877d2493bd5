set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pw_deep.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k fused > $OUT/tests_r05b_fused.log 2>&1; rc=$?; tail -3 $OUT/tests_r05b_fused.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_step.py --knob 14:0 --knob 14:1 --rounds 3 --steps 20 > $OUT/ab_r05b.txt 2>&1; rc=$?; cat $OUT/ab_r05b.txt | tail -8; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pass.sh r05b --smoke --configs "3"
