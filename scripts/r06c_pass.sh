set -u
OUT=gpurun_out; mkdir -p $OUT
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then echo "stopping after rc=$2"; exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_pw_deep.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests_r06c_deep.log 2>&1
rc=$?; tail -3 $OUT/tests_r06c_deep.log; step deep $rc
timeout -k 10 300 python -u scripts/pwd_bench.py --only dgrad > $OUT/pwd_bench_r06c.txt 2>&1
rc=$?; cat $OUT/pwd_bench_r06c.txt; step pwdbench $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_network.py -x -q -s -k "training_steps" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_r06c_net.log 2>&1
rc=$?; tail -3 $OUT/tests_r06c_net.log; step net $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r06c.log 2>&1
rc=$?; tail -1 $OUT/smoke_r06c.log; step smoke $rc
timeout -k 10 400 python bench.py --cpu-sample 0 > $OUT/bench3_r06c.json 2> $OUT/bench3_r06c.err
rc=$?; cut -c1-400 $OUT/bench3_r06c.json; step bench $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_pw_deep.py > $OUT/tests_r06c.log 2>&1
rc=$?; tail -3 $OUT/tests_r06c.log; step tests $rc
