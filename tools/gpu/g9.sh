set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/g9_$name.log 2>&1; local rc=$?;
         echo "$name rc=$rc"; if [ $rc -ge 124 ]; then tail -30 gpurun_out/g9_$name.log; exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_moe_gpu.py tests/test_conv_gpu.py tests/test_misc_gpu.py tests/test_mla_decode_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
tail -4 gpurun_out/g9_tests.log
grep -E "FAIL|Error|assert" gpurun_out/g9_tests.log | head -20
step moe 300 python -u tools/bench_moe.py
cat gpurun_out/g9_moe.log
