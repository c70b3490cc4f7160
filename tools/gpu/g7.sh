# staggered 8-phase grouped GEMM; MLA decode kernel-time profile; MoE/conv/misc tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof7
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/g7_$name.log 2>&1; local rc=$?;
         echo "$name rc=$rc"; if [ $rc -ge 124 ]; then tail -30 gpurun_out/g7_$name.log; exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_moe_gpu.py tests/test_conv_gpu.py tests/test_misc_gpu.py tests/test_mla_decode_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
tail -4 gpurun_out/g7_tests.log
grep -E "FAIL|Error|assert" gpurun_out/g7_tests.log | head -20
step moe 300 python -u tools/bench_moe.py
cat gpurun_out/g7_moe.log
step mlaprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7/mla -o mla --output-format csv -- python tools/bench_mla_decode.py
cat gpurun_out/g7_mlaprof.log | grep '^{'
step moeprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7/moe -o moe --output-format csv -- python tools/bench_moe.py
