# grouped GEMV decode path, vectorised dropout, wave-per-row KD, implicit-GEMM conv; profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof5
export TMPDIR=/tmp
# run one GPU step; stop the whole script on a timeout / signal / abort (rc >= 124)
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/g5_$name.log 2>&1; local rc=$?;
         echo "$name rc=$rc"; if [ $rc -ge 124 ]; then tail -30 gpurun_out/g5_$name.log; exit $rc; fi; }
step tests 500 python -u -m pytest tests/test_conv_gpu.py tests/test_misc_gpu.py tests/test_moe_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
tail -5 gpurun_out/g5_tests.log
grep -E "FAIL|Error" gpurun_out/g5_tests.log | head -20
step conv 300 python -u tools/bench_conv.py
cat gpurun_out/g5_conv.log
step kern 300 python -u tools/bench_kernels.py
cat gpurun_out/g5_kern.log
step moe 300 python -u tools/bench_moe.py
tail -12 gpurun_out/g5_moe.log
step dec 300 python -u bench/decode.py --model dsv3_style --batch 1 --prompt 1024 --new 64
step decg 300 python -u bench/decode.py --model dsv3_style --batch 1 --prompt 1024 --new 64 --graph
grep -h '^{' gpurun_out/g5_dec.log gpurun_out/g5_decg.log
step profdec 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5/dec -o dec --output-format csv -- python bench/decode.py --model dsv3_style --batch 1 --prompt 1024 --new 32 --graph
find gpurun_out/prof5 -name "*stats*"
