# 8-phase grouped GEMM, conv fixes, KD lane kernel, MLA split heuristic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof6
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/g6_$name.log 2>&1; local rc=$?;
         echo "$name rc=$rc"; if [ $rc -ge 124 ]; then tail -30 gpurun_out/g6_$name.log; exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_moe_gpu.py tests/test_conv_gpu.py tests/test_misc_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
tail -4 gpurun_out/g6_tests.log
grep -E "FAIL|Error|assert" gpurun_out/g6_tests.log | head -20
step moe 300 python -u tools/bench_moe.py
cat gpurun_out/g6_moe.log
step mla 300 python -u tools/bench_mla_decode.py
cat gpurun_out/g6_mla.log
step conv 300 python -u tools/bench_conv.py
cat gpurun_out/g6_conv.log
step kern 300 python -u tools/bench_kernels.py --only kd_loss_grad_65536x10_bf16,kd_loss_grad_16384x1000,kd_loss_16384x1000
cat gpurun_out/g6_kern.log
step dsv3 400 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --steps 4 --warmup 2
grep '^{' gpurun_out/g6_dsv3.log
