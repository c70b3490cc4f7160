set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_attention_dropout_gpu.py tests/test_kernels_gpu.py tests/test_parallel_tp_ep_gpu.py tests/test_xent_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g3_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/g3_pytest.log
tail -8 gpurun_out/g3_pytest.log
grep -E "PASS|FAIL" gpurun_out/g3_pytest.log | grep -c PASSED
( timeout -k 10 120 python -u tools/bench_attn.py &&
  timeout -k 10 120 python -u tools/bench_attn.py --T 4096 --H 128 --Hkv 128 --hd 192 --hdv 128 --pad 256 &&
  timeout -k 10 120 python -u tools/bench_attn.py --B 64 --T 197 --H 12 --Hkv 12 --hd 64 --noncausal &&
  timeout -k 10 120 python -u tools/bench_attn.py --T 4096 --H 16 --Hkv 1 --hd 256 &&
  timeout -k 10 120 python -u tools/bench_attn.py --B 128 --T 256 --H 1 --Hkv 1 --hd 256 --dropout 0.1 &&
  timeout -k 10 120 python -u tools/bench_attn.py --B 16 --T 256 --H 8 --Hkv 1 --hd 64 --dropout 0.1 ) > gpurun_out/g3_attn.txt 2>&1; echo "attn rc=$?"
grep attn -A1 gpurun_out/g3_attn.txt
