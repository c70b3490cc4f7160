timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider -k "flash or packed" > gpurun_out/pytest_attn.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_attn.log
if [ $rc -le 1 ]; then
timeout -k 10 300 python tools/bench_attn.py && timeout -k 10 300 python tools/bench_attn.py --T 2048 --B 4 && timeout -k 10 300 python tools/bench_attn.py --T 197 --B 64 --H 12 --Hkv 12 --hd 64 --noncausal
fi
