timeout -k 10 300 python -m pytest tests/test_llama_gpu.py -q -p no:cacheprovider > gpurun_out/pytest_llama.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_llama.log
if [ $rc -le 1 ]; then
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; grep metric gpurun_out/bench.log
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --no-opt-overlap > gpurun_out/bench_noov.log 2>&1; echo "bench rc=$?"; grep metric gpurun_out/bench_noov.log
fi
