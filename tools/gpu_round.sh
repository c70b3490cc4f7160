timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 4 --warmup 2 --layers 4 > gpurun_out/bench_l4.log 2>&1; rc=$?; echo "bench_l4 rc=$rc"; tail -5 gpurun_out/bench_l4.log
  if [ $rc -eq 0 ]; then timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -5 gpurun_out/bench.log; fi
fi
