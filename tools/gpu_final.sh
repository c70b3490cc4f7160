#!/bin/bash
# End-of-session validation: every GPU test, smoke(), the headline bench and the secondary benches
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/final_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/final_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/final_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/final_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/vit_train.py --steps 8 --warmup 2 > gpurun_out/final_vit.log 2>&1 || exit 4
timeout -k 10 300 python bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2 > gpurun_out/final_dsv3s.log 2>&1 || exit 5
timeout -k 10 300 python bench/gemma_tp.py --layers 28 --steps 3 --warmup 1 > gpurun_out/final_gemma.log 2>&1 || exit 6
grep -h metric gpurun_out/final_vit.log gpurun_out/final_dsv3s.log gpurun_out/final_gemma.log | cut -c1-300
