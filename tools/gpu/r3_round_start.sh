#!/bin/bash
# Round-3 check: GPU tests touched this round, the 1-GPU TP/EP overlap proxy, the LLaMA-shape
# attention micro-bench and the headline bench on this box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_fp32_models_gpu.py tests/test_kernels_gpu.py -k "fp32 or dgrad or adamw" > gpurun_out/r3s_pytest.log 2>&1
echo "pytest rc=$?"; tail -15 gpurun_out/r3s_pytest.log
timeout -k 10 300 python -u tools/bench_attn.py > gpurun_out/r3s_attn.log 2>&1 && grep attn gpurun_out/r3s_attn.log &&
timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3s_overlap.log 2>&1; echo "overlap rc=$?"
grep -v amdgpu.ids gpurun_out/r3s_overlap.log | tail -4 | cut -c1-600
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r3s_bench.log 2>&1; echo "bench rc=$?"
tail -2 gpurun_out/r3s_bench.log | cut -c1-400
