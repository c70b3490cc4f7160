#!/bin/bash
# Round-3 round-start check: the GPU tests touched by the ADVICE fixes, the headline bench and
# the LLaMA-shape attention micro-bench on this box (baseline for the attention work).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_fp32_models_gpu.py tests/test_kernels_gpu.py -k "fp32 or dgrad or adamw" > gpurun_out/r3s_pytest.log 2>&1
echo "pytest rc=$?"; tail -15 gpurun_out/r3s_pytest.log
timeout -k 10 300 python -u tools/bench_attn.py > gpurun_out/r3s_attn.log 2>&1 && cat gpurun_out/r3s_attn.log | grep attn &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r3s_bench.log 2>&1; echo "bench rc=$?"
tail -2 gpurun_out/r3s_bench.log | cut -c1-400
