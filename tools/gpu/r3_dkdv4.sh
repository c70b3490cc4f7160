#!/bin/bash
# dkdv4 (one-wave-per-SIMD dK/dV) correctness vs the single-wave kernel + ABBA timing at the
# LLaMA3-8B shape; then the overlap proxy at the default and 8 HW queues
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "flash or attention or attn or mla or packed or linear_act or activation" > gpurun_out/r3d4_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r3d4_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_attn.py --iters 20 --ab SPA_ATTN_DKDV=4 > gpurun_out/r3d4_attn.log 2>&1; echo "attn rc=$?"
grep -v amdgpu.ids gpurun_out/r3d4_attn.log
timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3o2_q4.log 2>&1; echo "q4 rc=$?"
grep -v amdgpu.ids gpurun_out/r3o2_q4.log | cut -c1-900
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3o2_q8.log 2>&1; echo "q8 rc=$?"
grep -v amdgpu.ids gpurun_out/r3o2_q8.log | cut -c1-900
timeout -k 10 400 python -u bench/parity.py --which B1,B3,B5,B7 --dtype fp32 --ref-loop --graph > gpurun_out/r3_parity_fp32.log 2>&1; echo "parity rc=$?"
grep -v amdgpu.ids gpurun_out/r3_parity_fp32.log | cut -c1-600
timeout -k 10 200 python -u tools/torch_op_profile_vit.py --rows 45 > gpurun_out/r3_vit_ops.log 2>&1; echo "vitops rc=$?"
tail -30 gpurun_out/r3_vit_ops.log | cut -c1-400
timeout -k 10 300 python -u bench/vit_train.py --steps 20 --warmup 5 > gpurun_out/r3_vit_bench.log 2>&1; echo "vit rc=$?"
grep -v amdgpu.ids gpurun_out/r3_vit_bench.log | tail -3 | cut -c1-600
