#!/bin/bash
# fused MLP epilogues: numerics tests, ABBA vs library GEMMs, ViT-B/16 bench both ways, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "mlp_fused or linear_act or grouped or wgrad" > gpurun_out/r3m_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r3m_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_vit_mlp.py > gpurun_out/r3m_mlp.log 2>&1; echo "mlp rc=$?"
grep -v amdgpu.ids gpurun_out/r3m_mlp.log
timeout -k 10 300 python -u bench/vit_train.py --steps 20 --warmup 5 > gpurun_out/r3m_vit_fused.log 2>&1; echo "vit rc=$?"
grep '^{' gpurun_out/r3m_vit_fused.log | cut -c1-300
SPA_MLP_EPI=0 timeout -k 10 300 python -u bench/vit_train.py --steps 20 --warmup 5 > gpurun_out/r3m_vit_lib.log 2>&1; echo "vit0 rc=$?"
grep '^{' gpurun_out/r3m_vit_lib.log | cut -c1-300
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3m_bench.log 2>&1; echo "bench rc=$?"
grep '^{' gpurun_out/r3m_bench.log | cut -c1-400
