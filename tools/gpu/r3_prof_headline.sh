#!/bin/bash
# headline step kernel profile, fused act-bwd test, overlap proxy with the multi-rank GEMM config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "mlp_fused or linear_act" > gpurun_out/r3p_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3p_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench/vit_train.py --steps 20 --warmup 5 > gpurun_out/r3p_vit.log 2>&1; echo "vit rc=$?"
grep '^{' gpurun_out/r3p_vit.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3p_prof -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r3p_prof.log 2>&1; echo "prof rc=$?"
grep '^{' gpurun_out/r3p_prof.log | cut -c1-300
find gpurun_out/r3p_prof -name "*.db" | head -3
for db in $(find gpurun_out/r3p_prof -name "*.db"); do python tools/rocpd_summary.py $db --top 40 > gpurun_out/r3p_prof_summary.txt 2>&1; done
head -50 gpurun_out/r3p_prof_summary.txt | cut -c1-160
timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 > gpurun_out/r3p_overlap.log 2>&1; echo "proxy rc=$?"
grep -v amdgpu.ids gpurun_out/r3p_overlap.log | cut -c1-900
