#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "flash or attention or attn or mla" > gpurun_out/r3h_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3h_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_attn.py --T 8192 --H 16 --Hkv 1 --hd 256 --iters 10 > gpurun_out/r3h_attn.log 2>&1; echo "attn rc=$?"
grep "attn B" gpurun_out/r3h_attn.log
timeout -k 10 400 python -u tools/overlap_proxy.py --layers 2 --which tp --batch 2 --seq 4096 --variants two_stream > gpurun_out/r3h_tpb.log 2>&1; echo "tpb rc=$?"
grep '^{' gpurun_out/r3h_tpb.log | cut -c1-800
