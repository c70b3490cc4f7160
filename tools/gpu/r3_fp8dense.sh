#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_moe_gpu.py tests/test_kernels_gpu.py -k "fp8 or flash or attention or attn or mla" > gpurun_out/r3fd_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3fd_pytest.log
[ $rc -eq 0 ] || exit 1
for acc in 1 4; do
for arm in bf16 fp8 fp8 bf16; do
  e=""; [ $arm = fp8 ] && e="--fp8"
  timeout -k 10 300 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum $acc --steps 4 --warmup 2 $e > gpurun_out/r3fd_dsv3_${arm}_$acc.log 2>&1 || exit 1
  echo "accum $acc $arm $(grep '^{' gpurun_out/r3fd_dsv3_${arm}_$acc.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done | tee gpurun_out/r3fd_dsv3_abba.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3fd_gemma_attn -o run -- python tools/bench_attn.py --T 8192 --H 16 --Hkv 1 --hd 256 --iters 5 > gpurun_out/r3fd_gemma_attn.log 2>&1; echo "gattn rc=$?"
grep "attn B" gpurun_out/r3fd_gemma_attn.log
python tools/rocpd_summary.py gpurun_out/r3fd_gemma_attn/run_results.db --top 12 --grep attn > gpurun_out/r3fd_gemma_attn_summary.txt 2>&1; head -20 gpurun_out/r3fd_gemma_attn_summary.txt | cut -c1-150
