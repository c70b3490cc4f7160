#!/bin/bash
# 8-phase fp8 kernel: tests, kernel A/B vs the register-staged kernel, dsv3_v3 end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_moe_gpu.py -k "fp8" > gpurun_out/r3b_fp8_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3b_fp8_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_fp8_g8.py > gpurun_out/r3b_fp8_g8_bench.txt 2>&1; rc=$?; echo "bench rc=$rc"
cat gpurun_out/r3b_fp8_g8_bench.txt | grep '^{'; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_fp8_g8.py --experts 64 --rows 49152 --dim 2048 --ffn 1408 --dense 0 > gpurun_out/r3b_fp8_g8_bench_dsv3s.txt 2>&1; rc=$?
grep '^{' gpurun_out/r3b_fp8_g8_bench_dsv3s.txt; [ $rc -eq 0 ] || exit 1
for arm in bf16 fp8 fp8reg fp8 bf16 fp8reg; do
  e=""; [ $arm != bf16 ] && e="--fp8"; g8=1; [ $arm = fp8reg ] && g8=0
  SPA_FP8_G8=$g8 timeout -k 10 300 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum 4 --steps 4 --warmup 2 $e > gpurun_out/r3b_dsv3_$arm.log 2>&1 || exit 1
  echo "accum 4 $arm $(grep '^{' gpurun_out/r3b_dsv3_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done | tee gpurun_out/r3b_dsv3_fp8g8_abba.txt
