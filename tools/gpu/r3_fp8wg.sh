#!/bin/bash
# fp8 expert Wgrad: numerics test, kernel A/B vs bf16 grouped dW, dsv3_v3 bf16 vs fp8 ABBA (accum 1 and 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_moe_gpu.py -k "fp8" > gpurun_out/r3w_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3w_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_fp8_wgrad.py > gpurun_out/r3w_bench.log 2>&1; echo "wg rc=$?"
grep '^{' gpurun_out/r3w_bench.log
for acc in 1 4; do
for arm in bf16 fp8 fp8 bf16; do
  e=""; [ $arm = fp8 ] && e="--fp8"
  timeout -k 10 300 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum $acc --steps 4 --warmup 2 $e > gpurun_out/r3w_dsv3_${arm}_$acc.log 2>&1 || exit 1
  echo "accum $acc $arm $(grep '^{' gpurun_out/r3w_dsv3_${arm}_$acc.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done | tee gpurun_out/r3w_dsv3_abba.txt
