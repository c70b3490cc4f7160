#!/bin/bash
# batch B: fused fp8 dual quantization (tests, kernel A/B, dsv3_v3 ABBA at accum 4), TP proxy trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_moe_gpu.py -k "fp8" > gpurun_out/r3b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3b_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_fp8_wgrad.py > gpurun_out/r3b_wg.log 2>&1; echo "wg rc=$?"
grep '^{' gpurun_out/r3b_wg.log
for acc in 4; do
for arm in bf16 fp8 fp8 bf16; do
  e=""; [ $arm = fp8 ] && e="--fp8"
  timeout -k 10 300 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum $acc --steps 4 --warmup 2 $e > gpurun_out/r3b_dsv3_${arm}_$acc.log 2>&1 || exit 1
  echo "accum $acc $arm $(grep '^{' gpurun_out/r3b_dsv3_${arm}_$acc.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done | tee gpurun_out/r3b_dsv3_abba.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3b_tpprof -o run -- python tools/overlap_proxy.py --which tp --arms pipelined --iters 2 --rounds 1 > gpurun_out/r3b_tpprof.log 2>&1; echo "tpprof rc=$?"
tail -2 gpurun_out/r3b_tpprof.log | cut -c1-300
