#!/bin/bash
# round-3 validation: every GPU test, smoke(), the headline bench, the secondary benches, B8 parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r3f_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3f_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r3f_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/r3f_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r3f_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/vit_train.py --steps 20 --warmup 5 > gpurun_out/r3f_vit.log 2>&1 || exit 4
timeout -k 10 300 python bench/dsv3_train.py --preset dsv3_style --steps 4 --warmup 2 > gpurun_out/r3f_dsv3s.log 2>&1 || exit 5
timeout -k 10 400 python bench/gemma_tp.py --layers 28 --steps 3 --warmup 1 > gpurun_out/r3f_gemma.log 2>&1 || exit 6
grep -h '^{' gpurun_out/r3f_vit.log gpurun_out/r3f_dsv3s.log gpurun_out/r3f_gemma.log | cut -c1-400
timeout -k 10 600 python -u bench/parity.py --which B8 --ref-loop --graph > gpurun_out/r3f_b8.log 2>&1; echo "b8 rc=$?"
grep '^{' gpurun_out/r3f_b8.log | cut -c1-500
