#!/bin/bash
# PV / dQ chain prefetch hints (FWD_PV_SCHED): in-tree _C.so (on) vs ab/_C_nopv.so (off), ABBA processes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "flash or attention or attn or mla" > gpurun_out/r3pv_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r3pv_pytest.log
[ $rc -eq 0 ] || exit 1
for arm in on off off on; do
  if [ $arm = off ]; then export SPA_EXT_SO=$GRAFT_REPO_ROOT/ab/_C_nopv.so; else unset SPA_EXT_SO; fi
  timeout -k 10 120 python -u tools/bench_attn.py --iters 20 > gpurun_out/r3pv_$arm.log 2>&1 || exit 1
  echo "$arm $(grep 'attn B' gpurun_out/r3pv_$arm.log)"
  timeout -k 10 120 python -u tools/bench_attn.py --T 8192 --H 16 --Hkv 1 --hd 256 --iters 10 > gpurun_out/r3pv_g_$arm.log 2>&1 || exit 1
  echo "$arm $(grep 'attn B' gpurun_out/r3pv_g_$arm.log)"
done | tee gpurun_out/r3pv_abba.txt
unset SPA_EXT_SO
