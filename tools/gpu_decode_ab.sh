#!/bin/bash
# decode tests, then in-launch split merge (SPA_DECODE_FUSED=1) vs separate combine kernel, same box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u -m pytest tests/test_decode_gpu.py tests/test_gemv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_decode.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_decode.log
[ $rc -eq 0 ] || exit 1
SPA_DECODE_FUSED=1 timeout -k 10 240 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_decode1.log 2>&1 || { tail -20 gpurun_out/pytest_decode1.log; exit 1; }
: > gpurun_out/decode_ab.log
for args in "--prompt 1024 --new 128 --graph" "--prompt 7936 --new 128 --graph" "--prompt 1024 --new 128 --batch 16 --graph"; do
  for f in 1 0; do
    echo "fused=$f $args" >> gpurun_out/decode_ab.log
    SPA_DECODE_FUSED=$f timeout -k 10 200 python bench/decode.py $args >> gpurun_out/decode_ab.log 2>&1 || exit 3
  done
done
grep -o 'fused=.*\|"decode_tok_s": [0-9.]*' gpurun_out/decode_ab.log
