#!/bin/bash
# decode kernel tests + KV-cached generation benches (GEMV on/off A/B in the same call)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u -m pytest tests/test_decode_gpu.py tests/test_gemv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_decode.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_decode.log
[ $rc -eq 0 ] || exit 1
: > gpurun_out/decode.log
timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 --graph >> gpurun_out/decode.log 2>&1 || exit 3
SPA_GEMV=0 timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 --graph >> gpurun_out/decode.log 2>&1 || exit 3
timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 >> gpurun_out/decode.log 2>&1 || exit 2
timeout -k 10 200 python bench/decode.py --prompt 7936 --new 128 --graph >> gpurun_out/decode.log 2>&1 || exit 2
timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 --batch 4 --graph >> gpurun_out/decode.log 2>&1 || exit 3
timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 --batch 16 --graph >> gpurun_out/decode.log 2>&1 || exit 3
grep metric gpurun_out/decode.log
