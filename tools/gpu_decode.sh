#!/bin/bash
# decode kernel tests + KV-cached generation benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_decode.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_decode.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 > gpurun_out/decode.log 2>&1 || exit 2
timeout -k 10 200 python bench/decode.py --prompt 7936 --new 128 >> gpurun_out/decode.log 2>&1 || exit 2
timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 --batch 16 >> gpurun_out/decode.log 2>&1 || exit 2
timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 --graph >> gpurun_out/decode.log 2>&1 || exit 3
timeout -k 10 200 python bench/decode.py --prompt 1024 --new 128 --batch 16 --graph >> gpurun_out/decode.log 2>&1 || exit 3
cat gpurun_out/decode.log | grep metric
