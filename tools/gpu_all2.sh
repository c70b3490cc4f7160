#!/bin/bash
# full GPU validation: tests, smoke, headline + secondary benches (each step time-limited)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1 || exit 3
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench.log | tr '\n' ' '; echo
timeout -k 10 300 python bench/dsv3_train.py --layers 4 > gpurun_out/dsv3.log 2>&1 || echo "dsv3 FAILED"
grep -o '"metric": "[^"]*"\|"value": [0-9.]*' gpurun_out/dsv3.log | tr '\n' ' '; echo
timeout -k 10 300 python bench/vit_train.py > gpurun_out/vit.log 2>&1 || echo "vit FAILED"
grep -o '"metric": "[^"]*"\|"value": [0-9.]*' gpurun_out/vit.log | tr '\n' ' '; echo
timeout -k 10 300 python bench/gemma_tp.py --layers 4 --seq 4096 > gpurun_out/gemma.log 2>&1 || echo "gemma FAILED"
grep -o '"metric": "[^"]*"\|"value": [0-9.]*' gpurun_out/gemma.log | tr '\n' ' '; echo
timeout -k 10 300 python bench/decode.py --prompt 1024 --new 128 --graph > gpurun_out/decode_llama.log 2>&1 || echo "llama decode FAILED"
grep -o '"decode_tok_s": [0-9.]*' gpurun_out/decode_llama.log
timeout -k 10 300 python bench/decode.py --model gemma_7b_mqa --prompt 1024 --new 128 --graph > gpurun_out/decode_gemma.log 2>&1 || echo "gemma decode FAILED"
grep -o '"decode_tok_s": [0-9.]*' gpurun_out/decode_gemma.log
