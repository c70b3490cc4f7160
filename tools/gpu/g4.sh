set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_attention_dropout_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g4_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/g4_pytest.log
tail -4 gpurun_out/g4_pytest.log
timeout -k 10 300 python -u bench/parity.py --which B5,B9,B13 --steps 30 > gpurun_out/g4_parity.jsonl 2>&1; echo "parity rc=$?"
grep '^{' gpurun_out/g4_parity.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4/b13 -o b13 --output-format csv -- python bench/parity.py --which B13 --steps 5 --warmup 2 > gpurun_out/g4_prof_b13.log 2>&1; echo "prof b13 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4/b9 -o b9 --output-format csv -- python bench/parity.py --which B9 --steps 5 --warmup 2 > gpurun_out/g4_prof_b9.log 2>&1; echo "prof b9 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4/b5 -o b5 --output-format csv -- python bench/parity.py --which B5 --steps 5 --warmup 2 > gpurun_out/g4_prof_b5.log 2>&1; echo "prof b5 rc=$?"
timeout -k 10 400 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --steps 4 --warmup 2 > gpurun_out/g4_dsv3v3.jsonl 2>&1; echo "dsv3 rc=$?"
grep '^{' gpurun_out/g4_dsv3v3.jsonl
find gpurun_out/prof4 -name "*stats*" | head
timeout -k 10 300 python -u -m pytest tests/test_mla_decode_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g4_mla.log 2>&1; echo "mla rc=$?"
tail -12 gpurun_out/g4_mla.log
timeout -k 10 300 python -u bench/decode.py --model dsv3_style --batch 1 --prompt 1024 --new 64 > gpurun_out/g4_decode_mla.jsonl 2>&1; echo "dec rc=$?"
timeout -k 10 300 python -u bench/decode.py --model dsv3_style --batch 1 --prompt 1024 --new 64 --graph >> gpurun_out/g4_decode_mla.jsonl 2>&1; echo "dec graph rc=$?"
grep '^{' gpurun_out/g4_decode_mla.jsonl
