set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_dropout_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "attention or attn" > gpurun_out/g25_t.log 2>&1; rc=$?; echo trc=$rc; tail -3 gpurun_out/g25_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_attn.py --B 256 --T 197 --H 12 --Hkv 12 --hd 64 --noncausal > gpurun_out/g25.log 2>&1 && \
timeout -k 10 300 python -u bench/vit_train.py --steps 6 --warmup 2 >> gpurun_out/g25.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p25 -o vit --output-format csv -- python3 bench/vit_train.py --steps 3 --warmup 1 > gpurun_out/g25p.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g25.log | cut -c1-250
