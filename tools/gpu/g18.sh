set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "bwd_variants" > gpurun_out/g18_t.log 2>&1; echo trc=$?; tail -3 gpurun_out/g18_t.log
timeout -k 10 200 python -u tools/bench_attn.py --ab SPA_ATTN_DKDV=3,SPA_ATTN_DKDV=3 > gpurun_out/g18.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_attn.py --B 64 --T 197 --H 12 --Hkv 12 --hd 64 --noncausal --ab SPA_ATTN_DKDV=3 >> gpurun_out/g18.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g18.log
