set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_attn.py --ab SPA_ATTN_FWD_PIPE=1 > gpurun_out/g15.log 2>&1 && \
timeout -k 10 200 python -u tools/bench_attn.py --B 64 --T 197 --H 12 --Hkv 12 --hd 64 --noncausal --ab SPA_ATTN_FWD_PIPE=1 >> gpurun_out/g15.log 2>&1; echo rc=$?
cat gpurun_out/g15.log | grep -v amdgpu.ids
