set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_attn.py > gpurun_out/g17.log 2>&1 && timeout -k 10 200 env SPA_ATTN_STAMP=1 python -u tools/bench_attn.py --iters 3 >> gpurun_out/g17.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g17.log
