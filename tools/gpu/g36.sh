set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > gpurun_out/g36.log 2>&1; echo brc=$?
grep -v amdgpu.ids gpurun_out/g36.log | cut -c1-250
timeout -k 10 300 python -u bench/vit_train.py --steps 8 --warmup 2 >> gpurun_out/g36.log 2>&1; echo vrc=$?
tail -1 gpurun_out/g36.log | cut -c1-200
timeout -k 10 200 python -u tools/bench_attn.py --B 256 --T 197 --H 12 --Hkv 12 --hd 64 --noncausal --ab SPA_ATTN_DKDV=3,SPA_ATTN_DKDV=2 >> gpurun_out/g36.log 2>&1; echo arc=$?
grep "attn B\|with SPA" gpurun_out/g36.log
