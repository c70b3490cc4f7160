set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/p19a gpurun_out/p19b
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p19a -o run --output-format csv -- python3 -u tools/bench_attn.py --iters 20 > gpurun_out/g19a.log 2>&1 && \
SPA_ATTN_DKDV=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p19b -o run --output-format csv -- python3 -u tools/bench_attn.py --iters 20 > gpurun_out/g19b.log 2>&1; echo rc=$?
for d in p19a p19b; do f=$(find gpurun_out/$d -name '*kernel_stats.csv' | head -1); echo "== $d"; grep -i "attn" $f | cut -c1-200 || true; done
