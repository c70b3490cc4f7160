# full-depth secondary configs, ViT profile, EP host trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof14
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/g14_$name.log 2>&1; local rc=$?;
         echo "$name rc=$rc"; if [ $rc -ge 124 ]; then tail -30 gpurun_out/g14_$name.log; exit $rc; fi; }
step vit 300 python -u bench/vit_train.py --steps 5 --warmup 2
grep -h '^{' gpurun_out/g14_vit.log
step vitprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof14/vit -o vit --output-format csv -- python bench/vit_train.py --steps 3 --warmup 1
step ep 300 python -u tools/ep_host_trace.py gpurun_out/ep_trace
grep -h '^{' gpurun_out/g14_ep.log
step gemma 600 python -u bench/gemma_tp.py --steps 3 --warmup 1
grep -h '^{' gpurun_out/g14_gemma.log
step dsv3s 600 python -u bench/dsv3_train.py --preset dsv3_style --steps 3 --warmup 1
grep -h '^{' gpurun_out/g14_dsv3s.log
