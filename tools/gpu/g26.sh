set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --mb 2 --accum 2 > gpurun_out/g26.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g26.log | cut -c1-330
timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --mb 4 --accum 1 > gpurun_out/g26b.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g26b.log | cut -c1-330
