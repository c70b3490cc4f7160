set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof13
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof13/b -o b --output-format csv -- python bench.py --steps 2 --warmup 1 > gpurun_out/g13.log 2>&1; echo rc=$?
grep '^{' gpurun_out/g13.log
