set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof12
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof12/f8 -o f8 --output-format csv -- python bench/dsv3_train.py --preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --steps 3 --warmup 1 --fp8 > gpurun_out/g12.log 2>&1; echo rc=$?
grep '^{' gpurun_out/g12.log
