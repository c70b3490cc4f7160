set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
A="--preset dsv3_v3 --layers 4 --experts 32 --dense-layers 1 --seq 4096 --mb 1 --steps 4 --warmup 2"
timeout -k 10 400 python -u bench/dsv3_train.py $A > gpurun_out/g29.log 2>&1 && \
timeout -k 10 400 python -u bench/dsv3_train.py $A --fp8 --bf16-moments >> gpurun_out/g29.log 2>&1 && \
timeout -k 10 300 python -u tools/torch_op_profile.py --fp8 --rows 45 > gpurun_out/g29p.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/g29.log | cut -c1-220
