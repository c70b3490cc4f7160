# rocprofv3 kernel stats of the DeepSeek-V3-width bench (4 layers, 32 experts, 1 GPU)
mkdir -p gpurun_out/prof_v3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v3 -o run -- python3 bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --steps 3 --warmup 1 > gpurun_out/prof_v3/bench.log 2>&1
