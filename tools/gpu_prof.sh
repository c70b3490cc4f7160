# profile the 4-layer LLaMA3-8B-shape step: per-kernel time summary
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_l4 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --layers 4 > gpurun_out/prof_l4.log 2>&1; echo "prof rc=$?"; tail -3 gpurun_out/prof_l4.log
fi
