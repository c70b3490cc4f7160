cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
timeout -k 10 600 python bench.py --steps 6 --warmup 2 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; grep metric gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run --output-format csv -- python bench.py --steps 2 --warmup 1 > gpurun_out/prof_full.log 2>&1; echo "prof rc=$?"
fi
