timeout -k 10 300 python -m pytest tests/test_misc_gpu.py -q -p no:cacheprovider > gpurun_out/pytest_misc.log 2>&1; echo rc=$?; tail -30 gpurun_out/pytest_misc.log
