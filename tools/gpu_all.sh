#!/bin/bash
# Full GPU test suite in one process
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo rc=$rc
tail -40 gpurun_out/pytest_gpu.log
exit $rc
