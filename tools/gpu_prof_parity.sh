#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o run --output-format csv -- python3 bench/parity.py --which B1 --steps 20 --warmup 3 > gpurun_out/prof_b1.log 2>&1
rc=$?; echo rc=$rc; tail -3 gpurun_out/prof_b1.log; exit $rc
