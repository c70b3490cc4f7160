mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_moe_gpu.py -k "mixed_head or deepseek_gpu" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t2.log 2>&1 &&
timeout -k 10 300 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --steps 4 --warmup 2 > gpurun_out/dsv3_v3.log 2>&1 &&
timeout -k 10 300 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --steps 4 --warmup 2 --fp8 >> gpurun_out/dsv3_v3.log 2>&1 &&
timeout -k 10 300 python -u bench/dsv3_train.py --layers 4 --steps 4 --warmup 2 >> gpurun_out/dsv3_v3.log 2>&1
