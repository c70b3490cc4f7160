mkdir -p gpurun_out
timeout -k 10 300 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum 4 --steps 3 --warmup 1 > gpurun_out/dsv3_accum.log 2>&1 &&
timeout -k 10 300 python -u bench/dsv3_train.py --preset dsv3_v3 --layers 4 --dense-layers 1 --experts 32 --mb 1 --accum 4 --steps 3 --warmup 1 --fp8 >> gpurun_out/dsv3_accum.log 2>&1 &&
timeout -k 10 300 python -u bench/dsv3_train.py --layers 4 --accum 4 --steps 3 --warmup 1 >> gpurun_out/dsv3_accum.log 2>&1
