# MLA (DeepSeek) KV-cached decode throughput on the compressed latent cache
mkdir -p gpurun_out
timeout -k 10 240 python -u bench/decode.py --model dsv3_style --prompt 1024 --new 64 > gpurun_out/decode_mla.jsonl 2> gpurun_out/decode_mla.err &&
timeout -k 10 240 python -u bench/decode.py --model dsv3_style --prompt 1024 --new 64 --batch 16 >> gpurun_out/decode_mla.jsonl 2>> gpurun_out/decode_mla.err &&
timeout -k 10 240 python -u bench/decode.py --model dsv3_v3 --layers 4 --set n_experts=32 --set n_dense_layers=1 --prompt 1024 --new 32 >> gpurun_out/decode_mla.jsonl 2>> gpurun_out/decode_mla.err
