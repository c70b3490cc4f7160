#!/usr/bin/env python
"""KV-cached generation throughput (serving-side bench): prompt prefill + N decode steps.

Default: LLaMA3-8B shape, bf16, random-init weights, synthetic prompt. Reports prefill
tok/s and decode tok/s (all sequences); one JSON line. The reference decodes by re-running
the whole prefix per token (llama3/LLaMA-jax.ipynb:1629: 20 tokens in 60.6 s on a T4)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from solvingpapers_amd.infer import GenerationStats  # noqa: E402


def build(model, layers, sets=()):
    kw = {} if layers is None else {"n_layers": layers}
    for kv in sets:                      # --set n_experts=32 etc. (int/float/str)
        k, v = kv.split("=", 1)
        for cast in (int, float):
            try:
                v = cast(v)
                break
            except ValueError:
                pass
        kw[k] = v
    if model.startswith("dsv3"):
        # MLA decode attends over the per-layer compressed latent cache (kv_lora + rope values
        # per token) with W_uk absorbed into q and W_uv applied after
        from solvingpapers_amd.models import deepseekv3
        return deepseekv3.DeepSeekV3(deepseekv3.config(model, **kw), device="cuda", dtype=torch.bfloat16, seed=1)
    if model.startswith("llama3"):
        from solvingpapers_amd.models import llama3
        return llama3.Llama3(llama3.config(model, **kw), device="cuda", dtype=torch.bfloat16, seed=1)
    from solvingpapers_amd.models import gemma
    return gemma.Gemma(gemma.config(model, **kw), device="cuda", dtype=torch.bfloat16, seed=1)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3_8b")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--prompt", type=int, default=1024)
    ap.add_argument("--new", type=int, default=128)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--graph", action="store_true", help="HIP-graph decode (one replay per token)")
    ap.add_argument("--set", action="append", default=[], help="config override key=value")
    a = ap.parse_args(argv)
    m = build(a.model, a.layers, a.set).eval()
    ids = torch.randint(0, m.c.vocab_size, (a.batch, a.prompt), device="cuda")
    st = GenerationStats()
    if a.graph:
        from solvingpapers_amd.infer import GraphDecoder
        dec = GraphDecoder(m, a.batch, a.prompt + a.new)
        dec.generate(ids[:, :64], 4)  # warm-up of the eager prefill path
        out = dec.generate(ids, a.new, stats=st)
    else:
        m.generate(ids[:, :64], 4, greedy=True)  # warm-up (kernels, allocator)
        out = m.generate(ids, a.new, greedy=True, stats=st)
    torch.cuda.synchronize()
    print(json.dumps({"metric": "decode tokens/s", "model": a.model, "graph": a.graph, "batch": a.batch, "prompt": a.prompt,
                      "new_tokens": st.new_tokens, "prefill_tok_s": round(st.prefill_tok_s, 1),
                      "decode_tok_s": round(st.decode_tok_s, 2),
                      "ms_per_token": round(1e3 * st.decode_s / max(1, st.new_tokens // a.batch), 3),
                      "dtype": "bf16", "data": "synthetic prompt, random-init weights",
                      "out_len": out.shape[1]}), flush=True)


if __name__ == "__main__":
    main()
