"""Time / peak memory of the LM head + CE at a LLaMA3-8B-like shape: materialised logits
(_LinearXentFn) vs vocab-chunked (_ChunkedLinearXent) at several chunk budgets."""
import json
import sys

import torch

sys.path.insert(0, ".")
from solvingpapers_amd.ops.xent import _LinearXentFn, chunked_linear_cross_entropy  # noqa: E402


def main():
    N, D, V = 8192, 4096, int(sys.argv[1]) if len(sys.argv) > 1 else 128256
    g = torch.Generator(device="cuda").manual_seed(0)
    h = (torch.randn(N, D, device="cuda", generator=g) * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(V, D, device="cuda", generator=g) * 0.02).bfloat16().requires_grad_()
    t = torch.randint(0, V, (N,), device="cuda", generator=g)
    arms = [("materialised", None)] + [(f"chunk{mb}MiB", (mb << 20) // (N * 2)) for mb in (256, 512, 1024)]
    for rnd in range(3):
        for name, cols in arms:
            h.grad = w.grad = None
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats()
            base = torch.cuda.memory_allocated()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                h.grad = w.grad = None
                loss = _LinearXentFn.apply(h, w, None, t, -100, 0.0) if cols is None else \
                    chunked_linear_cross_entropy(h, w, t, chunk_cols=cols)
                loss.backward()
            e1.record()
            torch.cuda.synchronize()
            if rnd == 2:
                print(json.dumps({"arm": name, "N": N, "D": D, "V": V, "ms_fwd_bwd": round(e0.elapsed_time(e1) / 3, 3),
                                  "peak_extra_gb": round((torch.cuda.max_memory_allocated() - base) / 1e9, 3),
                                  "loss": round(loss.item(), 5)}), flush=True)


if __name__ == "__main__":
    main()
