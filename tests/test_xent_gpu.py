"""Vocab-chunked fused LM head + CE on the GPU (csrc/kernels/xent.hip xent_chunk_stats /
xent_chunk_grad_, ops/xent.py _ChunkedLinearXent) against an fp32 PyTorch oracle, and against
the materialised-logits path; peak memory of both at a LLaMA3-8B-like head."""
import pytest
import torch
import torch.nn.functional as F

from solvingpapers_amd.ops import _ext
from solvingpapers_amd.ops.xent import _LinearXentFn, chunked_linear_cross_entropy

pytestmark = pytest.mark.gpu


def _oracle(h, w, b, t, sm):
    hf, wf = h.float().detach().requires_grad_(), w.float().detach().requires_grad_()
    bf = b.float().detach().requires_grad_() if b is not None else None
    loss = F.cross_entropy(F.linear(hf, wf, bf), t, ignore_index=-100, label_smoothing=sm)
    loss.backward()
    return loss.detach(), hf.grad, wf.grad, (bf.grad if bf is not None else None)


@pytest.mark.parametrize("V,chunk,sm,bias", [(50257, 8192, 0.0, False), (32000, 4096, 0.1, True),
                                             (4096, 4096, 0.0, False)])
def test_chunked_head_matches_fp32_oracle(V, chunk, sm, bias):
    assert _ext.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    N, D = 1000, 256
    h = (torch.randn(N, D, device="cuda", generator=g) * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(V, D, device="cuda", generator=g) * 0.05).bfloat16().requires_grad_()
    b = (torch.randn(V, device="cuda", generator=g) * 0.05).bfloat16().requires_grad_() if bias else None
    t = torch.randint(0, V, (N,), device="cuda", generator=g)
    t[::37] = -100
    ref = _oracle(h, w, b, t, sm)
    loss = chunked_linear_cross_entropy(h, w, t, bias=b, label_smoothing=sm, chunk_cols=chunk)
    (loss * 0.5).backward()
    assert abs(loss.item() - ref[0].item()) < 2e-3 * abs(ref[0].item())
    for got, want in ((h.grad, ref[1]), (w.grad, ref[2]), (b.grad if bias else None, ref[3])):
        if want is None:
            continue
        rel = ((got.float() - 0.5 * want).norm() / (0.5 * want).norm()).item()
        assert rel < 1.5e-2, rel


def test_chunked_head_peak_memory_below_materialised():
    """8192 x 128256 x 4096 bf16 (the LLaMA3-8B head): beyond the gradients themselves the chunked
    head (512 MiB chunks) holds about one chunk, the materialised one the whole 2.1 GB of logits."""
    N, D, V = 8192, 4096, 128256
    g = torch.Generator(device="cuda").manual_seed(1)
    h = (torch.randn(N, D, device="cuda", generator=g) * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(V, D, device="cuda", generator=g) * 0.02).bfloat16().requires_grad_()
    t = torch.randint(0, V, (N,), device="cuda", generator=g)
    peaks, losses = {}, {}
    for name in ("materialised", "chunked"):
        h.grad = w.grad = None
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        if name == "chunked":
            loss = chunked_linear_cross_entropy(h, w, t, chunk_cols=(1 << 29) // (N * 2))
        else:
            loss = _LinearXentFn.apply(h, w, None, t, -100, 0.0)
        loss.backward()
        torch.cuda.synchronize()
        peaks[name] = torch.cuda.max_memory_allocated() - base
        losses[name] = loss.item()
    assert abs(losses["chunked"] - losses["materialised"]) < 1e-3 * losses["materialised"]
    grads = (N * D + V * D) * 2
    chunk = 1 << 29
    assert peaks["chunked"] - grads <= 2 * chunk, peaks
    assert peaks["materialised"] - grads >= N * V * 2, peaks
    assert peaks["materialised"] - peaks["chunked"] >= 1.2e9, peaks
