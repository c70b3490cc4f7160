"""DeepSeek MLA latent-space decode (csrc/kernels/mla_decode.hip) against the fp32 formula,
one split and split-K (merge kernel), host and device valid lengths; and HIP-graph decoding of
a DeepSeek-V3-style model (GraphDecoder) against its own full forward."""
import math

import pytest
import torch

from solvingpapers_amd.ops import _ext
from solvingpapers_amd.ops.attention import mla_decode_attention

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _oracle(q, qr, cc, cr, scale, S):
    T = q.shape[1]
    s = (torch.einsum("bthc,bsc->bhts", q.float(), cc[:, :S].float())
         + torch.einsum("bthr,bsr->bhts", qr.float(), cr[:, :S].float())) * scale
    i = torch.arange(T, device=s.device)[:, None] + (S - T)
    j = torch.arange(S, device=s.device)[None, :]
    s = s.masked_fill(j > i, float("-inf"))
    return torch.einsum("bhts,bsc->bthc", torch.softmax(s, -1), cc[:, :S].float())


@pytest.mark.parametrize("B,T,H,C,R,S,Smax,nsplit", [
    (1, 1, 16, 512, 64, 1024, 1100, 0),     # dsv3_style decode, auto split
    (2, 1, 128, 512, 64, 300, 512, 1),      # V3 widths (128 heads = 8 row blocks), one split
    (2, 1, 128, 512, 64, 777, 1024, 5),     # ragged length, 5 splits
    (1, 7, 16, 512, 64, 200, 256, 0),       # 7 tokens at once (causal inside the new rows)
    (3, 1, 4, 64, 32, 90, 128, 2),          # dsv3_tiny widths
])
def test_mla_decode_matches_formula(B, T, H, C, R, S, Smax, nsplit):
    assert _ext.load()
    torch.manual_seed(0)
    q = torch.randn(B, T, H, C, device=DEV, dtype=torch.bfloat16)
    qr = torch.randn(B, T, H, R, device=DEV, dtype=torch.bfloat16)
    cc = torch.randn(B, Smax, C, device=DEV, dtype=torch.bfloat16)
    cr = torch.randn(B, Smax, R, device=DEV, dtype=torch.bfloat16)
    sc = 1.0 / math.sqrt(192)
    want = _oracle(q, qr, cc, cr, sc, S)
    got = mla_decode_attention(q, qr, cc, cr, sc, S, None, nsplit)
    assert rel(got, want) < 1.5e-2, rel(got, want)
    kv = torch.tensor([S], device=DEV, dtype=torch.int32)        # graph mode: device length
    got2 = mla_decode_attention(q, qr, cc, cr, sc, 0, kv, nsplit)
    assert rel(got2, want) < 1.5e-2


def test_dsv3_graph_decoder_matches_full_forward():
    from solvingpapers_amd.infer import GraphDecoder
    from solvingpapers_amd.models import deepseekv3 as ds
    torch.manual_seed(0)
    c = ds.config("dsv3_tiny", mtp_heads=0)
    m = ds.DeepSeekV3(c, device=DEV, dtype=torch.bfloat16, seed=1).eval()
    ids = torch.randint(0, c.vocab_size, (2, 30), device=DEV)
    with torch.no_grad():
        full = m(ids).float()
        dec = GraphDecoder(m, 2, 40)
        lg = [dec.prefill(ids[:, :20])]
        for t in range(20, 30):
            dec.ids.copy_(ids[:, t:t + 1])
            dec.graph.replay()
            lg.append(dec.logits.clone())
    assert rel(lg[0], full[:, 19]) < 3e-2
    assert rel(torch.stack(lg[1:], 1), full[:, 20:30]) < 3e-2
