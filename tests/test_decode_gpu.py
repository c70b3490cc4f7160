"""Split-K decode attention (csrc/kernels/decode.hip) vs the fp32 oracle, and KV-cached
generation on the GPU (decode kernel in the loop) vs full re-forward logits."""
import math

import pytest
import torch

from solvingpapers_amd.ops import _ext, reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


CASES = [
    # B, Tq, Tk, H, Hkv, hd, nsplit
    (1, 1, 8192, 32, 8, 128, 0),     # LLaMA3-8B decode step (GQA, 4 rows per kv head)
    (3, 1, 1000, 8, 2, 128, 0),      # ragged split
    (2, 4, 777, 8, 2, 64, 0),        # 4 new tokens (speculative / chunked), 16 rows
    (1, 1, 4096, 16, 1, 256, 0),     # Gemma-7B MQA: 16 rows on one kv head
    (2, 2, 50, 4, 4, 128, 1),        # single split
    (1, 1, 1, 4, 2, 64, 0),          # first token
    (2, 3, 300, 6, 3, 128, 7),       # odd split count, causal rows inside the cache
]


@pytest.mark.parametrize("B,Tq,Tk,H,Hkv,hd,ns", CASES)
def test_decode_attention_matches_oracle(B, Tq, Tk, H, Hkv, hd, ns):
    torch.manual_seed(0)
    q = torch.randn(B, Tq, H, hd, device=DEV, dtype=torch.bfloat16)
    # cache views with a padded max length, as the KV cache hands them over
    kc = torch.randn(B, Tk + 37, Hkv, hd, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(B, Tk + 37, Hkv, hd, device=DEV, dtype=torch.bfloat16)
    k, v = kc[:, :Tk], vc[:, :Tk]
    sc = 1 / math.sqrt(hd)
    out, lse = _ext.ops().attn_decode(q, k, v, sc, True, ns)
    of, lf = R.attention(q.float(), k.float(), v.float(), True, sc)
    assert rel(out, of) < 1e-2, rel(out, of)
    assert (lse - lf).abs().max().item() < 1e-2


def test_decode_attention_repeated_launches_rearm_split_counters():
    """Back-to-back launches with different split counts and grids, and a device kv_len that
    leaves trailing splits empty, must all match the oracle (with SPA_DECODE_FUSED=1 this also
    checks that every launch re-arms the per-(b, kv head) arrival counters)."""
    torch.manual_seed(1)
    sc = 1 / math.sqrt(128)
    for it, (B, Tk, ns) in enumerate([(1, 2000, 0), (2, 2000, 5), (1, 2000, 31), (2, 700, 0), (1, 2000, 0)]):
        q = torch.randn(B, 1, 32, 128, device=DEV, dtype=torch.bfloat16)
        k = torch.randn(B, Tk, 8, 128, device=DEV, dtype=torch.bfloat16)
        v = torch.randn(B, Tk, 8, 128, device=DEV, dtype=torch.bfloat16)
        n = Tk - 300 * (it % 2)
        kv_len = torch.tensor([n], device=DEV, dtype=torch.int32)
        out, _ = _ext.ops().attn_decode(q, k, v, sc, True, ns, kv_len)
        of, _ = R.attention(q.float(), k[:, :n].float(), v[:, :n].float(), True, sc)
        assert rel(out, of) < 1e-2, (it, rel(out, of))


def test_decode_attention_routes_prefill_to_flash():
    from solvingpapers_amd.ops import decode_attention, flash_attention
    q = torch.randn(1, 64, 8, 128, device=DEV, dtype=torch.bfloat16)  # 64 * 4 rows > 16 -> flash
    k = torch.randn(1, 64, 2, 128, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(1, 64, 2, 128, device=DEV, dtype=torch.bfloat16)
    assert torch.equal(decode_attention(q, k, v), flash_attention(q, k, v))


def test_llama_cached_steps_match_full_forward():
    from solvingpapers_amd.models import llama3
    torch.manual_seed(0)
    m = llama3.Llama3(llama3.config("llama3_tiny"), device=DEV, dtype=torch.bfloat16).eval()
    ids = torch.randint(0, m.c.vocab_size, (2, 40), device=DEV)
    with torch.no_grad():
        full = m(ids).float()
        cache = m.new_cache(2, 40)
        lg = [m.step(ids[:, :32], cache, 0)]
        for t in range(32, 40):
            lg.append(m.step(ids[:, t:t + 1], cache, t))
    got = torch.stack(lg[1:], 1)                 # logits after tokens 32..39
    assert rel(lg[0], full[:, 31]) < 2e-2
    assert rel(got, full[:, 32:40]) < 2e-2


def test_gemma_mqa_cached_steps_match_full_forward():
    from solvingpapers_amd.models import gemma
    torch.manual_seed(0)
    m = gemma.Gemma(gemma.config("gemma_tiny"), device=DEV, dtype=torch.bfloat16).eval()
    ids = torch.randint(0, m.c.vocab_size, (1, 24), device=DEV)
    with torch.no_grad():
        full = m(ids).float()
        cache = m.new_cache(1, 24)
        lg = [m.step(ids[:, :16], cache, 0)] + [m.step(ids[:, t:t + 1], cache, t) for t in range(16, 24)]
    assert rel(torch.stack(lg[1:], 1), full[:, 16:24]) < 2e-2


def test_graph_decoder_matches_eager_logits():
    """HIP-graph decode (device-side positions, fused RoPE + KV cache write, kv_len decode
    kernel, state advanced inside the graph) == full forward, teacher-forced."""
    from solvingpapers_amd.infer import GraphDecoder
    from solvingpapers_amd.models import llama3
    torch.manual_seed(0)
    m = llama3.Llama3(llama3.config("llama3_tiny"), device=DEV, dtype=torch.bfloat16).eval()
    ids = torch.randint(0, m.c.vocab_size, (2, 40), device=DEV)
    with torch.no_grad():
        full = m(ids).float()
        dec = GraphDecoder(m, 2, 48)
        lg = [dec.prefill(ids[:, :24])]
        for t in range(24, 40):
            dec.ids.copy_(ids[:, t:t + 1])
            dec.graph.replay()
            lg.append(dec.logits.clone())
    assert rel(lg[0], full[:, 23]) < 2e-2
    assert rel(torch.stack(lg[1:], 1), full[:, 24:40]) < 2e-2
    out = dec.generate(ids[:, :10], 6)
    ref = m.generate(ids[:, :10], 6, greedy=True)
    assert out.shape == ref.shape and torch.equal(out[:, :11], ref[:, :11])


def test_gemma_graph_decoder_matches_full_forward():
    """MQA graph decode: rotate_half RoPE + cache write fused, hd 64 decode kernel, == the
    full forward teacher-forced."""
    from solvingpapers_amd.infer import GraphDecoder
    from solvingpapers_amd.models import gemma
    torch.manual_seed(0)
    m = gemma.Gemma(gemma.config("gemma_tiny"), device=DEV, dtype=torch.bfloat16).eval()
    ids = torch.randint(0, m.c.vocab_size, (2, 30), device=DEV)
    with torch.no_grad():
        full = m(ids).float()
        dec = GraphDecoder(m, 2, 40)
        lg = [dec.prefill(ids[:, :20])]
        for t in range(20, 30):
            dec.ids.copy_(ids[:, t:t + 1])
            dec.graph.replay()
            lg.append(dec.logits.clone())
    assert rel(lg[0], full[:, 19]) < 2e-2
    assert rel(torch.stack(lg[1:], 1), full[:, 20:30]) < 2e-2
