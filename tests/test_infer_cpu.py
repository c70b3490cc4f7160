"""Inference layer (solvingpapers_amd/infer): KV-cached generation must reproduce the
reference's full re-forward decoding token for token (gpt/gpt-jax.ipynb:821-829 style
greedy argmax), plus sampler semantics."""
import pytest
import torch

from solvingpapers_amd.infer import GenerationStats, KVCache, generate, sample
from solvingpapers_amd.models import deepseekv3, gemma, gpt, llama3


def _greedy_reforward(model, ids, n):
    out = ids
    with torch.no_grad():
        for _ in range(n):
            out = torch.cat([out, model(out)[:, -1].argmax(-1, keepdim=True)], 1)
    return out


@pytest.mark.parametrize("family", ["llama3", "gemma", "dsv3", "dsv3_ref"])
def test_cached_generation_matches_reforward(family):
    torch.manual_seed(0)
    if family == "llama3":
        m = llama3.Llama3(llama3.config("llama3_tiny", vocab_size=128, dim=64, n_heads=4, n_kv_heads=2,
                                        ffn_hidden=128, max_seq_len=64))
    elif family == "gemma":
        m = gemma.Gemma(gemma.config("gemma_tiny", vocab_size=128, dim=64, n_heads=4, head_dim=16,
                                     ffn_hidden=128, max_seq_len=64))
    elif family == "dsv3":
        m = deepseekv3.DeepSeekV3(deepseekv3.config("dsv3_tiny"))
    else:
        m = deepseekv3.DeepSeekV3(deepseekv3.config("dsv3_ref", vocab_size=97, block_size=32, dim=64, n_layers=2,
                                                    n_heads=4, latent_dim=16, n_experts=4, top_k=2))
    m.eval()
    ids = torch.randint(0, 90, (2, 5))
    st = GenerationStats()
    out = m.generate(ids, 9, greedy=True, stats=st)
    assert st.cached and st.new_tokens == 18 and st.prompt_tokens == 10
    assert torch.equal(out, _greedy_reforward(m, ids, 9))


def test_generic_driver_uncached_model_crops_window():
    torch.manual_seed(0)
    m = gpt.GPT(gpt.config("gpt_tiny_cpu", block_size=8)).eval()

    class Uncached(torch.nn.Module):       # forward only: no new_cache / step protocol
        def __init__(self, inner):
            super().__init__()
            self.inner, self.c = inner, inner.c

        def forward(self, x):
            return self.inner(x)

    ids = torch.randint(0, 60, (1, 3))
    out = generate(Uncached(m).eval(), ids, 12, greedy=True)
    assert out.shape == (1, 15)
    ref = ids
    with torch.no_grad():
        for _ in range(12):
            ref = torch.cat([ref, m(ref[:, -8:])[:, -1].argmax(-1, keepdim=True)], 1)
    assert torch.equal(out, ref)


def test_generation_stops_at_context_limit():
    m = llama3.Llama3(llama3.config("llama3_tiny", vocab_size=64, dim=32, n_heads=2, n_kv_heads=1,
                                    ffn_hidden=64, max_seq_len=12))
    out = m.generate(torch.zeros(1, 10, dtype=torch.long), 20, greedy=True)
    assert out.shape[1] == 13  # 2 fed through the cache + the last sampled token


def test_eos_stops_and_pads():
    class Stub(torch.nn.Module):
        def new_cache(self, B, T):
            return None
        def step(self, ids, cache, pos):
            lg = torch.full((ids.shape[0], 10), -10.0)
            lg[:, 3] = 10.0  # always emits token 3
            return lg
    out = generate(Stub(), torch.zeros(2, 2, dtype=torch.long), 50, greedy=True, eos_token_id=3)
    assert out.shape[1] <= 2 + 16 and (out[:, 2:] == 3).all()


def test_samplers():
    g = torch.Generator().manual_seed(0)
    lg = torch.tensor([[0.0, 5.0, 1.0, -2.0]])
    assert sample(lg, greedy=True).item() == 1
    for _ in range(20):
        assert sample(lg, top_k=1, generator=g).item() == 1
        assert sample(lg, top_p=1e-6, generator=g).item() == 1      # nucleus keeps the top token
        assert sample(lg, top_k=2, generator=g).item() in (1, 2)
    counts = torch.bincount(torch.cat([sample(lg.expand(512, 4), temperature=100.0, generator=g)
                                       for _ in range(4)]).view(-1), minlength=4)
    assert (counts > 200).all()  # high temperature ~ uniform


def test_kv_cache_write_and_overflow():
    c = KVCache(2, 1, 4, 2, 8, dtype=torch.float32)
    k = torch.randn(1, 3, 2, 8)
    kv, vv = c.write(1, k, -k, 0)
    assert kv.shape == (1, 3, 2, 8) and torch.equal(kv, k) and torch.equal(vv, -k)
    assert c.nbytes() == 2 * 2 * 4 * 2 * 8 * 4
    with pytest.raises(ValueError):
        c.write(0, torch.randn(1, 2, 2, 8), torch.randn(1, 2, 2, 8), 3)


def test_topk_sampling_single_cached_call_and_eos_stop():
    """api.topk_sampling (deepseekv3.ipynb:1849-1873) runs ONE cached generate call: with
    top_k=1 it equals the reference's per-token full re-forward, and it stops right after EOS."""
    from solvingpapers_amd import api
    from solvingpapers_amd.models import deepseekv3 as ds
    m = ds.DeepSeekV3(ds.config("dsv3_tiny"), seed=0).eval()
    calls = {"n": 0}
    orig = m.generate

    def counted(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    m.generate = counted
    x = torch.randint(0, 512, (1, 4), generator=torch.Generator().manual_seed(0))
    out = api.topk_sampling(m, x, max_length=12, top_k=1)
    assert calls["n"] == 1 and out.shape == (1, 12)
    cur = x
    with torch.no_grad():
        for _ in range(8):
            cur = torch.cat([cur, m(cur)[:, -1].argmax(-1, keepdim=True)], 1)
    assert torch.equal(out, cur)
    eos = int(cur[0, 6])                         # the 3rd generated token
    first = int((cur[0, 4:] == eos).nonzero()[0, 0]) + 4
    out2 = api.topk_sampling(m, x, max_length=12, top_k=1, eos_token_id=eos)
    assert torch.equal(out2, cur[:, :first + 1])


def test_gpt_cached_generate_matches_window_reforward():
    """GPT now has a KV cache (learned positions): cached greedy decoding equals the reference's
    crop-and-re-forward loop (gpt/gpt-jax.ipynb:821-829), including past block_size where the
    window slides and the tail falls back to re-forwarding."""
    from solvingpapers_amd.models import gpt
    c = gpt.config("gpt_ref", num_layers=2, block_size=24, emb_dim=64)
    m = gpt.GPT(c, seed=0).eval()
    x = torch.randint(0, 65, (2, 5), generator=torch.Generator().manual_seed(1))
    out = m.generate(x, 30)
    cur = x
    with torch.no_grad():
        for _ in range(30):
            cur = torch.cat([cur, m(cur[:, -24:])[:, -1].argmax(-1, keepdim=True)], 1)
    assert torch.equal(out, cur)
    assert m.new_cache(2, 24)[0][0].shape == (2, 24, 1, 64)
