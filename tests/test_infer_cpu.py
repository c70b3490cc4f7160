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
    ids = torch.randint(0, 60, (1, 3))
    out = generate(m, ids, 12, greedy=True)
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
