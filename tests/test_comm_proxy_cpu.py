"""parallel/comm.py: the one-GPU stand-in group drives the TP / EP code paths unchanged (here on
the CPU, where it models no time): an 8-rank sequence-parallel TP Gemma and an 8-rank EP
DeepSeek-V3 run forward + backward on local shard shapes, plain and as overlapped pairs, and
the pairs give the same result as the plain forms."""
import torch

from solvingpapers_amd.parallel.comm import ProxyGroup, group_rank_size


import pytest


@pytest.mark.parametrize("nb", [2, 1])
def test_proxy_group_tp_gemma_pair_matches_plain(nb):
    """TP=8 sequence-parallel Gemma on the stand-in group: the overlapped chunk pair (batch
    halves, or sequence halves) == the plain SP forward, and its all-gathers / reduce-scatters
    ran. (The stand-in's gather replicates this rank's shard, so the sequence split -- whose
    halves gather different tokens -- is checked for running, not for equality.)"""
    from solvingpapers_amd.models import gemma
    from solvingpapers_amd.utils.flat import FlatParams
    c = gemma.config("gemma_tiny", vocab_size=64, dim=64, n_heads=8, head_dim=16, ffn_hidden=128)
    g1 = ProxyGroup(8, "cpu")
    assert group_rank_size(g1) == (0, 8)
    plain = gemma.Gemma(c, tp_group=g1, seed=3, tp_pipeline=False)
    pair = gemma.Gemma(c, tp_group=g1, seed=3)
    assert plain.sp and pair.sp and plain.layers[0].hl == 1 and plain.embed.shape[0] == 8   # TP=8 local shards
    ids = torch.randint(0, 64, (2, 17), generator=torch.Generator().manual_seed(0))[:nb]
    grads = []
    for m in (plain, pair):
        FlatParams(m)
        m.train()
        g1.reset_stats()
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        assert g1.calls > 0
        grads.append((loss.item(), {n: p.main_grad.clone() for n, p in m.named_parameters()}))
    assert pair._pair_split(ids[:, :-1]) == ("batch" if nb == 2 else "sequence")
    if nb == 1:
        return
    assert abs(grads[0][0] - grads[1][0]) < 1e-5
    for n, g in grads[0][1].items():
        assert torch.allclose(g, grads[1][1][n], atol=1e-5, rtol=1e-4), n


def test_proxy_group_ep_forward_pair_matches_plain():
    """EP=8 on the stand-in group: DeepSeekV3.forward_pair (micro-batches interleaved) == two
    plain forward() calls -- loss and expert / dense gradients -- and the exchanges ran."""
    from solvingpapers_amd.models import deepseekv3 as ds
    from solvingpapers_amd.utils.flat import FlatParams
    c = ds.config("dsv3_tiny", vocab_size=64, dim=32, n_heads=2, kv_lora_rank=16, qk_nope_dim=8, qk_rope_dim=8,
                  v_head_dim=16, n_experts=16, top_k=2, n_shared=1, expert_hidden=24, dense_hidden=48, n_layers=2,
                  n_dense_layers=1, aux_free=False, mtp_heads=0)
    g1 = ProxyGroup(8, "cpu")
    ids = torch.randint(0, 64, (2, 2, 13), generator=torch.Generator().manual_seed(1))
    outs = []
    for pair in (False, True):
        m = ds.DeepSeekV3(c, seed=3, ep_group=g1)
        assert m.layers[1].ffn.w13.shape[0] == 2                       # 16 experts / EP 8
        FlatParams(m)
        x0, y0, x1, y1 = ids[0, :, :-1], ids[0, :, 1:], ids[1, :, :-1], ids[1, :, 1:]
        loss = m.forward_pair(x0, y0, x1, y1) if pair else m(x0, y0) + m(x1, y1)
        loss.backward()
        outs.append((loss.item(), {n: p.main_grad.clone() for n, p in m.named_parameters()}))
    assert abs(outs[0][0] - outs[1][0]) < 1e-5
    for n, g in outs[0][1].items():
        assert torch.allclose(g, outs[1][1][n], atol=1e-5, rtol=1e-4), n
    assert g1.calls > 0


def test_proxy_group_synth_gather_shape_and_cache():
    """synth_gather: the stand-in all-gather returns one cached random buffer per gathered shape
    (no concatenation on the caller's stream); off: the shard replicated tp times."""
    x = torch.arange(6.0).reshape(1, 3, 2)
    g = ProxyGroup(4, "cpu")
    assert torch.equal(g.gathered(x, 1), torch.cat([x] * 4, dim=1))
    gs = ProxyGroup(4, "cpu", synth_gather=True)
    a, b = gs.gathered(x, 1), gs.gathered(x + 1, 1)
    assert a.shape == (1, 12, 2) and a is b and a.std() > 0
