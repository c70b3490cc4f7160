"""DeepSeek-V3 (SURVEY §2.1.4, T2 parity): the notebook's own classes (cells defining
precompute_pos_embeddings .. DeepSeekV3, deepseekv3/deepseekv3.ipynb) are exec'd on CPU
with a small config; our model loads their state dict and must match logits, loss,
every gradient and the aux-free routing-bias update. The MLA (paper) family is checked
for cached-decode == full-forward, MTP, MoE op semantics and training progress."""
import sys
from dataclasses import dataclass

import pytest
import torch

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import refexec  # noqa: E402

from solvingpapers_amd.models import deepseekv3 as ds  # noqa: E402

NB = "deepseekv3/deepseekv3.ipynb"


class _Args:
    block_size = 16
    batch_size = 2
    embeddings_dim = 64
    attn_dropout = 0.0
    vocab_size = 97
    heads = 4
    dropout = 0.0
    decoder_layers = 2
    experts = 4
    top_experts = 2
    use_shared_experts = True
    noisy_topk = False
    use_aux_free_load_balancing = True
    aux_free_bias_update_rate = 0.001
    mtp_heads = 0
    latent_dim = 16
    device = "cpu"
    ignore_pad_token_in_loss = False


def _ref_model(noisy=False):
    from torch.nn import RMSNorm
    args = type("_NoisyArgs", (_Args,), {"noisy_topk": True}) if noisy else _Args
    ns = refexec.exec_cells(NB, ["precompute_pos_embeddings", "apply_pos_embeddings", "Normalization", "swish",
                                 "SWiGLUExpert", "MoeLayer", "LatentAttention", "MHLA", "DecoderLayer", "Block",
                                 "DeepSeekV3"], {"modelargs": args, "RMSNorm": RMSNorm, "dataclass": dataclass})
    torch.manual_seed(0)
    ref = ns["DeepSeekV3"](embeddings_dim=64, vocab_size=97, dropout=0.0, mtp_heads=0, device="cpu")
    with torch.no_grad():
        for l in ref.decoder.decoder:
            l.moe_block.routing_bias.uniform_(-0.01, 0.01)
    return ref


def _ours(noisy=False):
    c = ds.config("dsv3_ref", vocab_size=97, block_size=16, dim=64, n_layers=2, n_heads=4, latent_dim=16,
                  n_experts=4, top_k=2, dropout=0.0, attn_dropout=0.0, noisy_topk=noisy)
    return ds.DeepSeekV3(c)


pytestmark = pytest.mark.skipif(not refexec.available(NB), reason="reference not mounted")


def test_dsv3_ref_state_dict_and_logits():
    ref, m = _ref_model(), _ours()
    sd = ref.state_dict()
    m.from_reference_state_dict(sd)
    out = m.to_reference_state_dict()
    assert set(sd) == set(out)
    for k in sd:
        assert sd[k].shape == out[k].shape and torch.equal(sd[k].float(), out[k]), k
    x = torch.randint(0, 97, (2, 16), generator=torch.Generator().manual_seed(1))
    ref.eval()
    m.eval()
    with torch.no_grad():
        a, b = ref(x, inference=True), m(x)
    assert torch.allclose(a, b, atol=1e-5), (a - b).abs().max()


def test_dsv3_ref_training_grads_and_bias_update():
    import torch.nn.functional as F
    ref, m = _ref_model(), _ours()
    m.from_reference_state_dict(ref.state_dict())
    ref.train()
    m.train()
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 97, (2, 16), generator=g)
    y = torch.randint(0, 97, (2, 16), generator=g)
    logits = ref(x)                               # training path: MTP loop inert -> plain decoder
    lr = F.cross_entropy(logits.view(-1, 97), y.view(-1))
    lr.backward()
    lo = m(x, y)
    lo.backward()
    assert abs(lr.item() - lo.item()) < 1e-5
    # routing bias updated once by the soft-mass rule in both
    for i, l in enumerate(ref.decoder.decoder):
        assert torch.allclose(l.moe_block.routing_bias, m.layers[i].ffn.routing_bias, atol=1e-7)
    # gradients: tied embedding, attention, experts, gate, shared expert
    assert torch.allclose(ref.decoder.embeddings.weight.grad, m.embed.grad, atol=1e-5)
    for i, l in enumerate(ref.decoder.decoder):
        a = m.layers[i].attn
        for h in range(4):
            rh = l.mhla.heads[h]
            assert torch.allclose(rh.query.weight.grad, a.wq.grad[h], atol=1e-5)
            assert torch.allclose(rh.W_k.weight.grad, a.wk.grad[h], atol=1e-5)
            assert torch.allclose(rh.W_v.weight.grad, a.wv.grad[h], atol=1e-5)
            if i == 0 and h == 0:
                assert torch.allclose(rh.W_dkv.weight.grad, a.wdkv.grad[0], atol=1e-5)
        mo = m.layers[i].ffn
        assert torch.allclose(l.moe_block.gate.weight.grad, mo.gate.grad, atol=1e-5)
        F_ = mo.F
        for e in range(4):
            ex = l.moe_block.experts[e]
            if ex.w1.weight.grad is None:
                continue
            assert torch.allclose(ex.w1.weight.grad, mo.w13.grad[e, :F_], atol=1e-5)
            assert torch.allclose(ex.w2.weight.grad, mo.w13.grad[e, mo.Fp:mo.Fp + F_], atol=1e-5)
            assert torch.allclose(ex.w3.weight.grad, mo.w2.grad[e, :, :F_], atol=1e-5)
            assert mo.w13.grad[e, F_:mo.Fp].abs().max() == 0          # padding stays inert
        sh = l.moe_block.shared_expert
        assert torch.allclose(sh.w1.weight.grad, mo.shared.w13.grad[:F_], atol=1e-5)


def test_dsv3_ref_noisy_topk_matches_reference():
    """noisy_topk=True (deepseekv3.ipynb:390,1026-1039): the extra ``noise`` Linear round-trips
    through the reference state dict, and with the same torch RNG state both models draw the
    same N(0,1) noise per (token, expert) in the same order -> equal logits, loss, gate / noise
    gradients and routing-bias update. The noise is on in eval too, as in the reference."""
    import torch.nn.functional as F
    ref, m = _ref_model(noisy=True), _ours(noisy=True)
    sd = ref.state_dict()
    assert any(k.endswith("moe_block.noise.weight") for k in sd)
    m.from_reference_state_dict(sd)
    out = m.to_reference_state_dict()
    assert set(sd) == set(out)
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 97, (2, 16), generator=g)
    y = torch.randint(0, 97, (2, 16), generator=g)
    ref.eval()
    m.eval()
    with torch.no_grad():
        torch.manual_seed(11)
        a = ref(x, inference=True)
        torch.manual_seed(11)
        b = m(x)
        torch.manual_seed(12)
        c = m(x)
    assert torch.allclose(a, b, atol=1e-5), (a - b).abs().max()
    assert not torch.allclose(b, c, atol=1e-6)                      # a different draw moves the routing
    ref.train()
    m.train()
    torch.manual_seed(13)
    lr = F.cross_entropy(ref(x).view(-1, 97), y.view(-1))
    lr.backward()
    torch.manual_seed(13)
    lo = m(x, y)
    lo.backward()
    assert abs(lr.item() - lo.item()) < 1e-5
    for i, l in enumerate(ref.decoder.decoder):
        mo = m.layers[i].ffn
        assert torch.allclose(l.moe_block.routing_bias, mo.routing_bias, atol=1e-7)
        assert torch.allclose(l.moe_block.gate.weight.grad, mo.gate.grad, atol=1e-5)
        assert torch.allclose(l.moe_block.noise.weight.grad, mo.noise.grad, atol=1e-5)


def test_dsv3_ref_cached_generate_matches_recompute():
    m = _ours().eval()
    x = torch.randint(0, 97, (1, 5), generator=torch.Generator().manual_seed(4))
    out = m.generate(x, 6, greedy=True)
    cur = x
    for _ in range(6):
        nxt = m(cur)[:, -1].argmax(-1, keepdim=True)
        cur = torch.cat([cur, nxt], 1)
    assert torch.equal(out, cur)


# ---------------------------------------------------------------- paper-style MLA family
def _tiny(**kw):
    return ds.DeepSeekV3(ds.config("dsv3_tiny", **kw), seed=0)


def test_mla_cached_decode_matches_full_forward():
    m = _tiny().eval()
    x = torch.randint(0, 512, (2, 9), generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        full = m(x)
        caches = m.new_cache(2, 9)
        n1, _ = m.hidden(x[:, :4], caches, 0)
        n2, _ = m.hidden(x[:, 4:], caches, 4)
        inc = torch.cat([m.logits(n1), m.logits(n2)], 1)
    assert torch.allclose(full, inc, atol=1e-4), (full - inc).abs().max()


def test_mla_moe_training_reduces_loss_and_balances():
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    m = _tiny()
    flat = FlatParams(m, groups=m.param_groups())
    opt = FlatAdamW(flat, lr=3e-3, weight_decay=0.0, max_grad_norm=1.0)
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 64, (4, 33), generator=g)           # learnable: small support
    losses = []
    for _ in range(25):
        opt.zero_grad()
        loss = m(x[:, :-1], x[:, 1:])
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 1.0, losses
    bias = m.moe_layers()[0].routing_bias
    assert bias.abs().max() > 0                                # counts rule moved the bias
    assert m.c.mtp_heads == 1 and len(m.mtp_layers) == 1


def test_moe_ops_match_dense_loop():
    from solvingpapers_amd.ops import moe as M
    torch.manual_seed(0)
    N, D, F, E, k = 37, 16, 24, 5, 2
    x = torch.randn(N, D, dtype=torch.float64, requires_grad=True)
    logits = torch.randn(N, E, dtype=torch.float64, requires_grad=True)
    bias = torch.randn(E) * 0.1
    W13 = torch.randn(E, 2 * F, D, dtype=torch.float64, requires_grad=True)
    W2 = torch.randn(E, D, F, dtype=torch.float64, requires_grad=True)
    idx, w = M.route(logits, k, bias, bias_in_weights=False)
    y, plan = M.moe_ffn(x, idx, w.double(), W13, W2)
    # dense loop oracle
    sel = torch.topk(logits.detach().float() + bias, k).indices
    assert torch.equal(sel.int(), idx)
    ws = torch.softmax(logits.gather(1, idx.long()), -1)
    ref = torch.zeros(N, D, dtype=torch.float64)
    for n in range(N):
        for j in range(k):
            e = int(idx[n, j])
            h = x[n] @ W13[e].t()
            a = torch.nn.functional.silu(h[:F]) * h[F:]
            ref[n] += ws[n, j] * (a @ W2[e].t())
    assert torch.allclose(y, ref, rtol=1e-5, atol=1e-5)    # gate weights are fp32
    assert plan.counts.sum() == N * k and int(plan.offsets[-1]) == N * k
    gy = torch.randn(N, D, dtype=torch.float64)
    ga = torch.autograd.grad(y, [x, logits, W13, W2], gy)
    gr = torch.autograd.grad(ref, [x, logits, W13, W2], gy)
    for a, b in zip(ga, gr):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("aux_free", [False, True])
def test_trainer_pairs_microbatches_like_one_by_one(aux_free):
    """Trainer.pair_microbatches (DeepSeekV3.forward_pair on each two micro-batches of an even
    grad_accum) trains to the same parameters -- and, with aux-free balancing, the same routing
    biases -- as the one-by-one loop. (At EP 1 the Trainer would not pair: forced here.)"""
    from solvingpapers_amd.train.trainer import TrainConfig, Trainer
    c = ds.config("dsv3_tiny", dropout=0.0, attn_dropout=0.0, aux_free=aux_free)
    gen = torch.Generator().manual_seed(1)
    ids = torch.randint(0, c.vocab_size, (8, 2, 33), generator=gen)
    params, biases = [], []
    for pair in (False, True):
        m = ds.DeepSeekV3(c, seed=0)
        assert not m.pair_overlaps()                       # EP 1: nothing to hide
        m.pair_overlaps = lambda: True
        tr = Trainer(m, TrainConfig(steps=2, grad_accum=4, lr=1e-3, pair_microbatches=pair),
                     lambda i: (ids[i, :, :-1], ids[i, :, 1:]))
        tr.fit()
        params.append(tr.flat.param.clone())
        biases.append(torch.cat([l.routing_bias for l in m.moe_layers()]))
    assert torch.allclose(params[0], params[1], atol=1e-5)     # summation order only
    assert torch.equal(biases[0], biases[1])
    if aux_free:
        assert biases[0].abs().max() > 0


def test_trainer_does_not_pair_without_overlap():
    """Pairing keeps two micro-batches' activations alive; the Trainer does it only when the
    model reports an overlap (pair_overlaps): at EP 1 / TP 1 it runs them one by one."""
    from solvingpapers_amd.train.trainer import TrainConfig, Trainer
    c = ds.config("dsv3_tiny", dropout=0.0, attn_dropout=0.0)
    ids = torch.randint(0, c.vocab_size, (4, 2, 17))
    m = ds.DeepSeekV3(c, seed=0)
    calls = []
    m.forward_pair = lambda *a: calls.append(1)
    Trainer(m, TrainConfig(steps=1, grad_accum=2, lr=1e-3), lambda i: (ids[i, :, :-1], ids[i, :, 1:])).fit()
    assert not calls


@pytest.mark.parametrize("which", ["dsv3", "llama3"])
def test_forward_waits_for_every_optimizer_bucket(which):
    """An overlapped optimizer updates bucket i on a side stream and the model must wait for it
    (param_wait_cb) before reading bucket i's parameters: one training forward waits for EVERY
    bucket of param_groups() -- DeepSeek-V3's expert buckets included."""
    from solvingpapers_amd.models import llama3
    if which == "dsv3":
        c = ds.config("dsv3_tiny", dropout=0.0, attn_dropout=0.0)
        m = ds.DeepSeekV3(c, seed=0)
        V = c.vocab_size
    else:
        c = llama3.config("llama3_tiny")
        m = llama3.Llama3(c)
        V = c.vocab_size
    seen = []
    m.param_wait_cb = seen.append
    ids = torch.randint(0, V, (2, 17))
    m(ids[:, :-1], ids[:, 1:])
    assert sorted(set(seen)) == list(range(len(m.param_groups())))
    # ...and through FlatParams.group_waiter every BUCKET is waited for, also when a frozen group
    # vanishes from the buckets (group index != bucket index)
    from solvingpapers_amd.utils.flat import FlatParams
    groups = m.param_groups()
    for p in groups[1]:
        p.requires_grad_(False)
    flat = FlatParams(m, groups=groups, hook_autograd=False)
    waited = []
    flat.wait_bucket = waited.append
    m.param_wait_cb = flat.group_waiter(groups)
    m(ids[:, :-1], ids[:, 1:])
    assert sorted(set(waited)) == [b.index for b in flat.buckets]


def test_stale_checkpoint_preset():
    """dsv3_ref_stale = the notebook's .ipynb_checkpoints copy (block 512, batch 32, one MTP head;
    deepseekv3/.ipynb_checkpoints/deepseekv3-checkpoint.ipynb:53-80); a shrunken copy trains one
    step through the MTP path."""
    c = ds.config("dsv3_ref_stale")
    ref = ds.config("dsv3_ref")
    assert (c.block_size, c.batch_size, c.mtp_heads) == (512, 32, 1)
    assert (c.dim, c.n_layers, c.n_heads, c.n_experts, c.top_k, c.latent_dim) == \
        (ref.dim, ref.n_layers, ref.n_heads, ref.n_experts, ref.top_k, ref.latent_dim)
    m = ds.DeepSeekV3(ds.config("dsv3_ref_stale", vocab_size=97, block_size=24, dim=64, n_layers=2, n_heads=4,
                                latent_dim=16, n_experts=4), seed=0)
    ids = torch.randint(0, 97, (2, 25))
    loss = m(ids[:, :-1], ids[:, 1:])
    loss.backward()
    assert torch.isfinite(loss)
    assert m.mtp_proj.grad is not None and torch.isfinite(m.mtp_proj.grad).all()   # the MTP head trained
