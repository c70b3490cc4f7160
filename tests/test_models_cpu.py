"""Model parity against the reference's own code (exec'd from the notebooks on CPU)
and CPU training smoke tests for the catalogue (SURVEY §4.2 tiers T2/T3)."""
import math

import pytest
import torch

import refexec


def _load_sd(ours, ref_sd, strict=True):
    missing, unexpected = ours.load_state_dict(ref_sd, strict=strict)
    return missing, unexpected


@pytest.mark.skipif(not refexec.available("gemma/gemma.ipynb"), reason="reference not mounted")
def test_gemma_ref_parity():
    from solvingpapers_amd.models import gemma
    class args:  # small config, reference semantics (gemma.ipynb:27-43)
        block_size = 16; batch_size = 2; embeddings_dims = 64; attn_dropout = 0.1; no_of_heads = 4
        dropout = 0.1; epochs = 1; max_lr = 2.5e-4; no_of_decoder_layers = 2; weight_decay_optim = 0.1
        beta_1 = 0.9; beta_2 = 0.95; device = "cpu"; no_kv_heads = 2; vocab_size = 30
    ns = refexec.exec_cells("gemma/gemma.ipynb", ["RMSNorm", "RotaryEmbeddings", "MQA", "GeGLU", "FFN",
                                                   "DecoderLayer", "Gemma"], {"args": args})
    torch.manual_seed(0)
    ref = ns["Gemma"](embeddings_dims=64, block_size=16, vocab_size=30, dropout=0.1).eval()
    c = gemma.GemmaRefConfig(block_size=16, embeddings_dims=64, no_of_heads=4, no_kv_heads=2, vocab_size=30,
                             no_of_decoder_layers=2)
    ours = gemma.GemmaRef(c).eval()
    ours.load_state_dict(ref.state_dict())
    x = torch.randint(0, 30, (2, 16))
    assert torch.allclose(ours(x), ref(x), atol=1e-4, rtol=1e-4)
    x = torch.randint(0, 30, (2, 11))  # T < block_size
    assert torch.allclose(ours(x), ref(x), atol=1e-4, rtol=1e-4)


def test_gemma_ref_param_count():
    from solvingpapers_amd.models import gemma
    assert sum(p.numel() for p in gemma.GemmaRef().parameters()) == 127_521_089  # gemma.ipynb:495


@pytest.mark.skipif(not refexec.available("vision transformer/ViT.ipynb"), reason="reference not mounted")
def test_vit_parity():
    from solvingpapers_amd.models import vit
    g = dict(num_classes=10, batch_size=4, num_channels=1, image_size=28, patch_size=7, num_patches=16,
             embedding_dim=64, attention_heads=4, transformer_blocks=4, learning_rate=1e-3, epochs=1,
             mlp_hidden_nodes=128)
    ns = refexec.exec_cells("vision transformer/ViT.ipynb", ["PatchEmbedding", "TransformerEncoder", "MLPHead", "ViT"], g)
    torch.manual_seed(0)
    ref = ns["ViT"]().eval()
    ours = vit.ViT(vit.config("vit_mnist_ref")).eval()
    ours.load_state_dict(ref.state_dict())
    x = torch.rand(3, 1, 28, 28)
    assert torch.allclose(ours(x), ref(x), atol=1e-4, rtol=1e-4)


@pytest.mark.skipif(not refexec.available("autoencoder/autoencoder.ipynb"), reason="reference not mounted")
def test_ae_vae_parity():
    from solvingpapers_amd.models import autoencoder as A
    ns = refexec.exec_cells("autoencoder/autoencoder.ipynb", ["AutoEncoder"])
    ref = ns["AutoEncoder"]()
    ours = A.AutoEncoder()
    ours.load_state_dict(ref.state_dict())
    x = torch.rand(5, 784)
    assert torch.allclose(ours(x), ref(x), atol=1e-6)
    ns = refexec.exec_cells("autoencoder/variational autoencoder.ipynb", ["VAE", "vae_loss"])
    ref = ns["VAE"]()
    ours = A.VAE()
    ours.load_state_dict(ref.state_dict())
    torch.manual_seed(3)
    r1, mu1, lv1 = ref(x)
    torch.manual_seed(3)
    r2, mu2, lv2 = ours(x)
    assert torch.allclose(r1, r2, atol=1e-6) and torch.allclose(mu1, mu2) and torch.allclose(lv1, lv2)
    from solvingpapers_amd.ops.misc import vae_loss
    assert torch.allclose(vae_loss(r2, x, mu2, lv2), ns["vae_loss"](r1, x, mu1, lv1), rtol=1e-5)


def test_kd_alexnet_luong_parity():
    import importlib.util, os
    from solvingpapers_amd.models import alexnet, kd, luong
    path = os.path.join(refexec.REF, "knowledge distillation/kd.py")
    if not os.path.exists(path):
        pytest.skip("reference not mounted")
    src = open(path).read()
    src = src.split("# data")[0].replace("from torchvision import datasets, transforms", "")
    ns = {}
    exec(compile(src, path, "exec"), ns)
    s, t = ns["Student"](), ns["Teacher"]()
    os_, ot = kd.Student(), kd.Teacher()
    os_.load_state_dict(s.state_dict()); ot.load_state_dict(t.state_dict())
    x = torch.rand(4, 1, 28, 28)
    assert torch.allclose(os_(x), s(x), atol=1e-5) and torch.allclose(ot(x), t(x), atol=1e-5)
    y = torch.randint(0, 10, (4,))
    a = ns["distillation_loss"](s(x), t(x), y, 7, 0.3)
    b = kd.distillation_loss(s(x), t(x), y, 7, 0.3)
    for u, v in zip(a, b):
        assert torch.allclose(u, v, atol=1e-6)
    asrc = open(os.path.join(refexec.REF, "alexnet/alexnet.py")).read()
    ans = {}
    exec(compile(asrc, "alexnet.py", "exec"), ans)
    ra = ans["AlexNet"](10).eval()
    oa = alexnet.AlexNet(10).eval()
    oa.load_state_dict(ra.state_dict())
    x = torch.rand(1, 3, 224, 224)
    assert torch.allclose(oa(x), ra(x), atol=1e-4)
    assert sum(p.numel() for p in oa.parameters()) == 46_787_978
    lns = refexec.exec_cells("attention/luong.ipynb", ["LuongAttention"])
    st, hs = torch.randn(3, 8), torch.randn(3, 5, 8)
    c1, w1 = lns["LuongAttention"](8)(st, hs)
    c2, w2 = luong.LuongAttention(8)(st, hs)
    assert torch.allclose(c1, c2, atol=1e-6) and torch.allclose(w1, w2, atol=1e-6)


def test_activation_value_table_matches_numpy_reference():
    import numpy as np
    from solvingpapers_amd.models import activations as A
    t = A.value_table()
    ref = A.numpy_reference()
    x = t["x"].numpy()
    assert np.allclose(t["relu"].numpy(), ref["relu"](x))
    assert np.allclose(t["leakyrelu"].numpy(), ref["leakyrelu"](x))
    assert np.allclose(t["prelu"].numpy(), ref["prelu"](x, 0.3))
    assert np.allclose(t["elu"].numpy(), ref["elu"](x, 0.4), atol=1e-6)
    assert np.allclose(t["gelu"].numpy(), ref["gelu"](x), atol=1e-5)


def test_gpt_counts_and_training():
    from solvingpapers_amd.models import gpt
    assert gpt.GPT(gpt.config("gpt_ref")).num_params() == 6_411_264
    from solvingpapers_amd.train.optim import FlatAdamW
    from solvingpapers_amd.utils.flat import FlatParams
    from solvingpapers_amd.data import CharTokenizer, get_batch, synthetic_corpus
    text = synthetic_corpus(20000)
    tok = CharTokenizer(text)
    data = torch.tensor(tok.encode(text))
    c = gpt.config("gpt_tiny_cpu", vocab_size=tok.vocab_size)
    m = gpt.GPT(c)
    flat = FlatParams(m, groups=m.param_groups())
    opt = FlatAdamW(flat, lr=3e-3, weight_decay=0.01)
    g = torch.Generator().manual_seed(0)
    losses = []
    for _ in range(60):
        x, y = get_batch(data, c.batch_size, c.block_size, g)
        opt.zero_grad()
        loss = m(x, y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 1.0, (losses[0], losses[-1])
    out = m.generate(torch.tensor([tok.encode("ROMEO:\n")]), 20)
    assert len(tok.decode(out[0].tolist())) == 27


def test_gpt_flax_layout_round_trip():
    from solvingpapers_amd.models import gpt
    a = gpt.GPT(gpt.config("gpt_tiny_cpu"), seed=1)
    b = gpt.GPT(gpt.config("gpt_tiny_cpu"), seed=2).from_reference_params(a.to_reference_params())
    for x, y in zip(a.parameters(), b.parameters()):
        assert torch.equal(x, y)
    d = a.to_reference_params()
    assert d["layers_0/attn/qkv/kernel"].shape == (128, 384) and d["lm_head/kernel"].shape == (128, 65)


def test_gpt_matches_flax_reference_math_fp64():
    """Numeric parity with gpt/gpt-jax.ipynb:321-472 (restated in fp64, tests/refimpl.py gpt_forward:
    fused QKV (in, out) kernel split q|k|v, -1e4 causal fill, tanh GELU, flax LayerNorm eps 1e-6,
    learned pos_embed, untied bias-free head) and its loss (:499-503), at gpt_ref widths (D256, one
    256-wide head, V65, T256) with 2 layers: the same Flax pytree loaded into models/gpt.py through
    from_reference_params gives equal logits and loss (rel <= 1e-10) and equal gradients."""
    from refimpl import gpt_forward, gpt_loss
    from solvingpapers_amd.models import gpt
    c = gpt.config("gpt_ref", num_layers=2)
    src = gpt.GPT(c, dtype=torch.float64, seed=3)
    d = src.to_reference_params(dtype=None)
    m = gpt.GPT(c, dtype=torch.float64, seed=9).from_reference_params(d).eval()
    ids = torch.randint(0, c.vocab_size, (2, c.block_size + 1), generator=torch.Generator().manual_seed(1))
    x, y = ids[:, :-1], ids[:, 1:]
    dr = {k: v.clone().requires_grad_(True) for k, v in d.items()}
    ref_logits = gpt_forward(dr, x, c.num_heads, c.num_layers)
    ref_loss = gpt_loss(ref_logits, y)
    ref_loss.backward()
    with torch.no_grad():
        logits = m(x)
    rel = ((logits - ref_logits.detach()).norm() / ref_logits.detach().norm()).item()
    assert logits.dtype == torch.float64 and rel <= 1e-10, rel
    loss = m(x, y)
    assert abs(loss.item() - ref_loss.item()) <= 1e-10 * abs(ref_loss.item()), (loss.item(), ref_loss.item())
    loss.backward()
    saved = {n: p.detach().clone() for n, p in m.named_parameters()}
    with torch.no_grad():                       # the gradients in the pytree layout
        for p in m.parameters():
            p.copy_(p.grad)
        grads = m.to_reference_params(dtype=None)
        for n, p in m.named_parameters():
            p.copy_(saved[n])
    for k, g in grads.items():
        want = dr[k].grad
        r = ((g - want).norm() / want.norm().clamp_min(1e-300)).item()
        assert r <= 1e-9, (k, r)


@pytest.mark.parametrize("kind", ["ae", "vae"])
def test_autoencoder_training_cpu(kind):
    from solvingpapers_amd.models import autoencoder as A
    _, hist = A.train(A.AEConfig(kind=kind, epochs=2, n_train=512, batch_size=64, device="cpu"), log=lambda *a: None)
    assert hist[-1] < hist[0]


def test_kd_and_vit_training_cpu():
    from solvingpapers_amd.models import kd, vit
    _, _, hist = kd.train(kd.KDConfig(epochs=2, teacher_epochs=1, n_train=1024, n_test=256, device="cpu"),
                          log=lambda *a: None)
    assert hist[-1][1] > 50.0  # synthetic MNIST-like digits are learnable
    _, accs = vit.train(vit.config("vit_mnist_ref"), epochs=2, device="cpu", n_train=1024, n_test=256,
                        log=lambda *a: None)
    assert accs[-1] > 30.0


def test_reference_named_api(tmp_path):
    """Reference entry-point names (solvingpapers_amd/api.py): pickle-free LLaMA pytree I/O,
    DSV3 get_lr / compute_mtp_loss / topk_sampling / checkpoint, estimate_loss."""
    import torch.nn.functional as F
    from solvingpapers_amd import api
    from solvingpapers_amd.models import deepseekv3 as ds, llama3
    m = llama3.Llama3(llama3.config("llama3_ref", vocab_size=64, dim=32, n_heads=4, n_kv_heads=2, ffn_hidden=64))
    tree = m.to_reference_params()
    p = str(tmp_path / "params.safetensors")
    api.save_params(tree, p)
    back = api.load_params(p)
    m2 = llama3.Llama3(llama3.config("llama3_ref", vocab_size=64, dim=32, n_heads=4, n_kv_heads=2, ffn_hidden=64), seed=3)
    m2.from_reference_params(back)
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    assert abs(api.get_lr(0) - 6e-4 / 401) < 1e-12 and abs(api.get_lr(20000) - 6e-5) < 1e-12
    # compute_mtp_loss vs the notebook's double loop
    B, T, D, C = 2, 5, 2, 7
    lg = torch.randn(B, T, D, C)
    tg = torch.randint(0, C, (B, T))
    idx = [min(i + k + 1, T - 1) for i in range(T) for k in range(D)]
    ref = F.cross_entropy(lg.reshape(-1, C), tg[:, idx].reshape(-1))
    assert torch.allclose(api.compute_mtp_loss(lg, tg), ref)
    dm = ds.DeepSeekV3(ds.config("dsv3_tiny", vocab_size=64, n_layers=1))
    out = api.topk_sampling(dm, torch.zeros(1, 3, dtype=torch.long), max_length=8, top_k=5,
                            generator=torch.Generator().manual_seed(0))
    assert out.shape == (1, 8)
    data = torch.randint(0, 64, (500,))
    est = api.estimate_loss(m, {"train": data, "val": data}, 2, 4, 16)
    assert set(est) == {"train", "val"} and all(v > 0 for v in est.values())
