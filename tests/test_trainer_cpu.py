"""Trainer: loss falls, JSONL metrics, checkpoint/resume is bit-exact (params, optimizer,
RNG, routing-bias buffers), NaN guard, reference checkpoint formats."""
import json
import os

import pytest
import torch

from solvingpapers_amd.train.trainer import NonFiniteLoss, TrainConfig, Trainer


def _gpt():
    from solvingpapers_amd.models import gpt
    return gpt.GPT(gpt.config("gpt_tiny_cpu", vocab_size=32, block_size=16, emb_dim=32, num_heads=2,
                              dropout_rate=0.1), seed=0)


def _batches(vocab=32, T=16, B=4):
    def fn(i):
        g = torch.Generator().manual_seed(1000 + i)
        base = torch.randint(0, 8, (B, 1), generator=g)
        x = (base + torch.arange(T + 1)) % vocab          # learnable: arithmetic sequences
        return x[:, :-1], x[:, 1:]
    return fn


def test_trainer_reduces_loss_and_logs(tmp_path):
    log = tmp_path / "m.jsonl"
    cfg = TrainConfig(steps=30, lr=3e-3, min_lr=3e-4, warmup=3, log_path=str(log), eval_every=10, eval_iters=2,
                      weight_decay=0.0)
    tr = Trainer(_gpt(), cfg, _batches(), _batches())
    hist = tr.fit()
    losses = [h["loss"] for h in hist if "loss" in h]
    assert losses[-1] < losses[0] * 0.6
    recs = [json.loads(l) for l in open(log)]
    assert any("val_loss" in r for r in recs) and all("lr" in r for r in recs if "loss" in r)
    steps = [r for r in recs if "loss" in r]
    # cumulative tokens (B 4 x T 16 per step), as the reference logs them
    assert [r["tokens"] for r in steps] == [64 * (r["step"] + 1) for r in steps]


def test_trainer_logs_mfu_from_model_flops(tmp_path):
    """A model with flops_per_token(T) gets an MFU figure per record (per-GPU model FLOP/s over
    TrainConfig.peak_flops); an explicit flops_per_token overrides it."""
    m = _gpt()
    m.flops_per_token = lambda T: 1e6 * T
    tr = Trainer(m, TrainConfig(steps=2, lr=1e-3, peak_flops=1e9), _batches())
    hist = tr.fit()
    for r in hist:
        assert r["mfu"] == pytest.approx(r["tok_per_s"] * 16e6 / 1e9)
    tr2 = Trainer(_gpt(), TrainConfig(steps=1, lr=1e-3, peak_flops=1e9, flops_per_token=5e5), _batches())
    assert tr2.fit()[0]["mfu"] == pytest.approx(tr2.history[0]["tok_per_s"] * 5e5 / 1e9)


def test_resume_is_bit_exact(tmp_path):
    cfg = dict(steps=6, lr=1e-3, weight_decay=0.1, clip=1.0, ckpt_every=3, keep=2, ckpt_dir=str(tmp_path / "a"))
    torch.manual_seed(0)
    straight = Trainer(_gpt(), TrainConfig(**{**cfg, "ckpt_dir": str(tmp_path / "s")}), _batches())
    straight.fit()
    torch.manual_seed(0)
    first = Trainer(_gpt(), TrainConfig(**{**cfg, "steps": 3}), _batches())
    first.fit()
    assert os.path.exists(tmp_path / "a" / "latest")
    torch.manual_seed(123)                                  # RNG must come from the checkpoint
    second = Trainer(_gpt(), TrainConfig(**cfg), _batches())
    second.fit()
    assert second.history[0]["step"] == 3
    assert second.history[-1]["tokens"] == straight.history[-1]["tokens"]    # restored from the checkpoint
    assert torch.equal(second.flat.param, straight.flat.param)
    assert torch.equal(second.opt.m, straight.opt.m)


def test_nan_guard_skips_then_aborts():
    class Bad(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.ones(4))

        def forward(self, x, y):
            return (self.w * float("nan")).sum()

    tr = Trainer(Bad(), TrainConfig(steps=10, max_bad_steps=3), lambda i: (torch.zeros(1, 4), None))
    with pytest.raises(NonFiniteLoss):
        tr.fit()
    assert torch.equal(tr.flat.param[:4], torch.ones(4))     # no update applied


def test_moe_routing_bias_checkpointed(tmp_path):
    from solvingpapers_amd.models import deepseekv3 as ds
    c = ds.config("dsv3_tiny", vocab_size=64, n_layers=2)
    m = ds.DeepSeekV3(c)
    fn = _batches(vocab=64)
    tr = Trainer(m, TrainConfig(steps=2, ckpt_dir=str(tmp_path), ckpt_every=2, lr=1e-3), fn)
    tr.fit()
    b = m.moe_layers()[0].routing_bias.clone()
    assert b.abs().max() > 0
    m2 = ds.DeepSeekV3(c, seed=9)
    tr2 = Trainer(m2, TrainConfig(steps=2, ckpt_dir=str(tmp_path), lr=1e-3), fn)
    assert tr2.maybe_resume()
    assert torch.equal(m2.moe_layers()[0].routing_bias, b)
    assert torch.equal(tr2.flat.param, tr.flat.param)


def test_reference_dsv3_checkpoint_roundtrip(tmp_path):
    from solvingpapers_amd.models import deepseekv3 as ds
    from solvingpapers_amd.train import checkpoint as ck
    c = ds.config("dsv3_ref", vocab_size=97, block_size=16, dim=64, n_layers=1, n_heads=4, latent_dim=16,
                  n_experts=4)
    m = ds.DeepSeekV3(c, seed=1)
    p = str(tmp_path / "checkpoint_latest.pt")
    ck.save_reference_dsv3(p, m, step=41, loss=1.5)
    obj = torch.load(p, weights_only=True)
    assert set(obj) == {"step", "model_state_dict", "optimizer_state_dict", "loss"}
    m2 = ds.DeepSeekV3(c, seed=2)
    assert ck.load_reference_dsv3(p, m2) == 42
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)


def test_cli_entrypoint_trains_and_checkpoints(tmp_path):
    from solvingpapers_amd.train.__main__ import main
    main(["gpt", "--preset", "gpt_tiny_cpu", "--steps", "4", "--set", "num_layers=1", "--device", "cpu",
          "--ckpt-dir", str(tmp_path), "--ckpt-every", "2", "--log", str(tmp_path / "m.jsonl")])
    assert (tmp_path / "latest").exists()
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert len(recs) == 4


def test_metric_hooks_use_reference_wandb_names(tmp_path):
    import json
    import math

    import pytest

    from solvingpapers_amd.train.metrics import JsonlHook, WandbHook, reference_names
    r = reference_names({"step": 3, "loss": 2.0, "lr": 1e-3, "grad_norm": 0.5, "ok": True}, tokens_per_step=4096)
    assert r == {"step": 3, "train_loss": 2.0, "train_perplexity": math.exp(2.0), "lr": 1e-3, "grad_norm": 0.5,
                 "tokens": 4 * 4096}
    v = reference_names({"step": 9, "val_loss": 1.5})
    assert v["val_perplexity"] == pytest.approx(math.exp(1.5))
    p = tmp_path / "m.jsonl"
    h = JsonlHook(str(p), tokens_per_step=10)
    h({"step": 0, "loss": 1.0, "lr": 0.1})
    h.close()
    assert json.loads(p.read_text())["train_loss"] == 1.0
    try:
        import wandb  # noqa: F401
    except ImportError:
        with pytest.raises(RuntimeError, match="wandb"):
            WandbHook("proj")
