"""Autoencoder and VAE on MNIST-shaped inputs.

Reference: autoencoder/autoencoder.ipynb (AE 784-256-32, ReLU on the latent (Q14),
Sigmoid output, MSE, Adam 1e-3, 5 epochs, batch 128) and
autoencoder/variational autoencoder.ipynb (VAE 784-256-128, reparameterise
:94-97, BCE(sum) + KL :117-120, Adam 1e-3, 10 epochs). State-dict keys match
the reference (encoder.{0,2}, decoder.{0,2}; VAE encoder.0, fc_mu, fc_logvar).
Hot ops: Linear (hipBLASLt) + HIP activation / fused MSE / VAE loss / reparam kernels.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as tnn

from .. import nn as snn
from ..ops.misc import mse_loss, reparameterize, vae_loss


class AutoEncoder(tnn.Module):
    def __init__(self, latent_dim=32, hidden_dim=256, input_dim=784):
        super().__init__()
        self.encoder = tnn.Sequential(snn.Linear(input_dim, hidden_dim), snn.ReLU(),
                                      snn.Linear(hidden_dim, latent_dim), snn.ReLU())
        self.decoder = tnn.Sequential(snn.Linear(latent_dim, hidden_dim), snn.ReLU(),
                                      snn.Linear(hidden_dim, input_dim), snn.Sigmoid())

    def forward(self, x):
        return self.decoder(self.encoder(x))


class VAE(tnn.Module):
    def __init__(self, input_dim=784, hidden_dim=256, latent_dim=128):
        super().__init__()
        self.encoder = tnn.Sequential(snn.Linear(input_dim, hidden_dim), snn.ReLU())
        self.fc_mu = snn.Linear(hidden_dim, latent_dim)
        self.fc_logvar = snn.Linear(hidden_dim, latent_dim)
        self.decoder = tnn.Sequential(snn.Linear(latent_dim, hidden_dim), snn.ReLU(),
                                      snn.Linear(hidden_dim, input_dim), snn.Sigmoid())

    def reparameterize(self, mu, logvar):
        return reparameterize(mu, logvar)

    def forward(self, x):
        h = self.encoder(x)
        mu, logvar = self.fc_mu(h), self.fc_logvar(h)
        z = self.reparameterize(mu, logvar)
        return self.decoder(z), mu, logvar


@dataclass
class AEConfig:
    kind: str = "ae"          # "ae" | "vae"
    batch_size: int = 128
    epochs: int = 5           # AE 5, VAE 10 in the reference
    lr: float = 1e-3
    n_train: int = 6000
    n_test: int = 1000
    device: str = "cuda" if torch.cuda.is_available() else "cpu"
    mnist_root: Optional[str] = None
    seed: int = 0


def train(cfg: AEConfig = AEConfig(), log=print):
    """Adam training loop (autoencoder.ipynb:122-139 / variational autoencoder.ipynb:159-176).
    Returns per-epoch average losses (MSE for AE; BCE-sum+KL per 128-image batch for VAE, Q18)."""
    from ..data.images import ImageBatches, mnist_or_synthetic
    from ..train.optim import FlatAdam
    from ..utils.flat import FlatParams
    torch.manual_seed(cfg.seed)
    (xtr, _), _ = mnist_or_synthetic(cfg.mnist_root, cfg.n_train, cfg.n_test, cfg.seed)
    model = (AutoEncoder() if cfg.kind == "ae" else VAE()).to(cfg.device)
    flat = FlatParams(model)
    opt = FlatAdam(flat, lr=cfg.lr)
    loader = ImageBatches(xtr, xtr, cfg.batch_size, True, cfg.device, cfg.seed)
    hist = []
    for ep in range(cfg.epochs):
        tot, nb = 0.0, 0
        for x, _ in loader:
            x = x.view(-1, 784)
            opt.zero_grad()
            if cfg.kind == "ae":
                loss = mse_loss(model(x), x)
            else:
                r, mu, lv = model(x)
                loss = vae_loss(r, x, mu, lv)
            loss.backward()
            opt.step()
            tot += float(loss.item())
            nb += 1
        hist.append(tot / nb)
        log(f"epoch {ep + 1}/{cfg.epochs} loss {hist[-1]:.6f}")
    return model, hist
