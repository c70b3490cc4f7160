"""Image data. MNIST IDX reader (the format torchvision's MNIST files use) and a
deterministic synthetic MNIST-like generator: 10 class templates (strokes) + noise +
random shifts, so classifiers/autoencoders have real structure to learn without
network access. Used by ViT / AE / VAE / KD / AlexNet entry points."""
from __future__ import annotations

import gzip
import os
import struct
from typing import Optional, Tuple

import numpy as np
import torch


def load_mnist_idx(images_path: str, labels_path: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """Read idx3-ubyte images (+ idx1-ubyte labels), optionally .gz. Returns float [N,1,28,28] in [0,1]."""
    op = gzip.open if images_path.endswith(".gz") else open
    with op(images_path, "rb") as f:
        magic, n, r, c = struct.unpack(">IIII", f.read(16))
        assert magic == 2051, "not an idx3 image file"
        imgs = np.frombuffer(f.read(n * r * c), dtype=np.uint8).reshape(n, 1, r, c)
    op = gzip.open if labels_path.endswith(".gz") else open
    with op(labels_path, "rb") as f:
        magic, n2 = struct.unpack(">II", f.read(8))
        assert magic == 2049 and n2 == n, "not an idx1 label file"
        labels = np.frombuffer(f.read(n), dtype=np.uint8)
    return torch.from_numpy(imgs.astype(np.float32) / 255.0), torch.from_numpy(labels.astype(np.int64))


def _templates(C: int, H: int, W: int, classes: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    t = np.zeros((classes, C, H, W), np.float32)
    yy, xx = np.mgrid[0:H, 0:W]
    for k in range(classes):
        for _ in range(3):  # three strokes per class
            x0, y0 = rng.uniform(0.2, 0.8, 2) * (W, H)
            ang = rng.uniform(0, np.pi)
            d = np.abs((xx - x0) * np.sin(ang) - (yy - y0) * np.cos(ang))
            along = np.abs((xx - x0) * np.cos(ang) + (yy - y0) * np.sin(ang))
            stroke = np.exp(-d ** 2 / (2 * (0.06 * H) ** 2)) * (along < 0.35 * H)
            t[k] += stroke[None].astype(np.float32) * rng.uniform(0.5, 1.0, (C, 1, 1))
    return np.clip(t, 0, 1)


def synthetic_images(n: int, C: int = 1, H: int = 28, W: int = 28, classes: int = 10, seed: int = 0,
                     noise: float = 0.15, template_seed: int = 1234) -> Tuple[torch.Tensor, torch.Tensor]:
    """``template_seed`` fixes the class templates (shared by train and test splits);
    ``seed`` draws labels, shifts and noise."""
    rng = np.random.default_rng(seed + 1)
    temp = _templates(C, H, W, classes, template_seed)
    y = rng.integers(0, classes, n)
    x = temp[y].copy()
    sh = rng.integers(-2, 3, (n, 2))
    for i in range(n):
        x[i] = np.roll(x[i], tuple(sh[i]), axis=(1, 2))
    x += rng.normal(0, noise, x.shape).astype(np.float32)
    return torch.from_numpy(np.clip(x, 0, 1)), torch.from_numpy(y.astype(np.int64))


def synthetic_mnist(n_train=6000, n_test=1000, seed=0):
    xtr, ytr = synthetic_images(n_train, seed=seed)
    xte, yte = synthetic_images(n_test, seed=seed + 100)
    return (xtr, ytr), (xte, yte)


def mnist_or_synthetic(root: Optional[str] = None, n_train=6000, n_test=1000, seed=0):
    """Real MNIST from IDX files under ``root`` if present, else synthetic."""
    if root:
        f = lambda s: os.path.join(root, s)
        cands = [("train-images-idx3-ubyte", "train-labels-idx1-ubyte", "t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")]
        for a, b, c, d in cands:
            for ext in ("", ".gz"):
                if os.path.exists(f(a + ext)):
                    return load_mnist_idx(f(a + ext), f(b + ext)), load_mnist_idx(f(c + ext), f(d + ext))
    return synthetic_mnist(n_train, n_test, seed)


class ImageBatches:
    """Minimal DataLoader replacement: shuffled mini-batches moved to ``device``."""

    def __init__(self, x, y, batch_size, shuffle=True, device=None, seed=0, drop_last=False):
        self.x, self.y, self.bs, self.shuffle, self.device, self.seed, self.drop_last = x, y, batch_size, shuffle, device, seed, drop_last
        self.epoch = 0

    def __len__(self):
        n = self.x.shape[0]
        return n // self.bs if self.drop_last else (n + self.bs - 1) // self.bs

    def __iter__(self):
        n = self.x.shape[0]
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        self.epoch += 1
        order = torch.randperm(n, generator=g) if self.shuffle else torch.arange(n)
        for k in range(len(self)):
            idx = order[k * self.bs:(k + 1) * self.bs]
            yield self.x[idx].to(self.device), self.y[idx].to(self.device)
