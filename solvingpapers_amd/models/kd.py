"""Knowledge distillation (Hinton et al.) — teacher/student MLPs on MNIST-shaped data.

Reference: knowledge distillation/kd.py (Teacher 784-1024-1024-10 :17-30, Student
784-256-10 :33-45, distillation_loss :48-68 with T=7, alpha=0.3, teacher pre-train 3
epochs then frozen, student 10 epochs :85-142, evaluate :145-156). The KD loss is the
fused HIP kd_loss kernel (soft + hard terms and d(student) in one pass per row).
State-dict keys match (net.{1,3,5} / net.{1,3}).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as tnn

from .. import nn as snn
from ..ops import cross_entropy
from ..ops.misc import distillation_loss  # noqa: F401  (re-exported: reference entry point)


class Teacher(tnn.Module):
    def __init__(self):
        super().__init__()
        self.net = tnn.Sequential(snn.Flatten(), snn.Linear(784, 1024), snn.ReLU(), snn.Linear(1024, 1024),
                                  snn.ReLU(), snn.Linear(1024, 10))

    def forward(self, x):
        return self.net(x)


class Student(tnn.Module):
    def __init__(self):
        super().__init__()
        self.net = tnn.Sequential(snn.Flatten(), snn.Linear(784, 256), snn.ReLU(), snn.Linear(256, 10))

    def forward(self, x):
        return self.net(x)


@dataclass
class KDConfig:
    batch_size: int = 128
    epochs: int = 10
    teacher_epochs: int = 3
    lr: float = 1e-3
    temperature: float = 7.0
    alpha: float = 0.3
    n_train: int = 6000
    n_test: int = 1000
    device: str = "cuda" if torch.cuda.is_available() else "cpu"
    mnist_root: Optional[str] = None
    seed: int = 0


@torch.inference_mode()
def evaluate(model, loader):
    """Top-1 accuracy (%) over the loader (kd.py:145-156; inference_mode per Q16)."""
    model.eval()
    correct = total = 0
    for x, y in loader:
        correct += int((model(x).argmax(1) == y).sum())
        total += y.numel()
    model.train()
    return 100.0 * correct / max(total, 1)


def train(cfg: KDConfig = KDConfig(), log=print):
    from ..data.images import ImageBatches, mnist_or_synthetic
    from ..train.optim import FlatAdam
    from ..utils.flat import FlatParams
    torch.manual_seed(cfg.seed)
    (xtr, ytr), (xte, yte) = mnist_or_synthetic(cfg.mnist_root, cfg.n_train, cfg.n_test, cfg.seed)
    train_loader = ImageBatches(xtr, ytr, cfg.batch_size, True, cfg.device, cfg.seed)
    test_loader = ImageBatches(xte, yte, cfg.batch_size, False, cfg.device)
    teacher, student = Teacher().to(cfg.device), Student().to(cfg.device)
    tflat = FlatParams(teacher)
    topt = FlatAdam(tflat, lr=cfg.lr)
    for ep in range(cfg.teacher_epochs):
        for x, y in train_loader:
            topt.zero_grad()
            cross_entropy(teacher(x), y).backward()
            topt.step()
        log(f"teacher epoch {ep + 1}: acc {evaluate(teacher, test_loader):.2f}%")
    teacher.eval()
    for p in teacher.parameters():
        p.requires_grad_(False)
    sflat = FlatParams(student)
    sopt = FlatAdam(sflat, lr=cfg.lr)
    hist = []
    for ep in range(cfg.epochs):
        tot = n = 0
        for x, y in train_loader:
            with torch.no_grad():
                tl = teacher(x)
            sopt.zero_grad()
            loss, hard, soft = distillation_loss(student(x), tl, y, cfg.temperature, cfg.alpha)
            loss.backward()
            sopt.step()
            tot += float(loss.item())
            n += 1
        acc = evaluate(student, test_loader)
        hist.append((tot / n, acc))
        log(f"epoch {ep + 1}/{cfg.epochs} loss {tot / n:.4f} student acc {acc:.2f}%")
    return teacher, student, hist
