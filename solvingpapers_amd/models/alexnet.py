"""AlexNet (Krizhevsky et al. 2012).

Reference: alexnet/alexnet.py:5-44 (model class only). bf16 convs run on the
implicit-GEMM MFMA kernels (csrc/kernels/conv.hip: fwd / data grad / weight grad, no
column buffer) and the feature stack stays channels-last end to end: LRN, MaxPool,
ReLU and dropout have NHWC-native HIP kernels. fp32 (parity) convs use HIP im2col +
fp32 GEMM. Input must be 193-224 px (Q15: Linear(256*5*5)).
State-dict keys match: features.{0,4,8,10,12}.*, classifier.{1,4,6}.*.
"""
from __future__ import annotations

import torch
import torch.nn as tnn

from .. import nn as snn


class AlexNet(tnn.Module):
    def __init__(self, classes: int, in_channels: int = 3):
        super().__init__()
        self.features = tnn.Sequential(
            snn.Conv2d(in_channels, 96, 11, stride=4, padding=1), snn.ReLU(), snn.LocalResponseNorm(5),
            snn.MaxPool2d(3, 2),
            snn.Conv2d(96, 256, 5, padding=2), snn.ReLU(), snn.LocalResponseNorm(5), snn.MaxPool2d(3, 2),
            snn.Conv2d(256, 384, 3, padding=1), snn.ReLU(),
            snn.Conv2d(384, 384, 3, padding=1), snn.ReLU(),
            snn.Conv2d(384, 256, 3, padding=1), snn.ReLU(),
            snn.MaxPool2d(3, 2),
        )
        self.classifier = tnn.Sequential(
            snn.Dropout(0.5), snn.Linear(256 * 5 * 5, 4096), snn.ReLU(),
            snn.Dropout(0.5), snn.Linear(4096, 4096), snn.ReLU(),
            snn.Linear(4096, classes),
        )

    def forward(self, x):
        x = self.features(x)
        return self.classifier(torch.flatten(x, 1))
