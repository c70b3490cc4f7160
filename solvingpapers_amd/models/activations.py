"""Activation-function suite (activation functions/GELU.ipynb, ReLU.ipynb).

relu, leaky_relu (0.01), prelu(alpha), elu(alpha), gelu (tanh approximation, as the
notebook's formula :54-55, and exact erf), silu, sigmoid — all on the templated HIP
elementwise kernel for GPU tensors. ``value_table`` reproduces the notebooks'
linspace(-10, 10, 50) printouts (PReLU alpha 0.3, ELU alpha 0.4).
"""
import numpy as np
import torch

from ..ops import act


def relu(x): return act(x, "relu")
def leakyrelu(x, alpha=0.01): return act(x, "leaky_relu", alpha)
def prelu(x, alpha): return act(x, "prelu", alpha)
def elu(x, alpha): return act(x, "elu", alpha)
def gelu(x): return act(x, "gelu_tanh")          # GELU.ipynb:54-55 formula
def gelu_exact(x): return act(x, "gelu")
def silu(x): return act(x, "silu")
def sigmoid(x): return act(x, "sigmoid")


def numpy_reference():
    """The notebooks' NumPy definitions, for parity tests."""
    return {
        "relu": lambda x: np.maximum(0, x),
        "leakyrelu": lambda x: np.where(x > 0, x, 0.01 * x),
        "prelu": lambda x, a: np.where(x > 0, x, a * x),
        "elu": lambda x, a: np.where(x > 0, x, a * (np.exp(x) - 1)),
        "gelu": lambda x: 0.5 * x * (1 + np.tanh(np.sqrt(2 / np.pi) * (x + 0.044715 * np.power(x, 3)))),
    }


def value_table(device="cpu"):
    x = torch.linspace(-10, 10, 50, device=device)
    return {
        "x": x.cpu(),
        "relu": relu(x).cpu(), "leakyrelu": leakyrelu(x).cpu(), "prelu": prelu(x, 0.3).cpu(),
        "elu": elu(x, 0.4).cpu(), "gelu": gelu(x).cpu(),
    }
