"""Luong global "dot" attention (attention/luong.ipynb:22-36) as a module over the
fused single-pass HIP kernel (score + softmax + weighted sum per batch row)."""
import torch.nn as tnn

from ..ops.misc import luong_attention


class LuongAttention(tnn.Module):
    def __init__(self, hidden_size):
        super().__init__()
        self.hidden_size = hidden_size

    def forward(self, st, ht):
        """st (B,H) or (B,1,H); ht (B,S,H) -> (context (B,H), weights (B,S,1))."""
        return luong_attention(st, ht)
