"""Hot-path ops: each is a hand-written gfx950 HIP kernel (csrc/kernels/*.hip)
registered as ``torch.ops.spa.*``, with a pure-PyTorch oracle for CPU tensors."""
from . import _ext, reference
from .activation import act, elu, geglu, gelu, glu, leaky_relu, prelu, relu, sigmoid, silu, swiglu
from .attention import attention_packed, decode_attention, flash_attention
from .embedding import embedding
from .linear import Linear, linear
from .moe import MoEPlan, combine, gather, grouped_gemm, grouped_linear, moe_ffn, permute, route
from .norm import layer_norm, rms_norm
from .rope import apply_rope, rope_packed_
from .xent import cross_entropy, linear_cross_entropy, per_row_loss

__all__ = [
    "act", "elu", "geglu", "gelu", "glu", "leaky_relu", "prelu", "relu", "sigmoid", "silu", "swiglu",
    "attention_packed", "decode_attention", "flash_attention", "embedding", "Linear", "linear", "layer_norm", "rms_norm",
    "apply_rope", "rope_packed_", "MoEPlan", "combine", "gather", "grouped_gemm", "grouped_linear", "moe_ffn",
    "permute", "route", "cross_entropy", "linear_cross_entropy", "per_row_loss", "reference",
]
