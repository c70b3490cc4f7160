"""solvingpapers_amd — an MI355X-native (gfx950 / CDNA4) re-implementation of the
prashantpandeygit/solvingpapers model catalogue: GPT, LLaMA3, Gemma, DeepSeek-V3
(MLA + MoE), ViT, AlexNet, AE/VAE, knowledge distillation, Luong attention and
the activation suite — PyTorch-ROCm framework layer, hand-written HIP kernels for
the hot ops, RCCL (torch.distributed "nccl") over xGMI for DP/TP/EP.
"""
__version__ = "0.1.0"

from . import ops  # noqa: F401
