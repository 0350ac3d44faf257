"""Scaled dot-product attention (reference: scripts/transformer/Modules.py:6-25).

The reference module materialises softmax(QK^T / T) and returns it; here the HIP flash
kernel (``vo_attention``) computes the output without the probability matrix, which no
caller on the path consumes (scripts/transformer/Models.py:119-124,190-195), so the
second return value is ``None``.
"""

import torch.nn as nn

from .. import ops


class ScaledDotProductAttention(nn.Module):
    def __init__(self, temperature):
        super().__init__()
        self.temperature = temperature

    def forward(self, qkv, lens, n_head):
        """qkv: (B, L, 3*D) fused projections; lens: (B,) int32 key lengths."""
        return ops.attention(qkv, lens, n_head), None
