"""FFTBlock and PostNet on HIP kernels.

FFTBlock <- scripts/transformer/Layers.py:11-30  (MHA -> mask -> PWFFN -> mask; the two
            masked_fill calls are fused into the LayerNorm kernels)
PostNet  <- scripts/transformer/Layers.py:67-137 (5 x Conv1d k5 + BatchNorm1d(eval), tanh on
            the first four; BatchNorm folded into the packed weights; the caller's
            ``postnet(x) + x`` residual can be fused into the last conv's epilogue)
"""

import torch
import torch.nn as nn

from .. import ops
from .._base import HipModule, fold_bn
from .SubLayers import MultiHeadAttention, PositionwiseFeedForward, lens_from_mask


class FFTBlock(HipModule):
    def __init__(self, d_model, n_head, d_k, d_v, d_inner, kernel_size, dropout=0.1):
        super().__init__()
        self.slf_attn = MultiHeadAttention(n_head, d_model, d_k, d_v, dropout=dropout)
        self.pos_ffn = PositionwiseFeedForward(d_model, d_inner, kernel_size, dropout=dropout)

    def run(self, x, lens):
        y = self.slf_attn.run(x, lens, mask_rows=True)
        return self.pos_ffn.run(y, lens)

    def forward(self, enc_input, mask=None, slf_attn_mask=None):
        self._check_inference()
        x = enc_input.to(self.compute_dtype).contiguous()
        B, L, _ = x.shape
        lens = lens_from_mask(mask) if mask is not None else torch.full(
            (B,), L, dtype=torch.int32, device=x.device)
        return self.run(x, lens), None


class ConvNorm(nn.Module):
    """Parameter holder with the reference key layout ``<i>.0.conv.{weight,bias}``."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=None,
                 dilation=1, bias=True, w_init_gain="linear"):
        super().__init__()
        if padding is None:
            padding = dilation * (kernel_size - 1) // 2
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                              padding=padding, dilation=dilation, bias=bias)


class PostNet(HipModule):
    def __init__(self, n_mel_channels=80, postnet_embedding_dim=512, postnet_kernel_size=5,
                 postnet_n_convolutions=5):
        super().__init__()
        chans = ([n_mel_channels] + [postnet_embedding_dim] * (postnet_n_convolutions - 1) +
                 [n_mel_channels])
        self.kernel_size = postnet_kernel_size
        self.convolutions = nn.ModuleList(
            nn.Sequential(
                ConvNorm(cin, cout, kernel_size=postnet_kernel_size,
                         padding=(postnet_kernel_size - 1) // 2),
                nn.BatchNorm1d(cout))
            for cin, cout in zip(chans[:-1], chans[1:]))

    def _build(self, device, dtype):
        layers = []
        for seq in self.convolutions:
            conv, bn = seq[0].conv, seq[1]
            scale, shift = fold_bn(bn)
            scale, shift = scale.to(device), shift.to(device)
            bias = conv.bias.detach().float().to(device) * scale + shift
            layers.append((ops.pack_conv_weight(conv.weight.to(device), dtype, row_scale=scale),
                           bias.contiguous(), conv.out_channels))
        return layers

    def run(self, x, residual=None, out_dtype=torch.float32):
        """x (B, T, n_mel) -> postnet(x) (+ residual) in out_dtype."""
        layers = self._packed(x.device, self._build)
        k = self.kernel_size
        h = x
        for i, (w, b, co) in enumerate(layers):
            last = i == len(layers) - 1
            h = ops.conv1d(h, w, b, Co=co, K=k, pad=(k - 1) // 2,
                           post_act=ops.ACT_NONE if last else ops.ACT_TANH,
                           res1=residual if last else None,
                           out_dtype=out_dtype if last else self.compute_dtype,
                           compute_dtype=self.compute_dtype)
        return h

    def forward(self, x):
        self._check_inference()
        return self.run(x.contiguous(), out_dtype=torch.float32)
