"""FFTBlock and PostNet on HIP kernels.

FFTBlock <- scripts/transformer/Layers.py:11-30  (MHA -> mask -> PWFFN -> mask; the two
            masked_fill calls are fused into the LayerNorm kernels)
PostNet  <- scripts/transformer/Layers.py:67-137 (5 x Conv1d k5 + BatchNorm1d(eval), tanh on
            the first four; BatchNorm folded into the packed weights; the caller's
            ``postnet(x) + x`` residual can be fused into the last conv's epilogue)
"""

import torch
import torch.nn as nn


from .. import autograd as AG
from .. import ops
from .._base import HipModule, fold_bn
from .SubLayers import MultiHeadAttention, PositionwiseFeedForward, lens_from_mask


class FFTBlock(HipModule):
    def __init__(self, d_model, n_head, d_k, d_v, d_inner, kernel_size, dropout=0.1):
        super().__init__()
        self.slf_attn = MultiHeadAttention(n_head, d_model, d_k, d_v, dropout=dropout)
        self.pos_ffn = PositionwiseFeedForward(d_model, d_inner, kernel_size, dropout=dropout)

    def run(self, x, lens, x16=None, want16=False):
        """x16 / want16: the bf16 copy of the fp32 residual stream handed between the LayerNorms and
        the convs that read them (mixed precision; see MultiHeadAttention.run)."""
        dual = x.dtype == torch.float32 and self.compute_dtype == torch.bfloat16
        if dual:
            y, y16 = self.slf_attn.run(x, lens, mask_rows=True, x16=x16, want16=True)
        else:
            y, y16 = self.slf_attn.run(x, lens, mask_rows=True), None
        return self.pos_ffn.run(y, lens, x16=y16, want16=want16 and dual)

    def train_run(self, x, lens, x16=None):
        """Training forward (autograd; dropout active), scripts/transformer/Layers.py:21-30.  Mixed
        precision (fp32 x, bf16 compute): the residual stream stays fp32 as in inference (a bf16 stream
        raised the decoder's forward drift from fp32 from 3.2e-3 to 6.0e-3 at C4, past the reference's
        own bf16 arithmetic) and the convs read the bf16 copies the LayerNorms write beside it; returns
        (y, y16), y16 None unless mixed.  x16: the bf16 copy of x (None: cast here)."""
        mha, ffn, cd = self.slf_attn, self.pos_ffn, self.compute_dtype
        dual = x.dtype == torch.float32 and cd == torch.bfloat16
        xin = (x16 if x16 is not None else x.to(cd)) if dual else x
        cd = self.contract_dtype  # ops.F32X3 for the mixed mode's fp32 encoder
        qkv = AG.qkv_linear(xin, mha.w_qs.weight, mha.w_ks.weight, mha.w_vs.weight, mha.w_qs.bias, mha.w_ks.bias,
                            mha.w_vs.bias, cd)
        att = AG.attention(qkv, lens, mha.n_head)
        y = AG.linear(att, mha.fc.weight, mha.fc.bias, compute_dtype=cd)
        k1, k2 = ffn.kernel_size
        x1, x1_16 = self._drop_norm(y, x, mha.dropout.p, mha.layer_norm, lens, dual)
        h = AG.conv1d(x1_16, ffn.w_1.weight, ffn.w_1.bias, K=k1, pad=(k1 - 1) // 2, relu=True, compute_dtype=cd)
        y2 = AG.conv1d(h, ffn.w_2.weight, ffn.w_2.bias, K=k2, pad=(k2 - 1) // 2, compute_dtype=cd)
        x2, x2_16 = self._drop_norm(y2, x1, ffn.dropout.p, ffn.layer_norm, lens, dual)
        return x2, (x2_16 if dual else None)

    @staticmethod
    def _drop_norm(y, res, p, ln, lens, dual):
        """LayerNorm(dropout_p(y) + res) (SubLayers.py:51-55,88-91): the dropout in the LayerNorm kernels
        (AG.layernorm_drop) when p > 0; returns (out, the copy the next conv reads)."""
        if p > 0.0:
            if dual:
                return AG.layernorm_drop(y, res, ln.weight, ln.bias, lens, p, True)
            out = AG.layernorm_drop(y, res, ln.weight, ln.bias, lens, p, False)
            return out, out
        if dual:
            return AG.layernorm_dual(y, res, ln.weight, ln.bias, lens)
        out = AG.layernorm(y, res, ln.weight, ln.bias, lens)
        return out, out

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
        self.dropout_p = 0.5  # F.dropout(..., 0.5, training), scripts/transformer/Layers.py:129-131
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

    def train_run(self, x):
        """Training forward: conv (HIP) -> BatchNorm1d with batch statistics -> tanh -> dropout(0.5)."""
        h = x
        k = self.kernel_size
        n = len(self.convolutions)
        for i, seq in enumerate(self.convolutions):
            conv, bn = seq[0].conv, seq[1]
            last = i == n - 1
            # the conv bias feeds a train-mode BatchNorm: its gradient is exactly 0 (bias_before_bn), not the
            # rounding noise of the column sums of a bf16 dY (measured 2x the reference's own bf16 noise)
            h = AG.conv1d(h, conv.weight, conv.bias, K=k, pad=(k - 1) // 2, compute_dtype=self.compute_dtype,
                          out_dtype=torch.float32 if last else self.compute_dtype, bias_before_bn=True)
            hb = AG.batch_norm_train(h, bn, (0, 1))  # channels-last (B, T, C): no transposes
            if not last:
                hb = torch.tanh(hb)
            h = AG.dropout(hb, self.dropout_p)
        return h

    def forward(self, x):
        self._check_inference()
        return self.run(x.contiguous(), out_dtype=torch.float32)
