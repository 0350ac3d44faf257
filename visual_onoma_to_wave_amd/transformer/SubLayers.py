"""FFT-block sub-layers on HIP kernels.

MultiHeadAttention   <- scripts/transformer/SubLayers.py:8-57
PositionwiseFeedForward <- scripts/transformer/SubLayers.py:60-93

Parameters keep the reference names (w_qs, w_ks, w_vs, fc, layer_norm; w_1, w_2,
layer_norm) so checkpoints load unchanged.  At pack time q/k/v are fused into one
(3D x D) projection so a block issues one GEMM for all three.
"""

import torch
import torch.nn as nn

from .. import ops
from .._base import HipModule
from .Modules import ScaledDotProductAttention


def lens_from_mask(mask):
    """(B, L) or (B, Lq, Lk) True-is-padding mask -> (B,) int32 valid lengths (prefix masks)."""
    if mask.dim() == 3:
        mask = mask[:, 0, :]
    return (~mask).sum(dim=1, dtype=torch.int32)


class MultiHeadAttention(HipModule):
    def __init__(self, n_head, d_model, d_k, d_v, dropout=0.1):
        super().__init__()
        self.n_head, self.d_k, self.d_v = n_head, d_k, d_v
        self.w_qs = nn.Linear(d_model, n_head * d_k)
        self.w_ks = nn.Linear(d_model, n_head * d_k)
        self.w_vs = nn.Linear(d_model, n_head * d_v)
        self.attention = ScaledDotProductAttention(temperature=float(d_k) ** 0.5)
        self.layer_norm = nn.LayerNorm(d_model)
        self.fc = nn.Linear(n_head * d_v, d_model)
        self.dropout = nn.Dropout(dropout)

    def _build(self, device, dtype):
        w = torch.cat([self.w_qs.weight, self.w_ks.weight, self.w_vs.weight], 0)
        b = torch.cat([self.w_qs.bias, self.w_ks.bias, self.w_vs.bias], 0)
        return dict(
            wqkv=ops.pack_conv_weight(w.to(device)[:, :, None], dtype),
            bqkv=b.detach().float().to(device).contiguous(),
            wfc=ops.pack_conv_weight(self.fc.weight.to(device)[:, :, None], dtype),
            bfc=self.fc.bias.detach().float().to(device).contiguous(),
            g=self.layer_norm.weight.detach().float().to(device).contiguous(),
            beta=self.layer_norm.bias.detach().float().to(device).contiguous(),
        )

    def run(self, x, lens, mask_rows=False, x16=None, want16=False):
        """x (B, L, D) residual stream (the compute dtype, or fp32 under bf16 compute: the
        decoder of the "mixed" precision keeps its residual stream and LayerNorm outputs in fp32,
        as bf16 autocast of the reference does); lens (B,) int32 -> LN(fc(attn) + x) (pad rows
        zeroed when mask_rows, as FFTBlock.masked_fill does), in x's dtype.  x16: x's bf16 copy
        (the q/k/v projection reads it: the same bits as converting x on the fly, half the bytes);
        want16 (fp32 x): returns (y, y16)."""
        p = self._packed(x.device, self._build)
        D = x.shape[-1]
        cd = self.compute_dtype
        qkv = ops.conv1d(x16 if x16 is not None else x, p["wqkv"], p["bqkv"], Co=3 * D, K=1, compute_dtype=cd,
                         out_dtype=cd)
        att, _ = self.attention(qkv, lens, self.n_head)
        y = ops.conv1d(att, p["wfc"], p["bfc"], Co=D, K=1, compute_dtype=cd, out_dtype=x.dtype)
        return ops.layernorm(y, p["g"], p["beta"], res=x, lens=lens if mask_rows else None, with_bf16=want16)

    def forward(self, q, k, v, mask=None):
        """Reference signature (self-attention only, as on the path): returns (out, None)."""
        self._check_inference()
        if not (q is k and k is v):
            raise NotImplementedError("only self-attention (q is k is v) is on the synthesis path")
        x = q.to(self.compute_dtype).contiguous()
        B, L, _ = x.shape
        lens = lens_from_mask(mask) if mask is not None else torch.full(
            (B,), L, dtype=torch.int32, device=x.device)
        return self.run(x, lens), None


class PositionwiseFeedForward(HipModule):
    def __init__(self, d_in, d_hid, kernel_size, dropout=0.1):
        super().__init__()
        self.kernel_size = tuple(kernel_size)
        self.w_1 = nn.Conv1d(d_in, d_hid, kernel_size=kernel_size[0], padding=(kernel_size[0] - 1) // 2)
        self.w_2 = nn.Conv1d(d_hid, d_in, kernel_size=kernel_size[1], padding=(kernel_size[1] - 1) // 2)
        self.layer_norm = nn.LayerNorm(d_in)
        self.dropout = nn.Dropout(dropout)

    def _build(self, device, dtype):
        return dict(
            w1=ops.pack_conv_weight(self.w_1.weight.to(device), dtype),
            b1=self.w_1.bias.detach().float().to(device).contiguous(),
            w2=ops.pack_conv_weight(self.w_2.weight.to(device), dtype),
            b2=self.w_2.bias.detach().float().to(device).contiguous(),
            g=self.layer_norm.weight.detach().float().to(device).contiguous(),
            beta=self.layer_norm.bias.detach().float().to(device).contiguous(),
        )

    def run(self, x, lens=None, x16=None, want16=False):
        """LN(w_2(relu(w_1(x))) + x) in x's dtype (the residual stream, see
        MultiHeadAttention.run), pad rows zeroed when lens is given.  x16 / want16: as
        MultiHeadAttention.run (w_1 reads x16)."""
        p = self._packed(x.device, self._build)
        k1, k2 = self.kernel_size
        d_hid = self.w_1.out_channels
        cd = self.compute_dtype
        h = ops.conv1d(x16 if x16 is not None else x, p["w1"], p["b1"], Co=d_hid, K=k1, pad=(k1 - 1) // 2,
                       post_act=ops.ACT_RELU, compute_dtype=cd, out_dtype=cd,
                       tag=getattr(self, "timer_tag", None))
        y = ops.conv1d(h, p["w2"], p["b2"], Co=x.shape[-1], K=k2, pad=(k2 - 1) // 2,
                       compute_dtype=cd, out_dtype=x.dtype)
        return ops.layernorm(y, p["g"], p["beta"], res=x, lens=lens, with_bf16=want16)

    def forward(self, x):
        self._check_inference()
        return self.run(x.to(self.compute_dtype).contiguous())
