"""Autograd wrappers for the training path (config C4, scripts/04_train.py:128-141).

The forward of every op is the same HIP kernel the inference path runs.  Backward:

* Conv1d / Linear input-gradient: HIP -- the conv kernel itself over dY with the weights
  re-packed taps-reversed / channels-swapped (``vo_pack_weight`` mode DGRAD);
* Conv1d / Linear weight and bias gradients: HIP -- ``vo_conv1d_wgrad`` (MFMA, fragments
  read transposed from LDS) and ``vo_colsum``;
* attention, LayerNorm and LengthRegulator backward: PyTorch-ROCm recomputation -- the
  initial fallback SURVEY.md 8(b) sanctions for C4.

All functions take and return channels-last (B, T, C) activations.
"""

import torch
import torch.nn.functional as F

from . import ops


class Conv1dFn(torch.autograd.Function):
    """y = post(conv1d(x, w, b, K, dil, pad)), post in {none, relu}; x (B, T, Ci), w (Co, Ci, K)."""

    @staticmethod
    def forward(ctx, x, w, b, K, dil, pad, relu, compute_dtype, out_dtype):
        Co = w.shape[0]
        wp = ops.pack_conv_weight(w, compute_dtype)
        y = ops.conv1d(x.contiguous(), wp, b.detach().float().contiguous() if b is not None else None, Co=Co,
                       K=K, dil=dil, pad=pad, post_act=ops.ACT_RELU if relu else ops.ACT_NONE,
                       out_dtype=out_dtype, compute_dtype=compute_dtype)
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.cfg = (K, dil, pad, relu, compute_dtype, b is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        K, dil, pad, relu, cdt, has_b = ctx.cfg
        gz = gy.contiguous()
        if relu:
            gz = gz * (y > 0).to(gz.dtype)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            wd = ops.pack_dgrad_weight(w, cdt)
            gx = ops.conv1d(gz.to(cdt) if gz.dtype != cdt else gz, wd, None, Co=w.shape[1], K=K, dil=dil,
                            pad=(K - 1) * dil - pad, T_out=x.shape[1], out_dtype=x.dtype, compute_dtype=cdt)
        if ctx.needs_input_grad[1]:
            if x.dtype in (torch.float32, torch.bfloat16) and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0:
                # MFMA weight gradient over transposed LDS reads (vo_conv1d_wgrad)
                gw = ops.conv1d_wgrad(gz.to(x.dtype).contiguous(), x.contiguous(), K, dil=dil, pad=pad).to(w.dtype)
            else:
                gw = torch.nn.grad.conv1d_weight(x.float().transpose(1, 2), w.shape, gz.float().transpose(1, 2),
                                                 padding=pad, dilation=dil)
        if has_b and ctx.needs_input_grad[2]:
            gb = ops.colsum(gz.contiguous())
        return gx, gw, gb, None, None, None, None, None, None


def conv1d(x, w, b, K=1, dil=1, pad=0, relu=False, compute_dtype=torch.bfloat16, out_dtype=None):
    return Conv1dFn.apply(x, w, b, K, dil, pad, relu, compute_dtype, out_dtype or x.dtype)


def linear(x, weight, bias, relu=False, compute_dtype=torch.bfloat16, out_dtype=None):
    return conv1d(x, weight[:, :, None], bias, 1, 1, 0, relu, compute_dtype, out_dtype)


def _ref_attention(qkv, lens, n_head):
    B, L, D3 = qkv.shape
    D = D3 // 3
    dk = D // n_head
    q, k, v = qkv.float().split(D, dim=-1)
    q = q.view(B, L, n_head, dk).transpose(1, 2)
    k = k.view(B, L, n_head, dk).transpose(1, 2)
    v = v.view(B, L, n_head, dk).transpose(1, 2)
    s = q @ k.transpose(-1, -2) / dk ** 0.5
    mask = torch.arange(L, device=qkv.device)[None, None, None, :] >= lens.long()[:, None, None, None]
    p = torch.softmax(s.masked_fill(mask, float("-inf")), dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    return (p @ v).transpose(1, 2).reshape(B, L, D)


class AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, lens, n_head):
        ctx.save_for_backward(qkv, lens)
        ctx.n_head = n_head
        return ops.attention(qkv.contiguous(), lens, n_head)

    @staticmethod
    def backward(ctx, go):
        qkv, lens = ctx.saved_tensors
        with torch.enable_grad():
            q = qkv.detach().float().requires_grad_(True)
            out = _ref_attention(q, lens, ctx.n_head)
            (g,) = torch.autograd.grad(out, q, go.float())
        return g.to(qkv.dtype), None, None


def attention(qkv, lens, n_head):
    return AttentionFn.apply(qkv, lens, n_head)


class LayerNormFn(torch.autograd.Function):
    """LN(x + res) * g + b with pad rows (t >= lens[b]) zeroed (FFTBlock.masked_fill)."""

    @staticmethod
    def forward(ctx, x, res, g, b, lens):
        ctx.save_for_backward(x, res, g, b, lens)
        return ops.layernorm(x.contiguous(), g.detach().float().contiguous(), b.detach().float().contiguous(),
                             res=res.contiguous() if res is not None else None, lens=lens)

    @staticmethod
    def backward(ctx, gy):
        x, res, g, b, lens = ctx.saved_tensors
        with torch.enable_grad():
            xi = x.detach().float().requires_grad_(True)
            ri = res.detach().float().requires_grad_(True) if res is not None else None
            gi = g.detach().requires_grad_(True)
            bi = b.detach().requires_grad_(True)
            h = xi + ri if ri is not None else xi
            y = F.layer_norm(h, (h.shape[-1],), gi, bi, 1e-5)
            if lens is not None:
                pad = torch.arange(y.shape[1], device=y.device)[None, :] >= lens.long()[:, None]
                y = y.masked_fill(pad[..., None], 0.0)
            ins = [t for t in (xi, ri, gi, bi) if t is not None]
            grads = torch.autograd.grad(y, ins, gy.float())
        gx = grads[0].to(x.dtype)
        gr = grads[1].to(res.dtype) if res is not None else None
        gg, gb = grads[-2], grads[-1]
        return gx, gr, gg, gb, None


def layernorm(x, res, g, b, lens=None):
    return LayerNormFn.apply(x, res, g, b, lens)


class LengthRegulateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dur, max_len, out_dtype):
        out, mel_len, idx = ops.length_regulate(x.contiguous(), dur, int(max_len), out_dtype=out_dtype,
                                                want_index=True)
        ctx.save_for_backward(idx)
        ctx.shape = x.shape
        ctx.xdtype = x.dtype
        ctx.mark_non_differentiable(mel_len)
        return out, mel_len

    @staticmethod
    def backward(ctx, go, _gm):
        (idx,) = ctx.saved_tensors
        B, T, D = ctx.shape
        gx = torch.zeros((B, T + 1, D), dtype=torch.float32, device=go.device)
        src = torch.where(idx >= 0, idx, torch.full_like(idx, T)).long()
        gx.scatter_add_(1, src[..., None].expand(-1, -1, D), go.float())
        return gx[:, :T].to(ctx.xdtype), None, None, None


def batch_norm_train(x, bn, dims):
    """Training-mode BatchNorm (batch statistics over ``dims``; the channel is the one dim left)
    with the running-stat update of ``nn.BatchNorm*`` (momentum, unbiased running variance,
    ``num_batches_tracked``).  Reductions and elementwise ops of PyTorch-ROCm on the tensor as it
    lies -- channels-last PostNet activations need no transpose, and the single-channel VFE
    maps reduce over all blocks (MIOpen's spatial kernels took ~200 us a call on both)."""
    n = 1
    for d in dims:
        n *= x.shape[d]
    mean = x.mean(dims, keepdim=True)
    xc = x - mean
    var = (xc * xc).mean(dims, keepdim=True)
    if bn.track_running_stats and bn.running_mean is not None:
        with torch.no_grad():
            bn.num_batches_tracked.add_(1)
            m = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
            bn.running_mean.mul_(1.0 - m).add_(mean.detach().flatten().to(bn.running_mean.dtype), alpha=m)
            bn.running_var.mul_(1.0 - m).add_(var.detach().flatten().to(bn.running_var.dtype),
                                              alpha=m * n / max(n - 1, 1))
    shape = [1] * x.dim()
    ch = [d for d in range(x.dim()) if d not in dims and d - x.dim() not in dims]
    shape[ch[0]] = x.shape[ch[0]]
    y = xc * torch.rsqrt(var + bn.eps)
    if bn.affine:
        y = y * bn.weight.view(shape) + bn.bias.view(shape)
    return y


def length_regulate(x, dur, max_len, out_dtype=None):
    return LengthRegulateFn.apply(x, dur, max_len, out_dtype or x.dtype)
