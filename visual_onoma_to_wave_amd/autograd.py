"""Autograd wrappers for the training path (config C4, scripts/04_train.py:128-141).

The forward of every op is the same HIP kernel the inference path runs.  Backward:

* Conv1d / Linear input-gradient: HIP -- the conv kernel itself over dY with the weights
  re-packed taps-reversed / channels-swapped (``vo_pack_weight`` mode DGRAD);
* Conv1d / Linear weight and bias gradients: HIP -- ``vo_conv1d_wgrad`` (MFMA, fragments
  read transposed from LDS) and ``vo_colsum``;
* LayerNorm backward: HIP -- ``vo_layernorm_bwd`` (row-wise input gradient, deterministic
  gamma / beta column sums);
* attention backward: HIP -- ``vo_attention_bwd`` (flash-style: the row log-sum-exp is rebuilt
  from q / k, dQ and dK / dV in two MFMA kernels, nothing of size L x L stored);
* LengthRegulator backward: HIP -- ``vo_length_regulate_bwd`` (segmented frame sums per token,
  deterministic);
* training-mode BatchNorm (PostNet, glyph encoder) forward / backward and the glyph encoder's
  3 x 3 conv forward / backward: HIP -- ``vo_bn_*`` and ``vo_vfe_conv_*`` (train_glue.hip).

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
            gz = ops.lrelu_mask(gz, y, 0.0)
        gx = gw = gb = None
        want_b = has_b and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[0]:
            wd = ops.pack_dgrad_weight(w, cdt)
            gx = ops.conv1d(gz.to(cdt) if gz.dtype != cdt else gz, wd, None, Co=w.shape[1], K=K, dil=dil,
                            pad=(K - 1) * dil - pad, T_out=x.shape[1], out_dtype=x.dtype, compute_dtype=cdt)
        if ctx.needs_input_grad[1]:
            if x.dtype in (torch.float32, torch.bfloat16) and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0:
                # MFMA weight gradient over transposed LDS reads (vo_conv1d_wgrad), in the forward's
                # compute dtype (an fp32 activation feeding a bf16 conv -- PostNet after its fp32
                # BatchNorm -- was contracted in bf16 by the forward too)
                fuse_b = want_b and gz.dtype == cdt  # bias = column sums of the same dY (no cast)
                r = ops.conv1d_wgrad(gz.to(cdt).contiguous(), x.to(cdt).contiguous(), K, dil=dil, pad=pad,
                                     with_bias=fuse_b)
                if fuse_b:
                    r, gb = r
                gw = r.to(w.dtype)
            else:
                gw = torch.nn.grad.conv1d_weight(x.float().transpose(1, 2), w.shape, gz.float().transpose(1, 2),
                                                 padding=pad, dilation=dil)
        if want_b and gb is None:
            gb = ops.colsum(gz.contiguous())
        return gx, gw, gb, None, None, None, None, None, None


def conv1d(x, w, b, K=1, dil=1, pad=0, relu=False, compute_dtype=torch.bfloat16, out_dtype=None):
    return Conv1dFn.apply(x, w, b, K, dil, pad, relu, compute_dtype, out_dtype or x.dtype)


def linear(x, weight, bias, relu=False, compute_dtype=torch.bfloat16, out_dtype=None):
    return conv1d(x, weight[:, :, None], bias, 1, 1, 0, relu, compute_dtype, out_dtype)


class AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, lens, n_head):
        # the row log-sum-exp is kept for the backward (B x H x L fp32): it need not rebuild it
        out, lse = ops.attention(qkv.contiguous(), lens, n_head, with_lse=True)
        ctx.save_for_backward(qkv, lens, out, lse)
        ctx.n_head = n_head
        return out

    @staticmethod
    def backward(ctx, go):
        qkv, lens, out, lse = ctx.saved_tensors
        return ops.attention_bwd(qkv.contiguous(), out, go.to(qkv.dtype).contiguous(), lens, ctx.n_head,
                                 lse=lse), None, None


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
        xr = x.contiguous()
        rr = res.contiguous() if res is not None else None
        if rr is not None and rr.dtype != xr.dtype:
            rr = rr.to(xr.dtype)
        gh, gg, gb = ops.layernorm_bwd(xr, gy.contiguous(), g.detach().float().contiguous(), res=rr, lens=lens)
        gr = (gh if res.dtype == gh.dtype else gh.to(res.dtype)) if res is not None else None
        return gh, gr, gg.to(g.dtype), gb.to(b.dtype), None


def layernorm(x, res, g, b, lens=None):
    return LayerNormFn.apply(x, res, g, b, lens)


class LengthRegulateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dur, max_len, out_dtype):
        out, mel_len, _ = ops.length_regulate(x.contiguous(), dur, int(max_len), out_dtype=out_dtype)
        ctx.save_for_backward(dur)
        ctx.shape = x.shape
        ctx.xdtype = x.dtype
        ctx.mark_non_differentiable(mel_len)
        return out, mel_len

    @staticmethod
    def backward(ctx, go, _gm):
        (dur,) = ctx.saved_tensors
        return ops.length_regulate_bwd(go.contiguous(), dur, ctx.shape[1], out_dtype=ctx.xdtype), None, None, None


class BatchNormTrainFn(torch.autograd.Function):
    """nn.BatchNorm* in training mode on HIP (``vo_bn_train_fwd`` / ``vo_bn_bwd``): batch
    statistics per channel, the running-stat update (momentum, unbiased running variance,
    ``num_batches_tracked`` += 1) done by the finalize kernel on the device -- nothing on the
    host, so the step stays graph-capturable."""

    @staticmethod
    def forward(ctx, x, weight, bias, bn):
        xc = x.contiguous()
        track = bn.track_running_stats and bn.running_mean is not None
        y, mr = ops.bn_train_fwd(xc, weight, bias, bn.eps, bn.momentum,
                                 bn.running_mean if track else None, bn.running_var if track else None,
                                 bn.num_batches_tracked if track else None)
        ctx.save_for_backward(xc, weight, mr)
        ctx.has_affine = weight is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, mr = ctx.saved_tensors
        dx, dg, db = ops.bn_bwd(x, gy.contiguous(), w, mr)
        if not ctx.has_affine:
            dg = db = None
        return dx, dg, db, None


def batch_norm_train(x, bn, dims):
    """Training-mode BatchNorm over ``dims`` (batch statistics; the channel is the one dim left):
    channels-last (B, T, C) with dims (0, 1) -- PostNet, no transposes -- or a single-channel
    (N, 1, H, W) map with dims (0, 2, 3) -- the glyph encoder."""
    if bn.momentum is None:
        raise NotImplementedError("batch_norm_train: cumulative-average BatchNorm (momentum=None)")
    if not ((x.dim() == 3 and tuple(dims) == (0, 1)) or (x.dim() == 4 and tuple(dims) == (0, 2, 3) and
                                                           x.shape[1] == 1)):
        raise NotImplementedError(f"batch_norm_train: layout {tuple(x.shape)} over dims {dims}")
    if bn.affine:
        return BatchNormTrainFn.apply(x, bn.weight, bn.bias, bn)
    return BatchNormTrainFn.apply(x, None, None, bn)


class VfeConvFn(torch.autograd.Function):
    """The glyph encoder's Conv2d(1, 1, 3, padding=1) (``vo_vfe_conv_fwd`` / ``vo_vfe_conv_bwd``)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        w10 = torch.cat([weight.detach().reshape(-1).float(), bias.detach().reshape(-1).float()])
        xc = x.contiguous()
        ctx.save_for_backward(xc, w10)
        ctx.wshape = weight.shape
        return ops.vfe_conv_fwd(xc, w10)

    @staticmethod
    def backward(ctx, gy):
        x, w10 = ctx.saved_tensors
        dx, dw = ops.vfe_conv_bwd(x, gy.contiguous(), w10)
        return dx, dw[:9].view(ctx.wshape), dw[9:]


def vfe_conv(x, conv):
    if conv.weight.shape != (1, 1, 3, 3) or conv.bias is None or conv.padding != (1, 1) or conv.stride != (1, 1):
        raise NotImplementedError("vfe_conv: the HIP path covers Conv2d(1, 1, 3, padding=1) with bias")
    return VfeConvFn.apply(x, conv.weight, conv.bias)


def length_regulate(x, dur, max_len, out_dtype=None):
    return LengthRegulateFn.apply(x, dur, max_len, out_dtype or x.dtype)


class BucketEmbedFn(torch.autograd.Function):
    """x + Embedding(table)[bucketize(target, bins)] (scripts/model/modules.py:53-64,101-104, teacher
    forced): forward vo_bucket_embed, backward dx = dy and dtable by vo_embed_bwd (row-ordered sums)."""

    @staticmethod
    def forward(ctx, x, table, target, bins):
        out, idx = ops.bucket_embed(x.contiguous(), target, bins.detach().float().contiguous(),
                                    table.detach().float().contiguous())
        ctx.save_for_backward(idx)
        ctx.n_table = table.shape[0]
        ctx.table_dtype = table.dtype
        ctx.mark_non_differentiable(idx)
        return out, idx

    @staticmethod
    def backward(ctx, go, _gi):
        (idx,) = ctx.saved_tensors
        dt = ops.embed_bwd(go.contiguous(), idx, ctx.n_table) if ctx.needs_input_grad[1] else None
        return go, (dt.to(ctx.table_dtype) if dt is not None else None), None, None


def bucket_embed(x, embedding, target, bins):
    """``x + embedding(torch.bucketize(target, bins))`` on HIP, differentiable in x and the table."""
    return BucketEmbedFn.apply(x, embedding.weight, target, bins)[0]
