"""Torch-tensor front end of the C ABI: shape checks, output allocation, stream plumbing.

Every function here launches a hand-written HIP kernel from ``lib/libvonoma.so`` on
the current torch stream of the tensors' device.  Tensors must be CUDA (ROCm)
tensors; there is no CPU path -- a CPU tensor raises.
"""

import ctypes

import numpy as np

import torch

from . import _lib, profiling
from ._lib import (ACT_LRELU, ACT_NONE, ACT_RELU, ACT_TANH, HEAD_DURATION, HEAD_ENERGY,  # noqa: F401
                   PACK_CONV, PACK_CONVT, VO_BF16, VO_F32, VO_F32X3)

_DT = {torch.float32: VO_F32, torch.bfloat16: VO_BF16}


class _F32X3:
    """``compute_dtype`` of a contraction over fp32 tensors computed as split-bf16 (VO_F32X3 in
    include/vonoma.h): each fp32 operand as hi + lo bf16, three bf16 MFMAs per product, <= 3 * 2^-18
    relative error per product.  Tensors, packed weights and results stay fp32 (storage_dtype)."""

    def __repr__(self):
        return "ops.F32X3"


F32X3 = _F32X3()


def storage_dtype(cdt):
    """The torch dtype of the tensors and packed weights of compute dtype ``cdt``."""
    return torch.float32 if cdt is F32X3 else cdt


def vo_dtype(t):
    try:
        return _DT[t if isinstance(t, torch.dtype) else t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t}") from None


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(t):
    if not t.is_cuda:
        raise RuntimeError("visual_onoma_to_wave_amd ops run on the GPU only (got a CPU tensor); "
                           "there is no CPU fallback")
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _contig(t, name):
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


# ----------------------------------------------------------------------------- conv1d

def conv1d(x, w_packed, bias, *, Co, K, dil=1, pad=0, T_out=None, out=None, out_dtype=None,
           pre_act=ACT_NONE, pre_slope=0.0, post_act=ACT_NONE, post_slope=0.0, res1=None,
           res2=None, out_scale=1.0, compute_dtype=torch.bfloat16, transposed=None, variant=0,
           tag=None, stride=1, groups=1, ymask=None, ymask_slope=0.0):
    """Channels-last conv: x (B, T_in, Ci) -> y (B, T_out, Co).

    ``w_packed``: [K][Co][Ci] in ``compute_dtype`` (see pack_conv_weight).
    ``transposed``: None or dict(stride=s, pad=p, cout=C_out) for the polyphase
    ConvTranspose1d; then Co = s*C_out, K = 2, pad = 1 and y is (B, s*T_in, C_out).
    ``stride`` / ``groups``: strided and grouped convs (HiFi-GAN discriminators); grouped
    weights are packed dense with zeros outside the diagonal blocks (pack_conv_weight groups=).
    ``ymask`` (the output's shape and strides, bf16): each output stored as
    round(round(v) * (ymask > 0 ? 1 : ymask_slope)) -- an input gradient put through the leaky-ReLU
    backward of the layer whose output ymask is (bit for bit vo_lrelu_mask on the stored output).
    """
    if x.dim() == 2:
        x = x.unsqueeze(0)
    B, T_in, ldx = x.shape
    if x.stride(2) != 1 or x.stride(1) != ldx:
        raise ValueError("conv1d: x must be row-contiguous (B, T, C)")
    Ci = w_packed.shape[2]
    if w_packed.shape[0] != K or w_packed.shape[1] != Co:
        raise ValueError(f"conv1d: packed weight {tuple(w_packed.shape)} != [{K}][{Co}][Ci]")
    if w_packed.dtype != storage_dtype(compute_dtype):
        raise ValueError("conv1d: packed weight dtype must equal the compute dtype")
    if compute_dtype is F32X3 and (x.dtype != torch.float32 or stride > 1 or groups > 1):
        raise ValueError("conv1d: F32X3 compute needs fp32 input, stride 1, no groups")
    out_dtype = out_dtype or x.dtype
    if transposed is not None:
        s, p, cout = transposed["stride"], transposed["pad"], transposed["cout"]
        T_rows = T_in + 1
        up_tout = transposed.get("tout", T_in * s + s - 2 * p)
        shape = (B, up_tout, cout)
        ldy = cout
    else:
        T_rows = T_out if T_out is not None else (T_in + 2 * pad - dil * (K - 1) - 1) // stride + 1
        shape = (B, T_rows, Co)
        ldy = Co
    if out is None:
        out = torch.empty(shape, dtype=out_dtype, device=x.device)
    if out.dim() == 2:
        out = out.unsqueeze(0)
    if transposed is None and not out.is_contiguous():
        # row-strided output view (phase-interleaved rows of a strided conv's input gradient):
        # rows ldy elements apart, channels contiguous; no residuals on such views
        if out.stride(2) != 1 or out.shape[2] != Co or res1 is not None or res2 is not None:
            raise ValueError("conv1d: a non-contiguous out must be a row-strided (B, T, Co) view")
        ldy = out.stride(1)
    else:
        _contig(out, "out")
    if res1 is not None and (res1.shape != out.shape or res1.dtype != out.dtype):
        raise ValueError("conv1d: res1 must match the output")
    if res2 is not None and (res2.shape != out.shape or res2.dtype != out.dtype):
        raise ValueError("conv1d: res2 must match the output")
    d = _lib.Conv1dDesc()
    d.x = x.data_ptr(); d.x_dtype = vo_dtype(x); d.x_bstride = x.stride(0); d.ldx = ldx
    d.w = w_packed.data_ptr(); d.bias = bias.data_ptr() if bias is not None else None
    d.y = out.data_ptr(); d.y_dtype = vo_dtype(out); d.y_bstride = out.stride(0); d.ldy = ldy
    d.res1 = res1.data_ptr() if res1 is not None else None
    d.res2 = res2.data_ptr() if res2 is not None else None
    d.B, d.T_in, d.T_out, d.Ci, d.Co = B, T_in, T_rows, Ci, Co
    d.K, d.dil, d.pad = K, dil, pad
    d.pre_act, d.pre_slope, d.post_act, d.post_slope = pre_act, pre_slope, post_act, post_slope
    d.out_scale = out_scale
    d.compute_dtype = VO_F32X3 if compute_dtype is F32X3 else vo_dtype(compute_dtype)
    if transposed is not None:
        d.transposed, d.up_stride, d.up_pad, d.up_cout, d.up_tout = 1, s, p, cout, up_tout
    d.variant = variant if (x.dtype == out.dtype == compute_dtype == torch.bfloat16) else 0
    d.stride, d.groups = stride, groups
    if ymask is not None:
        if ymask.dim() == 2:
            ymask = ymask.unsqueeze(0)
        if ymask.shape != out.shape or ymask.stride() != out.stride() or ymask.dtype != out.dtype:
            raise ValueError("conv1d: ymask must match the output (shape, strides, dtype)")
        d.ymask, d.ymask_slope = ymask.data_ptr(), float(ymask_slope)
    ws = None
    plain = (transposed is None and stride <= 1 and groups <= 1)
    deep_bf16 = (compute_dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and bias is None and res1 is None and
                 res2 is None and ymask is None and pre_act == ACT_NONE and post_act == ACT_NONE and out_scale == 1.0 and
                 Co <= 256 and Ci * K >= 2048 and B * T_rows >= 8192)
    if plain and ((storage_dtype(compute_dtype) == torch.float32 and T_rows <= 16) or deep_bf16):
        # split-reduction scratch: the short fp32 convs, the deep bf16 convs into <= 256 channels
        # (stream-ordered: freed after enqueue)
        nb = _lib.lib().vo_conv1d_workspace_size(ctypes.byref(d))
        if nb > 0:
            ws = torch.empty(nb // 4, dtype=torch.float32, device=x.device)
            d.workspace, d.workspace_bytes = ws.data_ptr(), nb
    timer = profiling.active()
    ev = timer.start() if (tag is not None and timer is not None and timer.watching(tag)) else None
    _lib.check(_lib.lib().vo_conv1d(ctypes.byref(d), _stream(x)), "vo_conv1d")
    if ev is not None:
        esz = x.element_size()
        flops = 2.0 * B * T_rows * Co * Ci * K / groups
        nbytes = (B * T_in * Ci * esz + out.numel() * out.element_size() +
                  (res1.numel() * res1.element_size() if res1 is not None else 0) +
                  (res2.numel() * res2.element_size() if res2 is not None else 0) +
                  w_packed.numel() * w_packed.element_size())
        timer.stop(tag, ev, flops, nbytes, kernel=f"conv1d_kernel<..., ROLE={d.variant}>")
    return out


def pack_dgrad_weight(w, dtype):
    """(Co, Ci, K) -> [K][Ci][Co] taps reversed: dX = conv1d(dY, this, Co=Ci, pad=(K-1)*dil - pad)."""
    w = w.detach().float().contiguous()
    Co, Ci, K = w.shape
    out = torch.empty((K, Ci, Co), dtype=dtype, device=w.device)
    _lib.check(_lib.lib().vo_pack_weight(_ptr(w), None, None, 2, Co, Ci, K, 1, _ptr(out), vo_dtype(dtype),
                                         _stream(w)), "vo_pack_weight")
    return out


def pack_conv_weight(w, dtype, g=None, row_scale=None, transposed_stride=None):
    """(Co, Ci, K) Conv1d weight (or (Ci, Co, 2s) ConvTranspose1d weight) -> packed.

    g: weight-norm gains (one per dim-0 slice), row_scale: per-output-channel multiplier.
    Returns [K][Co][Ci] (conv) or [2][s*Co][Ci] (transposed) in ``dtype``.
    """
    w = w.detach().float().contiguous()
    if transposed_stride is None:
        Co, Ci, K = w.shape
        out = torch.empty((K, Co, Ci), dtype=dtype, device=w.device)
        mode, stride = PACK_CONV, 1
    else:
        Ci, Co, K = w.shape
        s = transposed_stride
        out = torch.empty((2, s * Co, Ci), dtype=dtype, device=w.device)
        mode, stride = PACK_CONVT, s
    g = None if g is None else g.detach().float().reshape(-1).contiguous()
    rs = None if row_scale is None else row_scale.detach().float().reshape(-1).contiguous()
    _lib.check(_lib.lib().vo_pack_weight(_ptr(w), _ptr(g), _ptr(rs), mode, Co, Ci, K, stride,
                                         _ptr(out), vo_dtype(dtype), _stream(w)), "vo_pack_weight")
    return out


# ----------------------------------------------------------------------------- layer norm

def layernorm(x, gamma, beta, res=None, lens=None, out=None, out_dtype=None, eps=1e-5, with_bf16=False):
    """y = LN(x + res) * gamma + beta, rows t >= lens[b] zeroed.  x: (B, T, D).  ``with_bf16``
    (fp32 y only): returns (y, y16), y16 the bf16 copy of y written in the same pass
    (vo_layernorm_dual) for the next conv to read."""
    if x.dim() == 2:
        x = x.unsqueeze(0)
    B, T, D = x.shape
    _contig(x, "x")
    if res is not None:
        _contig(res, "res")
        if res.shape != x.shape:
            raise ValueError("layernorm: res shape mismatch")
    out = out if out is not None else torch.empty(x.shape, dtype=out_dtype or x.dtype, device=x.device)
    if with_bf16:
        if out.dtype != torch.float32:
            raise ValueError("layernorm: with_bf16 needs an fp32 output")
        out16 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        _lib.check(_lib.lib().vo_layernorm_dual(
            _ptr(x), vo_dtype(x), _ptr(res), vo_dtype(res) if res is not None else vo_dtype(x),
            _ptr(gamma), _ptr(beta), _ptr(lens), B, T, D, eps, _ptr(out), _ptr(out16), _stream(x)),
            "vo_layernorm_dual")
        return out, out16
    _lib.check(_lib.lib().vo_layernorm(
        _ptr(x), vo_dtype(x), _ptr(res), vo_dtype(res) if res is not None else vo_dtype(x),
        _ptr(gamma), _ptr(beta), _ptr(lens), B, T, D, eps, _ptr(out), vo_dtype(out), _stream(x)),
        "vo_layernorm")
    return out


def layernorm_bwd(x, gy, gamma, res=None, lens=None, eps=1e-5):
    """Backward of ``layernorm``: (gh, dgamma, dbeta); gh = dL/d(x + res) in x's dtype."""
    B, T, D = x.shape
    _contig(x, "x")
    _contig(gy, "gy")
    if res is not None:
        _contig(res, "res")
        if res.shape != x.shape or res.dtype != x.dtype:
            raise ValueError("layernorm_bwd: res must match x in shape and dtype")
    if gy.shape != x.shape:
        raise ValueError("layernorm_bwd: gy shape mismatch")
    L = _lib.lib()
    gh = torch.empty_like(x)
    dg = torch.empty(D, dtype=torch.float32, device=x.device)
    db = torch.empty(D, dtype=torch.float32, device=x.device)
    ws = torch.empty(int(L.vo_layernorm_bwd_workspace_size(B, T, D)) // 4, dtype=torch.float32, device=x.device)
    _lib.check(L.vo_layernorm_bwd(_ptr(x), _ptr(res), vo_dtype(x), _ptr(gy), vo_dtype(gy), _ptr(gamma), _ptr(lens),
                                  B, T, D, eps, _ptr(gh), _ptr(dg), _ptr(db), _ptr(ws), _stream(x)),
               "vo_layernorm_bwd")
    return gh, dg, db


def layernorm_bwd_ex(x, gy, gamma, res, lens=None, gy2=None, eps=1e-5):
    """Backward of ``layernorm(x, ..., res=res, out_dtype=float32, with_bf16=True)`` with a bf16 x and an
    fp32 res (the training decoder's fp32 residual stream): gy (fp32 or bf16) the gradient of y, gy2
    (bf16, optional) that of the y16 copy -- added in the kernel.  Returns (gh in x's dtype, gh32 =
    the same gradient in fp32 for res, dgamma, dbeta) (vo_layernorm_bwd_ex)."""
    B, T, D = x.shape
    for t, n in ((x, "x"), (gy, "gy"), (res, "res")):
        _contig(t, n)
    if x.dtype != torch.bfloat16 or res.dtype != torch.float32 or res.shape != x.shape or gy.shape != x.shape:
        raise ValueError("layernorm_bwd_ex: bf16 x, fp32 res, gy of x's shape")
    if gy2 is not None:
        _contig(gy2, "gy2")
        if gy2.dtype != torch.bfloat16 or gy2.shape != x.shape:
            raise ValueError("layernorm_bwd_ex: gy2 must be bf16 of x's shape")
    L = _lib.lib()
    gh = torch.empty_like(x)
    gh32 = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    dg = torch.empty(D, dtype=torch.float32, device=x.device)
    db = torch.empty(D, dtype=torch.float32, device=x.device)
    ws = torch.empty(int(L.vo_layernorm_bwd_workspace_size(B, T, D)) // 4, dtype=torch.float32, device=x.device)
    _lib.check(L.vo_layernorm_bwd_ex(_ptr(x), vo_dtype(x), _ptr(res), vo_dtype(res), _ptr(gy), vo_dtype(gy),
                                     _ptr(gy2), _ptr(gamma), _ptr(lens), B, T, D, eps, _ptr(gh), _ptr(gh32), _ptr(dg),
                                     _ptr(db), _ptr(ws), _stream(x)), "vo_layernorm_bwd_ex")
    return gh, gh32, dg, db


def layernorm_drop(x, gamma, beta, res, p, seed, salt, lens=None, with_bf16=False, eps=1e-5):
    """y = LN(dropout_p(x) + res) * gamma + beta, pad rows zeroed (vo_layernorm_drop): the dropout mask is
    vo_dropout's for the same (seed, salt) on x.  y in res's dtype; with_bf16 (fp32 y): returns (y, y16)."""
    B, T, D = x.shape
    for t, n in ((x, "x"), (res, "res")):
        _contig(t, n)
    if res.shape != x.shape:
        raise ValueError("layernorm_drop: res shape mismatch")
    y = torch.empty(x.shape, dtype=res.dtype, device=x.device)
    y16 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if with_bf16 else None
    _lib.check(_lib.lib().vo_layernorm_drop(
        _ptr(x), vo_dtype(x), _ptr(res), vo_dtype(res), _ptr(gamma), _ptr(beta), _ptr(lens), B, T, D, eps, _ptr(y),
        vo_dtype(y), _ptr(y16), float(p), _ptr(seed), int(salt), _stream(x)), "vo_layernorm_drop")
    return (y, y16) if with_bf16 else y


def layernorm_bwd_drop(x, gy, gamma, res, p, seed, salt, lens=None, gy2=None, eps=1e-5):
    """Backward of ``layernorm_drop``: (gh = dL/dx through the mask in x's dtype, gres = dL/dres in res's dtype,
    dgamma, dbeta); gy2 (bf16, optional): the gradient of the y16 copy, added in the kernel."""
    B, T, D = x.shape
    for t, n in ((x, "x"), (gy, "gy"), (res, "res")):
        _contig(t, n)
    if gy2 is not None:
        _contig(gy2, "gy2")
    L = _lib.lib()
    gh = torch.empty_like(x)
    gres = torch.empty_like(res)
    dg = torch.empty(D, dtype=torch.float32, device=x.device)
    db = torch.empty(D, dtype=torch.float32, device=x.device)
    ws = torch.empty(int(L.vo_layernorm_bwd_workspace_size(B, T, D)) // 4, dtype=torch.float32, device=x.device)
    _lib.check(L.vo_layernorm_bwd_drop(_ptr(x), vo_dtype(x), _ptr(res), vo_dtype(res), _ptr(gy), vo_dtype(gy),
                                       _ptr(gy2), _ptr(gamma), _ptr(lens), B, T, D, eps, float(p), _ptr(seed), int(salt),
                                       _ptr(gh), _ptr(gres), _ptr(dg), _ptr(db), _ptr(ws), _stream(x)),
               "vo_layernorm_bwd_drop")
    return gh, gres, dg, db


# ----------------------------------------------------------------------------- attention

def attention(qkv, lens, n_head, out=None, with_lse=False):
    """qkv (B, L, 3D) -> (B, L, D); keys t >= lens[b] masked.  with_lse: also the row log-sum-exp
    (B, H, L) fp32 that attention_bwd(..., lse=) consumes (vo_attention_lse)."""
    _contig(qkv, "qkv")
    B, L, D3 = qkv.shape
    D = D3 // 3
    dk = D // n_head
    out = out if out is not None else torch.empty((B, L, D), dtype=qkv.dtype, device=qkv.device)
    scale = 1.0 / float(dk) ** 0.5
    if with_lse:
        lse = torch.empty((B, n_head, L), dtype=torch.float32, device=qkv.device)
        _lib.check(_lib.lib().vo_attention_lse(_ptr(qkv), vo_dtype(qkv), _ptr(lens), B, L, n_head, dk,
                                               scale, _ptr(out), _ptr(lse), _stream(qkv)), "vo_attention_lse")
        return out, lse
    _lib.check(_lib.lib().vo_attention(_ptr(qkv), vo_dtype(qkv), _ptr(lens), B, L, n_head, dk,
                                       scale, _ptr(out), _stream(qkv)), "vo_attention")
    return out


def attention_bwd(qkv, out, dout, lens, n_head, lse=None):
    """Backward of ``attention``: dqkv (B, L, 3D) in qkv's dtype from the forward output and its
    gradient (flash-style recomputation, vo_attention_bwd); with the forward's row log-sum-exp (lse,
    attention(..., with_lse=True)) the bf16 path skips rebuilding it (vo_attention_bwd_lse)."""
    for t, n in ((qkv, "qkv"), (out, "out"), (dout, "dout")):
        _contig(t, n)
    B, L, D3 = qkv.shape
    D = D3 // 3
    if out.shape != (B, L, D) or dout.shape != (B, L, D):
        raise ValueError("attention_bwd: out / dout must be (B, L, D)")
    if out.dtype != qkv.dtype or dout.dtype != qkv.dtype:
        raise ValueError("attention_bwd: qkv, out and dout must share a dtype")
    dk = D // n_head
    L_ = _lib.lib()
    dqkv = torch.empty_like(qkv)
    ws = torch.empty(int(L_.vo_attention_bwd_workspace_size(B, L, n_head)) // 4, dtype=torch.float32,
                     device=qkv.device)
    if lse is not None:
        if lse.shape != (B, n_head, L) or lse.dtype != torch.float32 or not lse.is_contiguous():
            raise ValueError("attention_bwd: lse must be the forward's (B, H, L) fp32 row log-sum-exp")
        _lib.check(L_.vo_attention_bwd_lse(_ptr(qkv), _ptr(out), _ptr(dout), vo_dtype(qkv), _ptr(lens), B, L, n_head,
                                           dk, 1.0 / float(dk) ** 0.5, _ptr(lse), _ptr(dqkv), _ptr(ws),
                                           _stream(qkv)), "vo_attention_bwd_lse")
        return dqkv
    _lib.check(L_.vo_attention_bwd(_ptr(qkv), _ptr(out), _ptr(dout), vo_dtype(qkv), _ptr(lens), B, L, n_head, dk,
                                   1.0 / float(dk) ** 0.5, _ptr(dqkv), _ptr(ws), _stream(qkv)),
               "vo_attention_bwd")
    return dqkv


# ----------------------------------------------------------------------------- length regulator

def lr_lengths(dur):
    """(B, T) float durations -> (mel_len int64 (B,), mel_len int32 (B,))."""
    dur = _contig(dur.float(), "dur")
    B, T = dur.shape
    m64 = torch.empty(B, dtype=torch.int64, device=dur.device)
    m32 = torch.empty(B, dtype=torch.int32, device=dur.device)
    _lib.check(_lib.lib().vo_lr_lengths(_ptr(dur), B, T, _ptr(m64), _ptr(m32), _stream(dur)),
               "vo_lr_lengths")
    return m64, m32


def length_regulate(x, dur, max_len, out_dtype=None, want_index=False):
    """x (B, T_src, D), dur (B, T_src) float -> (out (B, max_len, D), mel_len int64, index)."""
    _contig(x, "x")
    dur = _contig(dur.float(), "dur")
    B, T, D = x.shape
    out = torch.empty((B, max_len, D), dtype=out_dtype or x.dtype, device=x.device)
    mel_len = torch.empty(B, dtype=torch.int64, device=x.device)
    index = torch.empty((B, max_len), dtype=torch.int32, device=x.device) if want_index else None
    _lib.check(_lib.lib().vo_length_regulate(_ptr(x), vo_dtype(x), _ptr(dur), B, T, D, max_len,
                                             _ptr(out), vo_dtype(out), _ptr(mel_len), _ptr(index),
                                             _stream(x)), "vo_length_regulate")
    return out, mel_len, index


def length_regulate_bwd(go, dur, T_src, out_dtype=torch.float32):
    """Backward of ``length_regulate``: go (B, max_len, D) -> gx (B, T_src, D)."""
    _contig(go, "go")
    dur = _contig(dur.float(), "dur")
    B, max_len, D = go.shape
    gx = torch.empty((B, T_src, D), dtype=out_dtype, device=go.device)
    _lib.check(_lib.lib().vo_length_regulate_bwd(_ptr(go), vo_dtype(go), _ptr(dur), B, T_src, D, max_len, _ptr(gx),
                                                 vo_dtype(gx), _stream(go)), "vo_length_regulate_bwd")
    return gx


# ----------------------------------------------------------------------------- variance heads

def duration_head(h, w, b, lens, d_control=1.0, want_round=True):
    B, T, D = h.shape
    pred = torch.empty((B, T), dtype=torch.float32, device=h.device)
    dr = torch.empty((B, T), dtype=torch.float32, device=h.device) if want_round else None
    d = _lib.HeadDesc()
    d.kind = HEAD_DURATION
    d.h, d.h_dtype = h.data_ptr(), vo_dtype(h)
    d.w, d.b = w.data_ptr(), float(b)
    d.lens = lens.data_ptr() if lens is not None else None
    d.B, d.T, d.D = B, T, D
    d.pred = pred.data_ptr()
    d.d_round = dr.data_ptr() if dr is not None else None
    d.d_control = float(d_control)
    d.x_dtype = vo_dtype(h)
    _lib.check(_lib.lib().vo_variance_head(ctypes.byref(d), _stream(h)), "vo_variance_head")
    return pred, dr


def energy_head(h, w, b, lens, x, bins, table, target=None, mean=0.0, std=1.0, control=1.0,
                want_index=False):
    """Energy prediction + bucketize + x += table[idx] (in place).  Returns (pred, idx)."""
    B, T, D = h.shape
    _contig(x, "x")
    pred = torch.empty((B, T), dtype=torch.float32, device=h.device)
    idx = torch.empty((B, T), dtype=torch.int32, device=h.device) if want_index else None
    tgt = _contig(target.float(), "target") if target is not None else None
    d = _lib.HeadDesc()
    d.kind = HEAD_ENERGY
    d.h, d.h_dtype = h.data_ptr(), vo_dtype(h)
    d.w, d.b = w.data_ptr(), float(b)
    d.lens = lens.data_ptr() if lens is not None else None
    d.B, d.T, d.D = B, T, D
    d.pred = pred.data_ptr()
    d.target = tgt.data_ptr() if tgt is not None else None
    d.bins, d.n_bins = bins.data_ptr(), bins.numel()
    d.e_mean, d.e_std, d.e_control = float(mean), float(std), float(control)
    d.table = table.data_ptr()
    d.x, d.x_dtype = x.data_ptr(), vo_dtype(x)
    d.idx_out = idx.data_ptr() if idx is not None else None
    _lib.check(_lib.lib().vo_variance_head(ctypes.byref(d), _stream(h)), "vo_variance_head")
    return pred, idx


def bucket_embed(x, target, bins, table):
    """Training-side energy embedding: out = x + table[bucketize(target, bins)] (out of place) ->
    (out, idx int32) (vo_bucket_embed; reference modules.py:53-64,101-104 with a target)."""
    _contig(x, "x")
    B, T, D = x.shape
    tgt = _contig(target.float(), "target")
    if tgt.shape != (B, T):
        raise ValueError(f"bucket_embed: target {tuple(tgt.shape)} vs x {tuple(x.shape)}")
    if table.dim() != 2 or table.shape[1] != D or table.dtype != torch.float32 or not table.is_contiguous():
        raise ValueError(f"bucket_embed: table must be a contiguous fp32 (n, {D}) tensor, got "
                         f"{tuple(table.shape)} {table.dtype}")
    out = torch.empty_like(x)
    idx = torch.empty((B, T), dtype=torch.int32, device=x.device)
    _lib.check(_lib.lib().vo_bucket_embed(_ptr(x), vo_dtype(x), _ptr(tgt), _ptr(bins), bins.numel(), _ptr(table),
                                          table.shape[0], B * T, D, _ptr(out), _ptr(idx), _stream(x)),
               "vo_bucket_embed")
    return out, idx


def embed_bwd(dy, idx, n_table):
    """dtable (n_table, D) fp32 = per-row sums of dy over the tokens of each index (row order)."""
    _contig(dy, "dy")
    D = dy.shape[-1]
    rows = dy.numel() // D
    dt = torch.empty((n_table, D), dtype=torch.float32, device=dy.device)
    _lib.check(_lib.lib().vo_embed_bwd(_ptr(dy), vo_dtype(dy), _ptr(idx), rows, D, n_table, _ptr(dt), _stream(dy)),
               "vo_embed_bwd")
    return dt


# ----------------------------------------------------------------------------- encoder glue

def vfe_stencil(images, conv_params, bn_params, slice_w, out_dtype):
    """images (B, 1, H, W) fp32 -> (B*n, H*slice_w) flattened stencil output."""
    images = _contig(images.float(), "images")
    B, C, H, W = images.shape
    if C != 1:
        raise ValueError("vfe_stencil: gray-scale (1 channel) images only")
    n = W // slice_w
    out = torch.empty((B * n, H * slice_w), dtype=out_dtype, device=images.device)
    _lib.check(_lib.lib().vo_vfe_stencil(_ptr(images), B, H, W, slice_w, n, _ptr(conv_params),
                                         _ptr(bn_params), conv_params.shape[0], _ptr(out),
                                         vo_dtype(out), _stream(images)), "vo_vfe_stencil")
    return out, n


def add_pos_class(x, pe=None, cls=None, cls_idx=None, per_token=False):
    """x (B, T, D) += pe[t] + cls[cls_idx[b]] (or cls[cls_idx[b, t]] when per_token), in place."""
    B, T, D = x.shape
    _contig(x, "x")
    if cls_idx is not None:
        cls_idx = _contig(cls_idx.long(), "cls_idx")
    _lib.check(_lib.lib().vo_add_pos_class(_ptr(x), vo_dtype(x), _ptr(pe), _ptr(cls), _ptr(cls_idx),
                                           1 if per_token else 0, B, T, D, _stream(x)),
               "vo_add_pos_class")
    return x


_LENS_DT = {torch.float32: 0, torch.int64: 2, torch.int32: 3}


def mask_from_lengths(lens, max_len, want_mask=True):
    """-> (mask (B, max_len) bool, True = padding; lens int32 (B,))."""
    lens = _contig(lens, "lens")
    if lens.dtype not in _LENS_DT:
        lens = lens.long()
    B = lens.shape[0]
    mask = torch.empty((B, max_len), dtype=torch.bool, device=lens.device) if want_mask else None
    l32 = torch.empty(B, dtype=torch.int32, device=lens.device)
    _lib.check(_lib.lib().vo_mask_from_lengths(_ptr(lens), _LENS_DT[lens.dtype], B, max_len,
                                               _ptr(mask), _ptr(l32), _stream(lens)),
               "vo_mask_from_lengths")
    return mask, l32


# ----------------------------------------------------------------------------- vocoder glue

def conv_post(x, w_kc, bias, slope=0.01):
    """x (B, T, C) -> tanh(conv(lrelu(x))) (B, T) fp32; w_kc (K, C) fp32."""
    _contig(x, "x")
    B, T, C = x.shape
    K = w_kc.shape[0]
    y = torch.empty((B, T), dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().vo_conv_post(_ptr(x), vo_dtype(x), _ptr(w_kc), float(bias), B, T, C, K,
                                       float(slope), _ptr(y), _stream(x)), "vo_conv_post")
    return y


def transpose_bct(x, out_dtype, ldy=None):
    """(B, C, T) fp32 -> (B, T, ldy) channels-last with zero channel padding."""
    x = _contig(x.float(), "x")
    B, C, T = x.shape
    ldy = ldy or C
    y = torch.empty((B, T, ldy), dtype=out_dtype, device=x.device)
    _lib.check(_lib.lib().vo_transpose_bct(_ptr(x), B, C, T, _ptr(y), vo_dtype(y), ldy, _stream(x)),
               "vo_transpose_bct")
    return y


# ----------------------------------------------------------------------------- fused ResBlock pair

def pack_frag(w_packed):
    """[K][C][C] bf16 conv pack (C = 64 / 128) -> the fragment order of the pair kernel (vo_pack_frag)."""
    _contig(w_packed, "w_packed")
    if (w_packed.dtype != torch.bfloat16 or w_packed.dim() != 3 or w_packed.shape[1] != w_packed.shape[2]
            or w_packed.shape[1] not in (64, 128)):
        raise ValueError("pack_frag: a [K][C][C] bf16 pack, C = 64 / 128")
    out = torch.empty_like(w_packed)
    _lib.check(_lib.lib().vo_pack_frag(_ptr(w_packed), _ptr(out), w_packed.shape[1], w_packed.shape[0],
                                       _stream(w_packed)), "vo_pack_frag")
    return out


def resblock_pair(x, w1, b1, w2, b2, K, dil, slope=0.1, out=None, out_scale=1.0, acc=None, tag=None, frag=False):
    """y = (x + c2(lrelu(c1_dil(lrelu(x))))) * out_scale (+ acc); x (B, T, C) bf16, C in {32, 64, 128}.
    frag: w1 / w2 are pack_frag packs (C = 64 / 128, K = 7 / 11; vo_resblock_pair_frag)."""
    _contig(x, "x")
    B, T, C = x.shape
    if x.dtype != torch.bfloat16 or w1.dtype != torch.bfloat16 or w2.dtype != torch.bfloat16:
        raise TypeError("resblock_pair: bf16 activations and packed bf16 weights")
    out = out if out is not None else torch.empty_like(x)
    if acc is not None and (acc.shape != x.shape or acc.dtype != x.dtype):
        raise ValueError("resblock_pair: acc must match x")
    timer = profiling.active()
    ev = timer.start() if (tag is not None and timer is not None and timer.watching(tag)) else None
    fn = _lib.lib().vo_resblock_pair_frag if frag else _lib.lib().vo_resblock_pair
    _lib.check(fn(_ptr(x), _ptr(w1), _ptr(b1), _ptr(w2), _ptr(b2), _ptr(out), _ptr(acc),
                  B, T, C, K, dil, float(slope), float(out_scale), _stream(x)),
               "vo_resblock_pair_frag" if frag else "vo_resblock_pair")
    if ev is not None:
        flops = 2.0 * 2.0 * B * T * C * C * K
        nbytes = 2.0 * x.numel() * 2 + (x.numel() * 2 if acc is not None else 0) + 2 * w1.numel() * 2
        name = "mrf_prw_kernel" if (C in (64, 128) and K in (7, 11)) else "mrf_pair_kernel"  # vo_pair_rw_try
        timer.stop(tag, ev, flops, nbytes, kernel=f"{name}<C={C}, ...>")
    return out


def resblock3(x, w1s, b1s, w2s, b2s, dils, slope=0.1, out=None, out_scale=1.0, acc=None, tag=None):
    """A whole K = 3 ResBlock1 (three (c1_d, c2) pairs) in one launch (vo_resblock3):
    y = x_3 * out_scale (+ acc); x (B, T, C) bf16, C in {32, 64, 128}; w1s / w2s: three packed
    [3][C][C] bf16 weights each, b1s / b2s three fp32 biases, dils the three dilations."""
    _contig(x, "x")
    B, T, C = x.shape
    if x.dtype != torch.bfloat16 or any(w.dtype != torch.bfloat16 for w in list(w1s) + list(w2s)):
        raise TypeError("resblock3: bf16 activations and packed bf16 weights")
    if not (len(w1s) == len(b1s) == len(w2s) == len(b2s) == len(dils) == 3):
        raise ValueError("resblock3: three stages")
    out = out if out is not None else torch.empty_like(x)
    if acc is not None and (acc.shape != x.shape or acc.dtype != x.dtype):
        raise ValueError("resblock3: acc must match x")
    arr = lambda ts: (ctypes.c_void_p * 3)(*[t.data_ptr() for t in ts])  # noqa: E731
    dil = (ctypes.c_int * 3)(*[int(d) for d in dils])
    timer = profiling.active()
    ev = timer.start() if (tag is not None and timer is not None and timer.watching(tag)) else None
    _lib.check(_lib.lib().vo_resblock3(_ptr(x), arr(w1s), arr(b1s), arr(w2s), arr(b2s), dil, _ptr(out), _ptr(acc),
                                       B, T, C, float(slope), float(out_scale), _stream(x)), "vo_resblock3")
    if ev is not None:
        flops = 3 * 2.0 * 2.0 * B * T * C * C * 3
        nbytes = 2.0 * x.numel() * 2 + (x.numel() * 2 if acc is not None else 0) + 6 * w1s[0].numel() * 2
        timer.stop(tag, ev, flops, nbytes, kernel=f"mrf_rb3_kernel<C={C}, ...>")
    return out


# ----------------------------------------------------------------------------- mel / STFT

def stft_mel(wav, window, fb, n_fft=1024, hop=256, n_mels=80, log_floor=1e-5):
    """wav (B, N) fp32 -> (log-mel (B, n_mels, 1 + N // hop), energy (B, 1 + N // hop))."""
    _contig(wav, "wav")
    B, N = wav.shape
    F = 1 + N // hop
    mel = torch.empty((B, n_mels, F), dtype=torch.float32, device=wav.device)
    energy = torch.empty((B, F), dtype=torch.float32, device=wav.device)
    _lib.check(_lib.lib().vo_stft_mel(_ptr(wav), B, N, _ptr(window), _ptr(fb), n_fft, hop, n_mels,
                                      float(log_floor), _ptr(mel), _ptr(energy), _stream(wav)),
               "vo_stft_mel")
    return mel, energy


def stft_mel_ex(wav, window, fb, n_fft=1024, hop=256, n_mels=80, pad=None, mag_eps=0.0, clip=False,
                log_floor=1e-5):
    """General framing (vo_stft_mel_ex): wav (B, N) fp32 -> log-mel (B, n_mels, F),
    F = 1 + (N + 2 pad - n_fft) // hop.  HiFi-GAN training mel: pad=(n_fft-hop)//2, mag_eps=1e-9."""
    _contig(wav, "wav")
    B, N = wav.shape
    pad = n_fft // 2 if pad is None else pad
    F = 1 + (N + 2 * pad - n_fft) // hop
    mel = torch.empty((B, n_mels, F), dtype=torch.float32, device=wav.device)
    _lib.check(_lib.lib().vo_stft_mel_ex(_ptr(wav), B, N, _ptr(window), _ptr(fb), n_fft, hop, n_mels, pad,
                                         float(mag_eps), int(bool(clip)), float(log_floor), _ptr(mel), None, None,
                                         _stream(wav)), "vo_stft_mel_ex")
    return mel


def stft_mel_bwd(wav, window, fb, gmel, n_fft=1024, hop=256, pad=None, mag_eps=1e-9, log_floor=1e-5):
    """Backward of ``stft_mel_ex`` (clip off): gmel (B, n_mels, F) = dL/dlogmel -> dL/dwav (B, N) fp32."""
    _contig(wav, "wav")
    _contig(gmel, "gmel")
    B, N = wav.shape
    n_mels = fb.shape[1]
    pad = n_fft // 2 if pad is None else pad
    F = 1 + (N + 2 * pad - n_fft) // hop
    if gmel.shape != (B, n_mels, F) or gmel.dtype != torch.float32 or wav.dtype != torch.float32:
        raise ValueError(f"stft_mel_bwd: gmel {tuple(gmel.shape)} {gmel.dtype} vs ({B}, {n_mels}, {F}) fp32")
    L = _lib.lib()
    dwav = torch.empty_like(wav)
    ws = torch.empty(int(L.vo_stft_mel_bwd_workspace_size(B, N, n_fft, hop, pad)) // 4, dtype=torch.float32,
                     device=wav.device)
    _lib.check(L.vo_stft_mel_bwd(_ptr(wav), B, N, _ptr(window), _ptr(fb), n_fft, hop, n_mels, pad, float(mag_eps),
                                 float(log_floor), _ptr(gmel), _ptr(dwav), _ptr(ws), _stream(wav)), "vo_stft_mel_bwd")
    return dwav


def stft_mag(wav, window, n_fft, hop, eps=1e-7):
    """torch.stft(center=True, reflect, onesided) magnitude sqrt(max(|X|^2, eps)) of wav (B, N) fp32
    with ``window`` zero-padded to n_fft -> (B, 1 + N // hop, n_fft // 2 + 1)."""
    _contig(wav, "wav")
    B, N = wav.shape
    if window.numel() != n_fft:
        raise ValueError("stft_mag: window must be zero-padded to n_fft")
    mag = torch.empty((B, 1 + N // hop, n_fft // 2 + 1), dtype=torch.float32, device=wav.device)
    _lib.check(_lib.lib().vo_stft_mag(_ptr(wav), B, N, _ptr(window), n_fft, hop, float(eps), _ptr(mag), _stream(wav)),
               "vo_stft_mag")
    return mag


def stft_mag_bwd(wav, window, gmag, n_fft, hop, eps=1e-7):
    """Backward of ``stft_mag``: gmag (B, F, bins) -> dL/dwav (B, N) fp32."""
    _contig(wav, "wav")
    _contig(gmag, "gmag")
    B, N = wav.shape
    if gmag.shape != (B, 1 + N // hop, n_fft // 2 + 1):
        raise ValueError("stft_mag_bwd: gmag shape")
    L = _lib.lib()
    dwav = torch.empty_like(wav)
    ws = torch.empty(int(L.vo_stft_mag_bwd_workspace_size(B, N, n_fft, hop)) // 4, dtype=torch.float32,
                     device=wav.device)
    _lib.check(L.vo_stft_mag_bwd(_ptr(wav), B, N, _ptr(window), n_fft, hop, float(eps), _ptr(gmag), _ptr(dwav),
                                 _ptr(ws), _stream(wav)), "vo_stft_mag_bwd")
    return dwav


def stft_loss_sums(xm, ym):
    """(sum (y - x)^2, sum y^2, sum |log y - log x|) over two magnitude tensors -> fp32 (3,)."""
    _contig(xm, "xm")
    _contig(ym, "ym")
    if xm.shape != ym.shape:
        raise ValueError("stft_loss_sums: shape mismatch")
    out = torch.empty(3, dtype=torch.float32, device=xm.device)
    ws = torch.empty(3 * 512, dtype=torch.float32, device=xm.device)
    _lib.check(_lib.lib().vo_stft_loss(_ptr(xm), _ptr(ym), xm.numel(), _ptr(out), _ptr(ws), _stream(xm)),
               "vo_stft_loss")
    return out


def stft_loss_grad(xm, ym, sums, w):
    """d(w[0] * spectral convergence + w[1] * log-magnitude L1)/dxm; w: fp32 (2,) on the device."""
    w = w.float().contiguous()
    gx = torch.empty_like(xm)
    _lib.check(_lib.lib().vo_stft_loss_grad(_ptr(xm), _ptr(ym), xm.numel(), _ptr(sums), _ptr(w), _ptr(gx),
                                            _stream(xm)), "vo_stft_loss_grad")
    return gx


# ----------------------------------------------------------------------------- training BatchNorm / glyph conv

def _rows(x):
    """Channels-last view as (M, C); a single-channel map (N, 1, H, W) is M = every pixel, C = 1."""
    _contig(x, "x")
    C = x.shape[-1] if x.dim() != 4 else x.shape[1]
    if x.dim() == 4 and C != 1:
        raise ValueError("bn: 4-d input must be single-channel (N, 1, H, W)")
    return x.numel() // C, C


def bn_train_fwd(x, gamma, beta, eps, momentum, running_mean=None, running_var=None, num_batches=None):
    """BatchNorm with batch statistics over channels-last x (..., C) or (N, 1, H, W) in fp32 / bf16:
    (y in x's dtype, mean_rstd (2C) fp32); running stats / num_batches updated in place when given."""
    M, C = _rows(x)
    L = _lib.lib()
    y = torch.empty_like(x)
    mr = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    ws = torch.empty(int(L.vo_bn_workspace_size(M, C)) // 4, dtype=torch.float32, device=x.device)
    for t, n in ((gamma, "gamma"), (beta, "beta"), (running_mean, "running_mean"), (running_var, "running_var")):
        if t is not None and (t.dtype != torch.float32 or t.numel() != C or not t.is_contiguous()):
            raise ValueError(f"bn_train_fwd: {n} must be contiguous fp32 of {C}")
    if num_batches is not None and num_batches.dtype != torch.int64:
        raise ValueError("bn_train_fwd: num_batches must be int64")
    _lib.check(L.vo_bn_train_fwd(_ptr(x), vo_dtype(x), M, C, _ptr(gamma), _ptr(beta), float(eps), float(momentum),
                                 _ptr(running_mean), _ptr(running_var), _ptr(num_batches), _ptr(mr), _ptr(ws), _ptr(y),
                                 _stream(x)), "vo_bn_train_fwd")
    return y, mr


def dropout(x, p, seed, salt=0, out=None):
    """Training dropout (vo_dropout): x / (1 - p) where hash(seed, salt, i) >= p 2^32, else 0; ``seed`` a
    device int64 tensor (one element), ``salt`` the dropout site.  The same call on a gradient with the
    same seed and salt is the backward."""
    _contig(x, "x")
    if x.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError("dropout: fp32 / bf16")
    if seed.dtype != torch.int64 or seed.numel() < 1 or seed.device != x.device:
        raise ValueError("dropout: seed must be an int64 tensor on x's device")
    out = out if out is not None else torch.empty_like(x)
    _lib.check(_lib.lib().vo_dropout(_ptr(x), vo_dtype(x), x.numel(), float(p), _ptr(seed), int(salt) & 0xFFFFFFFF,
                                     _ptr(out), _stream(x)), "vo_dropout")
    return out


def bn_bwd(x, gy, gamma, mean_rstd):
    """Backward of ``bn_train_fwd``: (dx in x's dtype, dgamma, dbeta) fp32."""
    M, C = _rows(x)
    _contig(gy, "gy")
    if gy.shape != x.shape:
        raise ValueError("bn_bwd: gy shape mismatch")
    L = _lib.lib()
    dx = torch.empty_like(x)
    dg = torch.empty(C, dtype=torch.float32, device=x.device)
    db = torch.empty(C, dtype=torch.float32, device=x.device)
    ws = torch.empty(int(L.vo_bn_workspace_size(M, C)) // 4, dtype=torch.float32, device=x.device)
    _lib.check(L.vo_bn_bwd(_ptr(x), vo_dtype(x), _ptr(gy), vo_dtype(gy), M, C, _ptr(gamma), _ptr(mean_rstd), _ptr(ws),
                           _ptr(dg), _ptr(db), _ptr(dx), _stream(x)), "vo_bn_bwd")
    return dx, dg, db


def _vfe_shape(x):
    _contig(x, "x")
    if x.dim() != 4 or x.shape[1] != 1 or x.dtype != torch.float32:
        raise ValueError(f"vfe conv: x must be (N, 1, H, W) fp32, got {tuple(x.shape)} {x.dtype}")
    return x.shape[0], x.shape[2], x.shape[3]


def vfe_conv_fwd(x, w10):
    """Conv2d(1, 1, 3, padding=1): x (N, 1, H, W) fp32, w10 = 9 kernel taps (row-major) + bias."""
    N, H, W = _vfe_shape(x)
    y = torch.empty_like(x)
    _lib.check(_lib.lib().vo_vfe_conv_fwd(_ptr(x), N, H, W, _ptr(w10), _ptr(y), _stream(x)), "vo_vfe_conv_fwd")
    return y


def vfe_conv_bwd(x, gy, w10):
    """Backward of ``vfe_conv_fwd``: (dx, dw10)."""
    N, H, W = _vfe_shape(x)
    _contig(gy, "gy")
    if gy.shape != x.shape or gy.dtype != torch.float32:
        raise ValueError("vfe_conv_bwd: gy must match x")
    L = _lib.lib()
    dx = torch.empty_like(x)
    dw = torch.empty(10, dtype=torch.float32, device=x.device)
    ws = torch.empty(int(L.vo_vfe_conv_workspace_size(N, H, W)) // 4, dtype=torch.float32, device=x.device)
    _lib.check(L.vo_vfe_conv_bwd(_ptr(x), _ptr(gy), N, H, W, _ptr(w10), _ptr(dx), _ptr(dw), _ptr(ws), _stream(x)),
               "vo_vfe_conv_bwd")
    return dx, dw


# ----------------------------------------------------------------------------- HiFi-GAN training (C5)

def pack_grouped_weight(w, dtype, groups=1, ci_pad=None, out=None):
    """(Co, Ci/groups, K) fp32 -> dense [K][Co][Ci_pad] block-diagonal (vo_conv1d groups mode).
    ``out``: a buffer of that shape and dtype whose entries outside the diagonal blocks are zero
    (a persistent packed weight): only the blocks are rewritten (vo_pack_grouped_blocks)."""
    w = w.detach().float().contiguous()
    Co, cig, K = w.shape
    Ci = cig * groups
    ci_pad = Ci if ci_pad is None else ci_pad
    if out is not None:
        if tuple(out.shape) != (K, Co, ci_pad) or out.dtype != dtype or not out.is_contiguous():
            raise ValueError(f"pack_grouped_weight: out {tuple(out.shape)} {out.dtype}, "
                             f"expected contiguous {(K, Co, ci_pad)} {dtype}")
        _lib.check(_lib.lib().vo_pack_grouped_blocks(_ptr(w), Co, Ci, K, groups, ci_pad, _ptr(out),
                                                     vo_dtype(dtype), _stream(w)), "vo_pack_grouped_blocks")
        return out
    out = torch.empty((K, Co, ci_pad), dtype=dtype, device=w.device)
    _lib.check(_lib.lib().vo_pack_grouped(_ptr(w), Co, Ci, K, groups, ci_pad, _ptr(out), vo_dtype(dtype),
                                          _stream(w)), "vo_pack_grouped")
    return out


PJ_GATHER, PJ_CONVT = 0, 1
_PJ_FIELDS = ("mode", "swap", "T", "rows", "width", "dst_rows", "ld", "rpg", "cpg", "cig", "K", "tap0", "tstep",
              "src_rows")


def pack_batch(jobs, dtype):
    """Many weight packs in one launch (vo_pack_batch; layouts in include/vonoma.h): jobs is a list of
    (src fp32 contiguous, dst contiguous tensor of ``dtype``, {field: int}[, element offset of the job's
    block in dst]).  Entries of dst a job does not name are left as they are."""
    if not jobs:
        return
    arr = (_lib.PackJob * len(jobs))()
    for e, job in zip(arr, jobs):
        src, dst, f = job[:3]
        off = job[3] if len(job) > 3 else None  # element offset of the job's (0, 0) in dst (a block of it)
        _contig(src, "src")
        _contig(dst, "dst")
        if src.dtype != torch.float32 or dst.dtype != dtype:
            raise ValueError("pack_batch: src must be fp32 and dst the batch dtype")
        rows_total = f["T"] * f["dst_rows"] * f["ld"]
        if off is None and dst.numel() != rows_total:
            raise ValueError(f"pack_batch: dst has {dst.numel()} elements, the job's layout {rows_total}")
        if off is not None:  # the last element the job writes must lie in dst
            last = (off + (f["T"] - 1) * f["dst_rows"] * f["ld"] + (f["rows"] - 1) * f["ld"] +
                    ((f["rows"] - 1) // f["rpg"]) * f["cpg"] + f["width"])
            if off < 0 or last > dst.numel():
                raise ValueError(f"pack_batch: a block at {off} of {dst.numel()} elements ends at {last}")
        e.src, e.dst = src.data_ptr(), dst.data_ptr() + (off or 0) * dst.element_size()
        for k in _PJ_FIELDS:
            setattr(e, k, int(f[k]))
    _lib.check(_lib.lib().vo_pack_batch(len(jobs), ctypes.cast(arr, ctypes.c_void_p), vo_dtype(dtype),
                                        _stream(jobs[0][1])), "vo_pack_batch")


def seq_remap(src, dst_rows, Td, Ss, lo, hi, shift):
    """Rows of a channels-last tensor remapped (vo_seq_remap): returns (dst_rows, C) with row
    r = (n, t) (n = r // Td, t = r % Td) = src row n Ss + t + shift for lo <= t < hi, else 0.
    ``src``: contiguous, its last dim the row."""
    _contig(src, "src")
    C = src.shape[-1]
    rows = src.numel() // C
    dst = torch.empty((dst_rows, C), dtype=src.dtype, device=src.device)
    _lib.check(_lib.lib().vo_seq_remap(_ptr(src), rows, _ptr(dst), dst_rows, C * src.element_size(), Td, Ss, lo, hi,
                                       shift, _stream(src)), "vo_seq_remap")
    return dst


def seq_remap2(jobs):
    """One or two remaps in one launch (vo_seq_remap2): each job a dict(src, dst_rows, Td, Ss, lo, hi,
    shift[, src2, Ss2, shift2]) -> its (dst_rows, C) tensor: row r = (n, t) (n = r // Td, t = r % Td)
    = src row n Ss + t + shift (+ src2 row n Ss2 + t + shift2, added in the dtype) for lo <= t < hi,
    else 0.  Sources contiguous with the same row (C) and dtype, rows of whole 16-byte units."""
    if not 1 <= len(jobs) <= 2:
        raise ValueError("seq_remap2: one or two jobs")
    ref = jobs[0]["src"]
    C = ref.shape[-1]
    arr = (_lib.RemapJob * len(jobs))()
    outs = []
    for i, j in enumerate(jobs):
        src, src2 = j["src"], j.get("src2")
        for t in (src, src2):
            if t is not None:
                _contig(t, "src")
                if t.shape[-1] != C or t.dtype != ref.dtype:
                    raise ValueError("seq_remap2: sources must share the row and dtype")
        dst = torch.empty((j["dst_rows"], C), dtype=ref.dtype, device=ref.device)
        outs.append(dst)
        a = arr[i]
        a.src, a.dst = src.data_ptr(), dst.data_ptr()
        a.src2 = src2.data_ptr() if src2 is not None else None
        a.src_rows = src.numel() // C
        a.src2_rows = src2.numel() // C if src2 is not None else 0
        a.dst_rows, a.Td, a.Ss, a.lo, a.hi, a.shift = j["dst_rows"], j["Td"], j["Ss"], j["lo"], j["hi"], j["shift"]
        a.Ss2, a.shift2 = j.get("Ss2", 0), j.get("shift2", 0)
    _lib.check(_lib.lib().vo_seq_remap2(len(jobs), arr, C * ref.element_size(), vo_dtype(ref), _stream(ref)),
               "vo_seq_remap2")
    return outs


def pack_dgrad_phase(w, groups, S, k_r, J, ci_out, co_in, dtype, out=None):
    """Stride phase k_r of a strided / grouped conv's input gradient: w (Co, Ci/groups, K) -> packed
    [J][ci_out][co_in] (taps k_r + S (J - 1 - t), channel roles swapped per group, zero padding).
    ``out``: a persistent buffer of that shape, zero outside the diagonal blocks (only they are written)."""
    w = w.detach().float().contiguous()
    Co, cig, K = w.shape
    shape = (J, ci_out, co_in)
    if out is not None:
        if tuple(out.shape) != shape or out.dtype != dtype or not out.is_contiguous():
            raise ValueError(f"pack_dgrad_phase: out {tuple(out.shape)} {out.dtype}, expected contiguous {shape} {dtype}")
    dst = out if out is not None else torch.empty(shape, dtype=dtype, device=w.device)
    _lib.check(_lib.lib().vo_pack_dgrad_phase(_ptr(w), Co, cig, K, groups, S, k_r, J, ci_out, co_in,
                                              1 if out is not None else 0, _ptr(dst), vo_dtype(dtype), _stream(w)),
               "vo_pack_dgrad_phase")
    return dst


def period_fold(wav, period, dtype):
    """wav (B, T) fp32 -> (B * period, ceil(T / period), 8) channels-last (MPD input)."""
    _contig(wav, "wav")
    B, T = wav.shape
    H = (T + period - 1) // period
    out = torch.empty((B * period, H, 8), dtype=dtype, device=wav.device)
    _lib.check(_lib.lib().vo_period_fold(_ptr(wav), B, T, period, _ptr(out), vo_dtype(dtype), _stream(wav)),
               "vo_period_fold")
    return out


def wav_cl8(wav, dtype):
    """(B, T) fp32 -> (B, T, 8) channels-last, channel 0 = wav (MSD input)."""
    _contig(wav, "wav")
    out = torch.empty(wav.shape + (8,), dtype=dtype, device=wav.device)
    _lib.check(_lib.lib().vo_wav_cl8(_ptr(wav), wav.numel(), _ptr(out), vo_dtype(dtype), _stream(wav)),
               "vo_wav_cl8")
    return out


def avgpool_wav(wav):
    """AvgPool1d(4, 2, padding=2) over (B, T) fp32 -> (B, T // 2 + 1)."""
    _contig(wav, "wav")
    B, T = wav.shape
    out = torch.empty((B, T // 2 + 1), dtype=torch.float32, device=wav.device)
    _lib.check(_lib.lib().vo_avgpool_wav(_ptr(wav), B, T, _ptr(out), _stream(wav)), "vo_avgpool_wav")
    return out


def period_fold_bwd(g, B, T, period):
    """Adjoint of ``period_fold``: g (B * period, H, 8) -> dL/dwav (B, T) fp32."""
    _contig(g, "g")
    H = (T + period - 1) // period
    if g.shape != (B * period, H, 8):
        raise ValueError(f"period_fold_bwd: g {tuple(g.shape)} vs ({B * period}, {H}, 8)")
    gw = torch.empty((B, T), dtype=torch.float32, device=g.device)
    _lib.check(_lib.lib().vo_period_fold_bwd(_ptr(g), vo_dtype(g), B, T, period, _ptr(gw), _stream(g)),
               "vo_period_fold_bwd")
    return gw


def _ptr_table(ts):
    return ctypes.cast((ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts]), ctypes.c_void_p)


def _wn_check(vs, gs):
    if len(vs) != len(gs):
        raise ValueError("weight_norm: as many g as v")
    for v, g in zip(vs, gs):
        _contig(v, "v")
        _contig(g, "g")
        if v.dtype != torch.float32 or g.dtype != torch.float32:
            raise ValueError("weight_norm: fp32 v and g")
        if g.numel() != v.shape[0] or v.device != vs[0].device:
            raise ValueError(f"weight_norm: g {tuple(g.shape)} vs v {tuple(v.shape)} (one gain per row of dim 0)")
    rows = [v.shape[0] for v in vs]
    lens = [v.numel() // v.shape[0] for v in vs]
    return (ctypes.c_int * len(vs))(*rows), (ctypes.c_int * len(vs))(*lens)


def weight_norm(vs, gs):
    """w_k = g_k * v_k / ||v_k||, norms over every dim but 0 (torch._weight_norm(v, g, 0)), for a list
    of layers in one launch per 24 layers (vo_weight_norm) -> list of w."""
    if not vs:
        return []
    rows, lens = _wn_check(vs, gs)
    ws = [torch.empty_like(v) for v in vs]
    _lib.check(_lib.lib().vo_weight_norm(len(vs), _ptr_table(vs), _ptr_table(gs), _ptr_table(ws), rows, lens,
                                          _stream(vs[0])), "vo_weight_norm")
    return ws


def spectral_norm(Ws, us, vs, power, eps=1e-12):
    """torch.nn.utils.spectral_norm's weight for many layers (vo_spectral_norm): Ws = weight_orig
    (rows, ...) fp32, us / vs the u / v buffers (updated in place when ``power``) -> (w list, the u and
    v copies sigma used, sigma list (1-element tensors))."""
    n = len(Ws)
    if n == 0:
        return [], [], [], []
    arr = (_lib.SnLayer * n)()
    outs = []
    for e, W, u, v in zip(arr, Ws, us, vs):
        for t, name in ((W, "W"), (u, "u"), (v, "v")):
            _contig(t, name)
            if t.dtype != torch.float32:
                raise ValueError(f"spectral_norm: {name} must be fp32")
        rows, L = W.shape[0], W.numel() // W.shape[0]
        if u.numel() != rows or v.numel() != L:
            raise ValueError("spectral_norm: u / v do not match the weight")
        o = dict(u_out=torch.empty_like(u), v_out=torch.empty_like(v), vraw=torch.empty_like(v),
                 s=torch.empty_like(u), sigma=torch.empty(1, dtype=torch.float32, device=W.device),
                 w=torch.empty_like(W))
        outs.append(o)
        e.W, e.u, e.v = W.data_ptr(), u.data_ptr(), v.data_ptr()
        for k in ("u_out", "v_out", "vraw", "s", "sigma", "w"):
            setattr(e, k, o[k].data_ptr())
        e.rows, e.L = rows, L
    _lib.check(_lib.lib().vo_spectral_norm(n, ctypes.cast(arr, ctypes.c_void_p), 1 if power else 0, float(eps),
                                           _stream(Ws[0])), "vo_spectral_norm")
    return [o["w"] for o in outs], [o["u_out"] for o in outs], [o["v_out"] for o in outs], [o["sigma"] for o in outs]


def spectral_norm_bwd(gs, Ws, us, vs, sigmas):
    """Gradients wrt weight_orig of spectral_norm's weights (vo_spectral_norm_bwd): gs / Ws (rows, ...)
    fp32, us / vs / sigmas as the forward used them -> [gW] (gW = g / s - (sum(g W) / s^2) u v^T)."""
    n = len(gs)
    arr = (_lib.SnBwdLayer * n)()
    outs = []
    keep = []
    for e, g, W, u, v, sg in zip(arr, gs, Ws, us, vs, sigmas):
        g = g.float().contiguous()
        for t, name in ((W, "W"), (u, "u"), (v, "v"), (sg, "sigma")):
            _contig(t, name)
        if g.shape != W.shape:
            raise ValueError("spectral_norm_bwd: gradient and weight shapes differ")
        o = torch.empty_like(W)
        outs.append(o)
        keep.append(g)
        e.g, e.W, e.u, e.v, e.sigma, e.gW = g.data_ptr(), W.data_ptr(), u.data_ptr(), v.data_ptr(), sg.data_ptr(), o.data_ptr()
        e.rows, e.L = W.shape[0], W.numel() // W.shape[0]
    L = _lib.lib()
    p = ctypes.cast(arr, ctypes.c_void_p)
    ws = torch.empty(max(1, int(L.vo_spectral_norm_bwd_workspace_size(n, p)) // 4), dtype=torch.float32,
                     device=Ws[0].device)
    _lib.check(L.vo_spectral_norm_bwd(n, p, _ptr(ws), _stream(Ws[0])), "vo_spectral_norm_bwd")
    return outs


def weight_norm_bwd(vs, gs, dws):
    """Backward of ``weight_norm``: lists of dL/dw -> (dL/dv list, dL/dg list)."""
    if not vs:
        return [], []
    rows, lens = _wn_check(vs, gs)
    for v, d in zip(vs, dws):
        _contig(d, "dw")
        if d.shape != v.shape or d.dtype != torch.float32:
            raise ValueError("weight_norm_bwd: dw must match v (fp32)")
    dvs = [torch.empty_like(v) for v in vs]
    dgs = [torch.empty_like(g) for g in gs]
    _lib.check(_lib.lib().vo_weight_norm_bwd(len(vs), _ptr_table(vs), _ptr_table(gs), _ptr_table(dws),
                                              _ptr_table(dvs), _ptr_table(dgs), rows, lens, _stream(vs[0])),
               "vo_weight_norm_bwd")
    return dvs, dgs


def wav_cl8_bwd(g):
    """Adjoint of ``wav_cl8``: g (B, T, 8) -> (B, T) fp32 (channel 0)."""
    _contig(g, "g")
    if g.shape[-1] != 8:
        raise ValueError("wav_cl8_bwd: g must end in 8 channels")
    gw = torch.empty(g.shape[:-1], dtype=torch.float32, device=g.device)
    _lib.check(_lib.lib().vo_wav_cl8_bwd(_ptr(g), vo_dtype(g), gw.numel(), _ptr(gw), _stream(g)), "vo_wav_cl8_bwd")
    return gw


def avgpool_wav_bwd(g, T):
    """Adjoint of ``avgpool_wav``: g (B, T // 2 + 1) fp32 -> (B, T) fp32."""
    _contig(g, "g")
    B = g.shape[0]
    if g.shape[1] != T // 2 + 1 or g.dtype != torch.float32:
        raise ValueError("avgpool_wav_bwd: g must be (B, T // 2 + 1) fp32")
    gx = torch.empty((B, T), dtype=torch.float32, device=g.device)
    _lib.check(_lib.lib().vo_avgpool_wav_bwd(_ptr(g), B, T, _ptr(gx), _stream(g)), "vo_avgpool_wav_bwd")
    return gx


GAN_L1, GAN_ONE_MINUS_SQ, GAN_SQ = 0, 1, 2


def _rows_view(t):
    """(..., width) view with unit column stride -> (rows, width, ld) for the reductions."""
    if t.stride(-1) != 1:
        raise ValueError("gan_reduce: last dim must be contiguous")
    width = t.shape[-1]
    lead = t.reshape(-1, width) if t.dim() != 2 else t
    if lead.dim() != 2 or (lead.shape[0] > 1 and lead.stride(0) < width):
        raise ValueError("gan_reduce: view not expressible as rows x width")
    return lead, lead.shape[0], width, lead.stride(0) if lead.shape[0] > 1 else width


def gan_reduce(kind, a, b=None, out=None):
    """sum over a of |a - b| (GAN_L1), (1 - a)^2 or a^2 -> fp32 scalar tensor (accumulated into out)."""
    la, rows, width, lda = _rows_view(a)
    ldb = 0
    if b is not None:
        lb, rb, wb, ldb = _rows_view(b)
        if (rb, wb) != (rows, width) or b.dtype != a.dtype:
            raise ValueError("gan_reduce: a / b mismatch")
        b = lb
    if out is None:
        out = torch.zeros((), dtype=torch.float32, device=a.device)
    ws = torch.empty(512, dtype=torch.float32, device=a.device)  # block partials (deterministic sum)
    _lib.check(_lib.lib().vo_gan_reduce(kind, _ptr(la), lda, _ptr(b), ldb, rows, width, vo_dtype(a), _ptr(out),
                                        _ptr(ws), _stream(a)), "vo_gan_reduce")
    return out


def gan_reduce_grad(kind, a, b, scale, out=None):
    """d(scale * sum)/da in a contiguous tensor shaped like a (scale: fp32 device scalar); ``out``: a
    contiguous tensor of a's dtype and size to write it into (returned reshaped like a)."""
    la, rows, width, lda = _rows_view(a)
    ldb = 0
    if b is not None:
        b, _, _, ldb = _rows_view(b)
    if out is not None:
        if not out.is_contiguous() or out.numel() != rows * width or out.dtype != a.dtype:
            raise ValueError("gan_reduce_grad: out must be contiguous, of a's dtype and size")
        ga = out
    else:
        ga = torch.empty((rows, width), dtype=a.dtype, device=a.device)
    _lib.check(_lib.lib().vo_gan_reduce_grad(kind, _ptr(la), lda, _ptr(b), ldb, rows, width, vo_dtype(a),
                                             _ptr(scale.float().contiguous()), _ptr(ga), width, _stream(a)),
               "vo_gan_reduce_grad")
    return ga.reshape(a.shape)


def _gan_terms(kinds, As, Bs, outs=None):
    arr = (_lib.GanTerm * len(kinds))()
    keep = []
    for i, (k, a, b) in enumerate(zip(kinds, As, Bs)):
        la, rows, width, lda = _rows_view(a)
        e = arr[i]
        e.kind, e.a, e.lda, e.rows, e.width = k, la.data_ptr(), lda, rows, width
        keep.append(la)
        if b is not None:
            lb, rb, wb, ldb = _rows_view(b)
            if (rb, wb) != (rows, width) or b.dtype != a.dtype:
                raise ValueError("gan_reduce_multi: a / b mismatch")
            e.b, e.ldb = lb.data_ptr(), ldb
            keep.append(lb)
        if outs is not None:
            o = outs[i]
            if not o.is_contiguous() or o.numel() != rows * width or o.dtype != a.dtype:
                raise ValueError("gan_reduce_grad_multi: out must be contiguous, of a's dtype and size")
            e.ga, e.ldg = o.data_ptr(), width
    if any(a.dtype != As[0].dtype for a in As):
        raise ValueError("gan_reduce_multi: one dtype for all terms")
    return arr, keep


def gan_reduce_multi(kinds, As, Bs, scale=None):
    """[gan_reduce(kinds[i], As[i], Bs[i])] * scale as one (n,) fp32 vector in one launch pair
    (vo_gan_reduce_multi; each sum bit for bit gan_reduce's).  ``scale``: (n,) fp32 device vector."""
    n = len(kinds)
    arr, keep = _gan_terms(kinds, As, Bs)
    out = torch.empty(n, dtype=torch.float32, device=As[0].device)
    L = _lib.lib()
    ws = torch.empty(int(L.vo_gan_reduce_multi_workspace_size(n)) // 4, dtype=torch.float32, device=As[0].device)
    sc = scale.float().contiguous() if scale is not None else None
    _lib.check(L.vo_gan_reduce_multi(n, ctypes.cast(arr, ctypes.c_void_p), vo_dtype(As[0]), _ptr(sc), _ptr(out),
                                     _ptr(ws), _stream(As[0])), "vo_gan_reduce_multi")
    del keep
    return out


def gan_reduce_grad_multi(kinds, As, Bs, scale, outs=None):
    """[gan_reduce_grad(kinds[i], As[i], Bs[i], scale[i])] in one launch (vo_gan_reduce_grad_multi);
    ``outs``: contiguous tensors to write them into (default: new tensors shaped like As)."""
    if outs is None:
        outs = [torch.empty(a.shape, dtype=a.dtype, device=a.device) for a in As]
    arr, keep = _gan_terms(kinds, As, Bs, outs)
    sc = scale.float().contiguous()
    _lib.check(_lib.lib().vo_gan_reduce_grad_multi(len(kinds), ctypes.cast(arr, ctypes.c_void_p), vo_dtype(As[0]),
                                                   _ptr(sc), _stream(As[0])), "vo_gan_reduce_grad_multi")
    del keep
    return outs


# ----------------------------------------------------------------------------- training input pipeline

def glyph_batch(strips, char_widths, cell, margin, device, W_out=None):
    """Grayscale uint8 strips (list of (H, W_b)) + per-character widths (list of int arrays, or
    None for already-centred strips) -> (B, 1, H, W_out) fp32 on ``device`` (vo_glyph_batch:
    per-character centring into ``cell`` columns, white padding, ToTensor)."""
    B = len(strips)
    H = int(strips[0].shape[0])
    widths = [int(s.shape[1]) for s in strips]
    if any(int(s.shape[0]) != H for s in strips):
        raise ValueError("glyph_batch: strips must share their height")
    offs = np.zeros(B, np.int64)
    offs[1:] = np.cumsum([H * w for w in widths])[:-1]
    packed = np.concatenate([np.ascontiguousarray(s, dtype=np.uint8).reshape(-1) for s in strips])
    if char_widths is not None:
        cw = [np.asarray(w, np.int64).reshape(-1) for w in char_widths]
        if any(int(w.max(initial=0)) > cell for w in cw):
            raise ValueError(f"glyph_batch: a character is wider than the {cell}-pixel cell")
        for w, s in zip(cw, widths):
            if int(w.sum()) > s:
                raise ValueError("glyph_batch: character widths exceed the strip")
        char_off = np.zeros(B + 1, np.int32)
        char_off[1:] = np.cumsum([len(w) for w in cw])
        starts = np.concatenate([np.concatenate([[0], np.cumsum(w)[:-1]]) if len(w) else np.zeros(0, np.int64)
                                 for w in cw]).astype(np.int32)
        lens = np.concatenate(cw).astype(np.int32)
        w_out = max(len(w) for w in cw) * cell + 2 * margin
    else:
        char_off = starts = lens = None
        w_out = max(widths) + 2 * margin
    W_out = W_out or w_out
    dev = torch.device(device)
    t = lambda a: torch.from_numpy(a).to(dev, non_blocking=True) if a is not None else None  # noqa: E731
    px_d, off_d, w_d = t(packed), t(offs), t(np.asarray(widths, np.int32))
    co_d, cs_d, cl_d = t(char_off), t(starts), t(lens)
    out = torch.empty((B, 1, H, W_out), dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().vo_glyph_batch(_ptr(px_d), _ptr(off_d), _ptr(w_d), _ptr(co_d), _ptr(cs_d), _ptr(cl_d), B,
                                         H, int(cell), int(margin), int(W_out), _ptr(out), _stream(out)),
               "vo_glyph_batch")
    return out


# ----------------------------------------------------------------------------- offline feature extraction

def spec_features(wav, window, fb, n_fft=1024, hop=256, log_floor=1e-5):
    """torchaudio-framed log-mel (B, n_mels, F), frame energy (B, F) and per-frame power
    statistics (B, F, 2) of wav (B, N) (vo_stft_mel_ex, clipped input, center=True)."""
    _contig(wav, "wav")
    B, N = wav.shape
    F = 1 + N // hop
    mel = torch.empty((B, fb.shape[1], F), dtype=torch.float32, device=wav.device)
    energy = torch.empty((B, F), dtype=torch.float32, device=wav.device)
    fstats = torch.empty((B, F, 2), dtype=torch.float32, device=wav.device)
    _lib.check(_lib.lib().vo_stft_mel_ex(_ptr(wav), B, N, _ptr(window), _ptr(fb), n_fft, hop, fb.shape[1],
                                         n_fft // 2, 0.0, 1, float(log_floor), _ptr(mel), _ptr(energy),
                                         _ptr(fstats), _stream(wav)), "vo_stft_mel_ex")
    return mel, energy, fstats


def char_features(energy, fstats, durations, n_bins):
    """energy (B, F), fstats (B, F, 2), durations: list of B int arrays -> (energy_char, kurtosis_char)
    lists (per-character mean energy, spectral kurtosis) via vo_char_features."""
    B, F = energy.shape
    dur = np.concatenate([np.asarray(d, np.int32).reshape(-1) for d in durations])
    off = np.zeros(B + 1, np.int32)
    off[1:] = np.cumsum([len(d) for d in durations])
    dev = energy.device
    dur_d, off_d = torch.from_numpy(dur).to(dev), torch.from_numpy(off).to(dev)
    e = torch.empty(int(off[-1]), dtype=torch.float32, device=dev)
    k = torch.empty(int(off[-1]), dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().vo_char_features(_ptr(energy.contiguous()), _ptr(fstats.contiguous()), F, _ptr(dur_d),
                                           _ptr(off_d), B, int(n_bins), _ptr(e), _ptr(k), _stream(energy)),
               "vo_char_features")
    return [e[off[i]:off[i + 1]] for i in range(B)], [k[off[i]:off[i + 1]] for i in range(B)]


# ----------------------------------------------------------------------------- training backward

def conv1d_wgrad(a, b, K, S=1, dil=1, pad=0, pre_a=None, pre_b=None, transposed=False, groups=1, with_bias=False,
                 split=False):
    """Weight gradient on MFMA (vo_conv1d_wgrad).  Conv1d: a = dY (B, T_out, Co), b = x (B, T_in, Ci)
    -> dW (Co, Ci / groups, K).  ConvTranspose1d (transposed=True): a = x (B, T_in, Ci), b = dY
    (B, T_up, Co) -> dW (Ci, Co, K).  pre_a / pre_b: leaky-ReLU slope applied to that operand
    (None = identity).  with_bias (conv form): also the bias gradient, column sums of a, from the
    same launch (vo_conv1d_wgrad_bias) -> (dW, db).  split (fp32 operands, stride 1, ungrouped): contract
    them as split-bf16 (VO_F32X3, see F32X3)."""
    _contig(a, "a")
    _contig(b, "b")
    if a.dtype != b.dtype:
        raise TypeError("conv1d_wgrad: operand dtypes differ")
    B, T_A, M = a.shape
    _, T_B, N = b.shape
    if M % groups or N % groups:
        raise ValueError(f"conv1d_wgrad: channels {M} / {N} not divisible by groups {groups}")
    if with_bias and (pre_a is not None or transposed):
        raise ValueError("conv1d_wgrad: the fused bias gradient needs the conv form with a = dY as stored")
    mg, ng = M // groups, N // groups
    L = _lib.lib()
    w = torch.empty((M, ng, K), dtype=torch.float32, device=a.device)  # written in weight order
    db = torch.empty(M, dtype=torch.float32, device=a.device) if with_bias else None
    ws = torch.empty(int(L.vo_conv1d_wgrad_workspace_size(B, T_A, mg, ng, K, groups)) // 4, dtype=torch.float32,
                     device=a.device)  # row-split partials, added in a fixed order (deterministic)
    slope = pre_a if pre_a is not None else (pre_b if pre_b is not None else 0.0)
    if pre_a is not None and pre_b is not None and pre_a != pre_b:
        raise ValueError("conv1d_wgrad: one slope for both operands")
    dt = vo_dtype(a)
    if split:
        if a.dtype != torch.float32 or S != 1 or groups != 1 or transposed:
            raise ValueError("conv1d_wgrad: split needs fp32 operands, stride 1, ungrouped, conv form")
        dt = VO_F32X3
    _lib.check(L.vo_conv1d_wgrad_bias(_ptr(a), M, T_A, _ptr(b), N, T_B, B, mg, ng, K, S, dil, pad, groups,
                                      int(pre_a is not None), int(pre_b is not None), float(slope), dt,
                                      _ptr(w), _ptr(db), _ptr(ws), _stream(a)), "vo_conv1d_wgrad")
    return (w, db) if with_bias else w


def lrelu_mask(g, ref, slope, out=None, add=None, summand=None):
    """g * (ref > 0 ? 1 : slope) (leaky-ReLU / ReLU backward); g, ref (..., C) with row-contiguous
    last dims (ref may be a channel slice of a wider tensor).  out=g computes in place.  ``add``
    (g's shape and dtype): that rounded result plus ``add`` in the same pass (vo_lrelu_mask_add).
    ``summand`` (g's shape and dtype): the mask of round(g + summand) (vo_lrelu_mask_sum)."""
    if g.shape != ref.shape:
        raise ValueError("lrelu_mask: g and ref shapes differ")
    if add is not None and summand is not None:
        raise ValueError("lrelu_mask: add or summand, not both")
    if summand is not None:
        if summand.shape != g.shape or summand.dtype != g.dtype:
            raise ValueError("lrelu_mask: summand must match g")
        C = g.shape[-1]
        g, ref, summand = g.contiguous(), ref.contiguous(), summand.contiguous()
        out = torch.empty_like(g) if out is None else _contig(out, "out")
        _lib.check(_lib.lib().vo_lrelu_mask_sum(_ptr(g), C, vo_dtype(g), _ptr(ref), C, vo_dtype(ref), _ptr(summand),
                                                C, g.numel() // C, C, float(slope), _ptr(out), C, _stream(g)),
                   "vo_lrelu_mask_sum")
        return out
    if add is not None:
        if add.shape != g.shape or add.dtype != g.dtype:
            raise ValueError("lrelu_mask: add must match g")
        C = g.shape[-1]
        g, ref, add = g.contiguous(), ref.contiguous(), add.contiguous()
        out = torch.empty_like(g) if out is None else _contig(out, "out")
        _lib.check(_lib.lib().vo_lrelu_mask_add(_ptr(g), C, vo_dtype(g), _ptr(ref), C, vo_dtype(ref), _ptr(add), C,
                                                g.numel() // C, C, float(slope), _ptr(out), C, _stream(g)),
                   "vo_lrelu_mask_add")
        return out
    C = g.shape[-1]

    def row_strided(t):  # (..., C) rows at a common stride (a channel slice of a wider tensor is fine)
        return t.dim() >= 2 and t.stride(-1) == 1 and all(
            t.stride(i) == t.stride(i + 1) * t.shape[i + 1] for i in range(t.dim() - 2))
    if not row_strided(g):
        g, out = g.contiguous(), None
    if not row_strided(ref):
        ref = ref.contiguous()
    if out is not None and not row_strided(out):
        raise ValueError("lrelu_mask: out must be row-strided (..., C)")
    out = torch.empty(g.shape, dtype=g.dtype, device=g.device) if out is None else out
    rows = g.numel() // C
    ld = lambda t: t.stride(-2)  # noqa: E731
    _lib.check(_lib.lib().vo_lrelu_mask(_ptr(g), ld(g), vo_dtype(g), _ptr(ref), ld(ref), vo_dtype(ref), rows, C,
                                        float(slope), _ptr(out), ld(out), _stream(g)), "vo_lrelu_mask")
    return out


def colsum(x):
    """(..., C) -> (C,) fp32 column sums (bias gradient)."""
    _contig(x, "x")
    C = x.shape[-1]
    if C % 8:
        x = torch.nn.functional.pad(x, (0, 8 - C % 8)).contiguous()
        return colsum(x)[:C]
    rows = x.numel() // C
    L = _lib.lib()
    out = torch.empty(C, dtype=torch.float32, device=x.device)
    ws = torch.empty(int(L.vo_colsum_workspace_size(rows, C)) // 4, dtype=torch.float32, device=x.device)
    _lib.check(L.vo_colsum(_ptr(x), rows, C, C, vo_dtype(x), _ptr(out), _ptr(ws), _stream(x)), "vo_colsum")
    return out
