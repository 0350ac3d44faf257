"""Autograd ops of the HiFi-GAN training path (config C5).

Every forward is a HIP kernel of libvonoma.so on channels-last (B, T, C) activations:
``vo_conv1d`` (dense, strided, grouped, polyphase-transposed; pre / post activation,
residual, MRF accumulate fused), ``vo_period_fold`` / ``vo_wav_cl8`` / ``vo_avgpool_wav``
(discriminator inputs), ``vo_gan_reduce`` (losses) and ``vo_stft_mel_ex`` (mel loss).

Backward, per op:
  * input gradient of a stride-1 dense conv: the conv kernel over dY with the weights
    re-packed taps-reversed / channels-swapped (as in C4); of a polyphase ConvTranspose1d:
    the strided conv kernel (dX = conv1d(dY, W, stride s, pad p));
  * loss gradients: ``vo_gan_reduce_grad``;
  * weight / bias gradients of dense and grouped convs (generator, MPD, MSD, conv_post):
    ``vo_conv1d_wgrad[_grouped]`` (MFMA over transposed LDS reads) and ``vo_colsum``;
  * input gradient of strided / grouped discriminator convs: the conv kernel once per stride
    phase (taps of the phase reversed, channel roles swapped, rows interleaved) -- ``_dgrad``;
  * the mel-loss STFT backward: ``vo_stft_mel_bwd`` (per frame: the spectrum recomputed, the
    mel / log chain rule, an inverse FFT in LDS; then a deterministic gather over frames and
    reflect mirrors);
  * the discriminator input transforms (period fold, channels-last copy, average pool):
    ``vo_period_fold_bwd`` / ``vo_wav_cl8_bwd`` / ``vo_avgpool_wav_bwd``;
  * MIOpen ``convolution_backward`` only for layouts none of the above covers (none in
    HiFi-GAN V1) -- the fallback SURVEY.md 8(b) sanctions.
"""

from dataclasses import dataclass, replace
from typing import Optional, Tuple

import os
import weakref

import torch
import torch.nn.functional as F

from .. import ops


@dataclass(frozen=True)
class ConvSpec:
    K: int
    pad: int
    dil: int = 1
    stride: int = 1
    groups: int = 1
    pre_slope: Optional[float] = None       # leaky-ReLU applied to the input while staging
    post: Optional[str] = None              # None | "lrelu" | "tanh" (not combined with residuals)
    post_slope: float = 0.1
    out_scale: float = 1.0
    transposed: Optional[Tuple[int, int]] = None  # (stride, pad) of a ConvTranspose1d (K = 2 stride)
    ci_pad: Optional[int] = None            # input channels padded with zeros (1-channel inputs -> 8)
    co_pad: Optional[int] = None            # output channels padded with zero rows (Co = 1 -> 4)

    def plain(self):
        return (self.stride == 1 and self.groups == 1 and self.transposed is None and self.ci_pad is None
                and self.co_pad is None)


_POST = {None: ops.ACT_NONE, "lrelu": ops.ACT_LRELU, "tanh": ops.ACT_TANH}


def _pack(w, spec, dtype, slot=None):
    """``slot(shape, dtype)`` (optional): a persistent zero-initialised buffer that the grouped
    layout is written into in place -- its diagonal blocks only (``ops.pack_grouped_weight(out=)``)."""
    if spec.transposed is not None:
        return ops.pack_conv_weight(w, dtype, transposed_stride=spec.transposed[0])
    if spec.plain():
        return ops.pack_conv_weight(w, dtype)
    if spec.co_pad is not None and spec.co_pad > w.shape[0]:
        w = torch.cat([w.detach(), w.new_zeros((spec.co_pad - w.shape[0],) + tuple(w.shape[1:]))])
    return _pack_grouped(w, dtype, spec.groups, spec.ci_pad, slot)


def _pack_grouped(w, dtype, groups, ci_pad, slot):
    if slot is None:
        return ops.pack_grouped_weight(w, dtype, groups, ci_pad)
    Co, cig, K = w.shape
    return ops.pack_grouped_weight(w, dtype, groups, ci_pad, out=slot((K, Co, cig * groups if ci_pad is None else ci_pad),
                                                                      dtype, w.device))


def _bias(b, spec, n, wkey=None):
    """The bias as an fp32 vector of n (>= its length: padded output channels get 0).  A padded bias
    is cached at the parameter's version (the D step and the G step's two passes run each conv_post
    three times per step: one pad launch pair instead of three; capture-aware like the weight packs)."""
    pad = lambda: F.pad(b.detach().float(), (0, n - b.numel())).contiguous()  # noqa: E731
    if b.numel() >= n:
        return b.detach().float().contiguous()
    if wkey is None:
        return pad()
    # keyed on the conv module (a tensor key would be compared with ==, a device op) and the bias version
    return _cached((wkey[0], b._version), f"bias{n}", pad)


def out_len(spec, T_in):
    if spec.transposed is not None:
        s, p = spec.transposed
        return (T_in - 1) * s - 2 * p + spec.K
    return (T_in + 2 * spec.pad - spec.dil * (spec.K - 1) - 1) // spec.stride + 1


_PACKS = weakref.WeakKeyDictionary()  # module -> {(spec, dtype, kind...): (versions, packed weight)}
# Inside a HIP-graph capture only packs recorded by that capture may be reused (an eager pack
# would be read, never rewritten, by every replay); replays change parameters without bumping
# their version counters, so the eager cache is dropped after each (reset_pack_cache).
_CAPTURE_PACKS = weakref.WeakKeyDictionary()


def reset_pack_cache():
    _PACKS.clear()
    _CAPTURE_PACKS.clear()


# Persistent packed buffers of the grouped (block-diagonal) layouts, per module and pack tag:
# zeroed once, then only their diagonal blocks are rewritten when the weights change (the dense
# repack wrote groups x more bytes, mostly zeros, after every optimizer step).  They outlive the
# version cache above (a HIP graph captures the in-place updates at stable addresses).
_SLOTS = weakref.WeakKeyDictionary()


def _slot_fn(wkey, tag):
    if wkey is None:
        return None

    def get(shape, dtype, device):
        per = _SLOTS.setdefault(wkey[0], {})
        buf = per.get(tag)
        if buf is None or tuple(buf.shape) != tuple(shape) or buf.dtype != dtype or buf.device != device:
            buf = torch.zeros(shape, dtype=dtype, device=device)
            per[tag] = buf
        return buf
    return get


# Version of a spectral-normed conv's weight, which moves with each training-mode power iteration:
# never equal to a cached one, so every use re-packs -- into the module's persistent slots (the
# grouped layouts' diagonal blocks only), not a dense buffer per call.
VOLATILE = object()


def weight_key(m):
    """Cache key of a conv module's effective weight: the module and its parameters' version
    counters (bumped by every optimizer step / load_state_dict); ``(m, VOLATILE)`` (re-packed on
    every use) for spectral-normed convs."""
    if hasattr(m, "weight_g"):
        return (m, m.weight_v._version, m.weight_g._version)
    if hasattr(m, "weight_orig"):
        return (m, VOLATILE)
    return (m, m.weight._version)


def volatile(wkey):
    return wkey is None or wkey[1] is VOLATILE


# pack_builds: packs built on first use at a new parameter version (tests: zero after prepack)
STATS = {"pack_builds": 0}


def _cached(wkey, tag, build):
    if volatile(wkey):
        return build()
    per = (_CAPTURE_PACKS if torch.cuda.is_current_stream_capturing() else _PACKS).setdefault(wkey[0], {})
    hit = per.get(tag)
    if hit is not None and hit[0] == wkey[1:]:
        return hit[1]
    val = build()
    if isinstance(tag, tuple):
        STATS["pack_builds"] += 1
    per[tag] = (wkey[1:], val)
    return val


def _conv_fwd(x, w, b, res1, res2, spec, cdt, wkey=None):
    tag = (spec, cdt, "fwd")
    wp = _cached(wkey, tag, lambda: _pack(w, spec, cdt, _slot_fn(wkey, tag)))
    if spec.transposed is not None:
        s, p = spec.transposed
        cout = w.shape[1]
        return ops.conv1d(x, wp, _bias(b, spec, cout), Co=s * cout, K=2, pad=1,
                          pre_act=ops.ACT_LRELU if spec.pre_slope is not None else ops.ACT_NONE,
                          pre_slope=spec.pre_slope or 0.0, transposed=dict(stride=s, pad=p, cout=cout),
                          res1=res1, res2=res2, out_scale=spec.out_scale, out_dtype=x.dtype, compute_dtype=cdt)
    Co = wp.shape[1]
    return ops.conv1d(x, wp, _bias(b, spec, Co, wkey), Co=Co, K=spec.K, dil=spec.dil, pad=spec.pad,
                      T_out=out_len(spec, x.shape[1]),
                      pre_act=ops.ACT_LRELU if spec.pre_slope is not None else ops.ACT_NONE,
                      pre_slope=spec.pre_slope or 0.0, post_act=_POST[spec.post], post_slope=spec.post_slope,
                      res1=res1, res2=res2, out_scale=spec.out_scale, out_dtype=x.dtype, compute_dtype=cdt,
                      stride=spec.stride, groups=spec.groups)


def _dgrad(gz, w, spec, x, cdt, wkey=None, ymask=None, ymask_slope=0.0):
    """Input gradient of a strided and/or grouped conv (dil 1) on the HIP conv kernel, by phase:
    input row i = S m + r receives taps k = k_r + S j (k_r = (r + pad) mod S) from output rows
    m + c_r - j, so each residue r is a stride-1 grouped conv over dY with those taps reversed and
    the channel roles swapped, written to rows r, r + S, ... of dX (row-strided output view).
    ``ymask`` (x's shape, contiguous): dX stored through the leaky-ReLU mask of it (vo_conv1d ymask)."""
    S, K, pad, g = spec.stride, spec.K, spec.pad, spec.groups
    if spec.dil != 1:
        raise NotImplementedError("strided / grouped input gradient with dilation")
    Co, cig, _ = w.shape
    cog, Ci = Co // g, cig * g
    # dgrad conv weight (Ci, Co / g, K): per group the (cog x cig) blocks transposed
    ci_out = x.shape[-1]  # >= Ci (1-channel inputs padded to 8)
    if ci_out > Ci and g != 1:
        raise NotImplementedError("strided / grouped input gradient: padded input channels with groups")
    gzp = _pad_channels(gz.to(cdt))
    co_in = gzp.shape[-1]  # >= Co (Co = 1 padded to 8); extra channels multiply zero weights
    B, T_in = x.shape[0], x.shape[1]
    out = torch.empty((B, T_in, ci_out), dtype=x.dtype, device=x.device)
    for r in range(S):
        k_r = (r + pad) % S
        taps = list(range(k_r, K, S))
        rows = (T_in - r + S - 1) // S
        if rows <= 0:
            continue
        view = out[:, r::S]
        if not taps:
            view.zero_()
            continue
        mview = ymask[:, r::S] if ymask is not None else None
        J = len(taps)
        c_r = (r + pad - k_r) // S
        tag = (spec, cdt, "dgrad", r, ci_out, co_in)

        def build(k_r=k_r, tag=tag, J=J):
            # tap t <- k_r + S (J - 1 - t), channel roles swapped per group: one packing launch
            slot = _slot_fn(wkey, tag)
            out = None if slot is None else slot((J, ci_out, co_in), cdt, w.device)
            return ops.pack_dgrad_phase(w, g, S, k_r, J, ci_out, co_in, cdt, out=out)
        wp = _cached(wkey, tag, build)
        ops.conv1d(gzp, wp, None, Co=ci_out, K=J, pad=J - 1 - c_r, T_out=rows, out=view, compute_dtype=cdt,
                   groups=g if ci_out == Ci else 1, ymask=mview, ymask_slope=ymask_slope)
    return out


def _pad_channels(t, mult=8):
    """(B, T, C) -> C zero-padded to a multiple of ``mult`` (the wgrad kernel's vector width)."""
    C = t.shape[-1]
    if C % mult:
        t = F.pad(t, (0, mult - C % mult))
    return t.contiguous()


def _ncw(t):
    return t.transpose(1, 2).float().contiguous()


RES_LINK = os.environ.get("VO_RES_LINK", "1") != "0"  # 0: autograd sums the residual gradients (A/B)


class ResLink:
    """Hands a residual's gradient from the conv that adds it (``res1`` of the second conv of a
    HiFi-GAN ResBlock pair) to the conv that read the same tensor as its input (the pair's first
    conv), which adds it in its leaky-ReLU mask pass -- instead of autograd summing the two
    gradients of that tensor with a separate add kernel.  Only for a tensor with exactly those
    two uses."""

    def __init__(self):
        self.armed = False
        self.g = None


class ConvFn(torch.autograd.Function):
    """y = (post(conv(pre(x), w) + b) + res1) * out_scale + res2, channels-last.  ``link``:
    (ResLink, "in" | "res"): this conv's input ("in") / res1 ("res") is the linked tensor.  ``tap``
    (leaky-ReLU post-activation): also return y a second time (same storage) for a second consumer
    (a discriminator feature map): the backward gets the two gradients apart and sums them in its
    mask pass (vo_lrelu_mask_sum) instead of autograd adding them first.  ``in_mask`` (slope): x is
    the leaky-ReLU output of the conv before, whose only gradient is this conv's input gradient:
    that gradient is masked as the input-gradient conv stores it (vo_conv1d ymask); ``out_masked``:
    the conv after does that for this conv's output, so its backward skips its own mask pass."""

    @staticmethod
    def forward(ctx, x, w, b, res1, res2, spec, cdt, wkey=None, link=None, tap=False, in_mask=None, out_masked=False):
        if spec.post is not None and (res1 is not None or res2 is not None):
            raise ValueError("ConvFn: post-activation with residual inputs is not differentiable here")
        y = _conv_fwd(x.contiguous(), w, b, res1, res2, spec, cdt, wkey)
        ctx.spec, ctx.cdt, ctx.wkey = spec, cdt, wkey
        ctx.link = None
        if link is not None:
            lk, role = link
            if role == "in":  # armed when this conv's backward will run and can take the residual
                lk.armed = (x.requires_grad and spec.pre_slope is not None and spec.transposed is None
                            and x.shape[-1] % 8 == 0 and res1 is None and res2 is None)
                ctx.link = (lk, "in") if lk.armed else None
            elif role == "res" and lk.armed and res1 is not None and res1.requires_grad:
                ctx.link = (lk, "res")
        ctx.has = (res1 is not None, res2 is not None)
        ctx.in_mask, ctx.out_masked = in_mask, out_masked and spec.post == "lrelu" and not tap
        ctx.save_for_backward(x, w, y if spec.post is not None else None)
        if tap:
            if spec.post != "lrelu" or res1 is not None or res2 is not None or spec.out_scale != 1.0:
                raise ValueError("ConvFn: tap needs a leaky-ReLU post-activation and no residuals")
            ctx.set_materialize_grads(False)  # an unused output's gradient stays None (no zero fill)
            return y, y.detach()
        return y

    @staticmethod
    def backward(ctx, gy, *tap_g):
        x, w, y = ctx.saved_tensors
        spec, cdt = ctx.spec, ctx.cdt
        gf = tap_g[0] if tap_g else None
        if gy is None:
            gy, gf = gf, None
        if gy is None:
            return (None,) * 12
        gy = gy.contiguous()
        g_res2 = gy if ctx.has[1] and ctx.needs_input_grad[4] else None
        gz = gy * spec.out_scale if spec.out_scale != 1.0 else gy
        g_res1 = gz if ctx.has[0] and ctx.needs_input_grad[3] else None
        lk, role = ctx.link if ctx.link is not None else (None, None)
        if role == "res" and g_res1 is not None:  # the residual's gradient goes to the linked input conv
            lk.g, g_res1 = g_res1, None
        if spec.post == "lrelu" and ctx.out_masked:
            pass  # gy arrives masked (the next conv's input-gradient epilogue)
        elif spec.post == "lrelu":
            ok = gf is not None and gf.dtype == gz.dtype and gf.shape == gz.shape and gz.shape[-1] % 8 == 0
            if gf is not None and not ok:
                gz, gf = gz + gf, None
            gz = ops.lrelu_mask(gz, y, spec.post_slope, summand=gf)
        elif spec.post == "tanh":
            yf = y.float()
            gz = (gz.float() * (1.0 - yf * yf)).to(gz.dtype)
        if spec.co_pad is not None and (gz.shape[-1] % 8 or spec.groups != 1 or spec.transposed is not None):
            # (a dY of whole 8-channel vectors goes on as it is: the padded rows' input-gradient weights
            # are zero and their weight / bias gradient rows are dropped below)
            gz = gz[..., : w.shape[0]].contiguous()
        ci = w.shape[0] if spec.transposed is not None else w.shape[1] * spec.groups
        xin = x[..., :ci] if x.shape[-1] != ci else x
        gx = gw = gb = None
        need_x, need_w, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        ga = None
        im = ctx.in_mask
        ga_masked = False
        if need_x and spec.plain():
            # cached per parameter version: a discriminator's next D step runs its backward at the
            # versions its G step's backward already packed
            wd = _cached(ctx.wkey, (spec, cdt, "dgrad_plain"), lambda: ops.pack_dgrad_weight(w, cdt))
            ym = x if (im is not None and x.dtype == torch.bfloat16 and x.is_contiguous()) else None
            ga = ops.conv1d(gz.to(cdt), wd, None, Co=w.shape[1], K=spec.K, dil=spec.dil,
                            pad=(spec.K - 1) * spec.dil - spec.pad, T_out=x.shape[1], out_dtype=x.dtype,
                            compute_dtype=cdt, ymask=ym, ymask_slope=im or 0.0)
            ga_masked = ym is not None
            need_x = False
        elif need_x and spec.transposed is None and spec.dil == 1:
            ym = x if (im is not None and x.dtype == torch.bfloat16 and x.is_contiguous()) else None
            ga = _dgrad(gz, w, spec, x, cdt, ctx.wkey, ymask=ym, ymask_slope=im or 0.0)
            ga_masked = ym is not None
            if ga.shape[-1] != ci:
                ga = ga[..., :ci]
            need_x = False
        elif need_x and spec.transposed is not None:
            s, p = spec.transposed
            # ConvTranspose1d(Ci -> Co, k, s, p) adjoint = Conv1d(Co -> Ci, W as (Ci, Co, k), stride s, pad p)
            wc = _cached(ctx.wkey, (spec, cdt, "dgrad_convt"), lambda: ops.pack_conv_weight(w, cdt))
            ga = ops.conv1d(gz.to(cdt), wc, None, Co=w.shape[0], K=spec.K, pad=p, stride=s, T_out=x.shape[1],
                            out_dtype=x.dtype, compute_dtype=cdt)
            need_x = False
        g = spec.groups
        grouped_ok = g == 1 or (spec.transposed is None and x.shape[-1] == ci and (ci // g) % 8 == 0
                                and (w.shape[0] // g) % 8 == 0)
        if (need_w or need_b) and grouped_ok:
            # weight / bias gradient on MFMA (vo_conv1d_wgrad[_grouped], vo_colsum)
            gzc = _pad_channels(gz.to(x.dtype))
            if need_w:
                if spec.transposed is not None:
                    s, p = spec.transposed
                    dw = ops.conv1d_wgrad(_pad_channels(x), gzc, spec.K, S=s, pad=p, pre_a=spec.pre_slope,
                                          transposed=True)
                    gw = dw[: w.shape[0], : w.shape[1]].to(w.dtype)
                else:
                    # bias gradient from the same launch when dY needed no cast (column sums of gzc)
                    fuse_b = need_b and gz.dtype == x.dtype
                    dw = ops.conv1d_wgrad(gzc, _pad_channels(x) if g == 1 else x, spec.K, S=spec.stride,
                                          dil=spec.dil, pad=spec.pad, pre_b=spec.pre_slope, groups=g,
                                          with_bias=fuse_b)
                    if fuse_b:
                        dw, db = dw
                        gb = db[: w.shape[0]]
                    gw = dw[: w.shape[0], : w.shape[1]].to(w.dtype)
            if need_b and gb is None:
                gb = ops.colsum(gz.contiguous())[: w.shape[1] if spec.transposed is not None else w.shape[0]]
            need_w = need_b = False
        if need_x or need_w or need_b:
            a = xin if spec.pre_slope is None else torch.where(xin > 0, xin, xin * spec.pre_slope)
            if spec.transposed is not None:
                s, p = spec.transposed
                stride, pad, tr = [s], [p], True
            else:
                stride, pad, tr = [spec.stride], [spec.pad], False
            gi, gw2, gb2 = torch.ops.aten.convolution_backward(
                _ncw(gz), _ncw(a), w.float(), [w.shape[1] if tr else w.shape[0]], stride, pad, [spec.dil], tr, [0],
                spec.groups, [need_x, need_w, need_b])
            if need_x:
                ga = gi.transpose(1, 2).to(x.dtype)
            if need_w:
                gw = gw2.to(w.dtype)
            if need_b:
                gb = gb2
        if ga is not None and im is not None and not ga_masked:
            ga = ops.lrelu_mask(ga, xin, im)
        if ga is not None:
            add = None
            if role == "in" and lk.g is not None:  # this conv reads the linked tensor: its residual gradient joins here
                add, lk.g = lk.g, None
            if add is not None and add.dtype == ga.dtype and ga.shape == add.shape:
                ga = ops.lrelu_mask(ga, xin, spec.pre_slope, out=ga if ga.is_contiguous() else None, add=add)
            elif add is not None:
                raise RuntimeError("ConvFn: linked residual gradient does not match the input gradient")
            elif spec.pre_slope is not None:
                ga = ops.lrelu_mask(ga, xin, spec.pre_slope, out=ga if ga.is_contiguous() else None)
            if ga.shape[-1] != x.shape[-1]:
                ga = F.pad(ga, (0, x.shape[-1] - ga.shape[-1]))
            gx = ga
        if not ctx.needs_input_grad[1]:
            gw = None
        if not ctx.needs_input_grad[2]:
            gb = None
        return gx, gw, gb, g_res1, g_res2, None, None, None, None, None, None, None


# Many short sequences (the MPD's period columns: 96-352 sequences of 10-51 rows at C5): the conv
# kernel tiles every sequence on its own -- a 16- to 256-row tile for 10-51 rows, each tile streaming
# the whole (1024 x 1024 x 5) weight -- so these layers ran at 0.27 PF/s and below.  Laid end to end
# with their zero padding between them they are ONE sequence that the kernel tiles densely; the
# outputs that straddle two sequences are computed and dropped (their gradient is zero, so the
# input and weight gradients over the joined sequence are the per-sequence ones).
FLAT_T = int(os.environ.get("VO_FLAT_T", "64"))  # join sequences of up to this many output rows (0: off)


class JoinSeqFn(torch.autograd.Function):
    """(N, T, C) -> (1, N S_in, C): each sequence at offset ``pad`` of its S_in rows, zeros around it
    (vo_seq_remap; the adjoint gathers the rows back)."""

    @staticmethod
    def forward(ctx, x, pad, S_in):
        N, T, C = x.shape
        ctx.dims = (N, T, pad, S_in)
        return ops.seq_remap(x.contiguous(), N * S_in, S_in, T, pad, pad + T, -pad).view(1, N * S_in, C)

    @staticmethod
    def backward(ctx, g):
        N, T, pad, S_in = ctx.dims
        C = g.shape[-1]
        return ops.seq_remap(g.contiguous(), N * T, T, S_in, 0, T, pad).view(N, T, C), None, None


class SplitSeqFn(torch.autograd.Function):
    """(1, R, C) joined conv output -> (N, T_out, C): rows n S_out + t, t < T_out (the slots of
    outputs that straddle two sequences are dropped; their gradient is zero)."""

    @staticmethod
    def forward(ctx, yj, N, S_out, T_out):
        R, C = yj.shape[1], yj.shape[2]
        ctx.dims = (R, S_out, T_out)
        return ops.seq_remap(yj.contiguous(), N * T_out, T_out, S_out, 0, T_out, 0).view(N, T_out, C)

    @staticmethod
    def backward(ctx, g):
        R, S_out, T_out = ctx.dims
        C = g.shape[-1]
        return ops.seq_remap(g.contiguous(), R, S_out, T_out, 0, T_out, 0).view(1, R, C), None, None, None


REJOIN = os.environ.get("VO_REJOIN", "1") != "0"  # 0: split + join between consecutive joined convs (A/B)


class RejoinFn(torch.autograd.Function):
    """One joined conv feeding the next: (1, R, C) joined output -> ((N, T, C) its split output, (1,
    N S_in, C) the next conv's joined input, each sequence at offset ``pad`` of its S_in rows) in one
    vo_seq_remap2 launch; the backward gathers both gradients and adds them in the same launch (the
    split and join adjoints plus autograd's add of the two, bit for bit)."""

    @staticmethod
    def forward(ctx, yj, N, S_out, T, pad, S_in):
        C = yj.shape[-1]
        ctx.dims = (yj.shape[1], N, S_out, T, pad, S_in)
        # an output that carries no gradient (the D step's detached feature maps) arrives as None, and
        # the backward then gathers the other one alone instead of adding a zero-filled tensor
        ctx.set_materialize_grads(False)
        y, xj = ops.seq_remap2([dict(src=yj, dst_rows=N * T, Td=T, Ss=S_out, lo=0, hi=T, shift=0),
                                dict(src=yj, dst_rows=N * S_in, Td=S_in, Ss=S_out, lo=pad, hi=pad + T, shift=-pad)])
        return y.view(N, T, C), xj.view(1, N * S_in, C)

    @staticmethod
    def backward(ctx, gy, gxj):
        R, N, S_out, T, pad, S_in = ctx.dims
        job = dict(dst_rows=R, Td=S_out, lo=0, hi=T)
        if gy is not None:
            job.update(src=gy.contiguous(), Ss=T, shift=0)
            if gxj is not None:
                job.update(src2=gxj.contiguous(), Ss2=S_in, shift2=pad)
        elif gxj is not None:
            job.update(src=gxj.contiguous(), Ss=S_in, shift=pad)
        else:
            return None, None, None, None, None, None
        (g,) = ops.seq_remap2([job])
        return g.view(1, R, g.shape[-1]), None, None, None, None, None


def _join_plan(spec, T):
    """(T_out, S_out, S_in) of a joined conv over sequences of T rows: output slots and input rows
    per sequence (its padding, then zeros)."""
    S_out = -(-(T + 2 * spec.pad) // spec.stride)
    return out_len(spec, T), S_out, spec.stride * S_out


def _join_input(x, spec):
    N, T, C = x.shape
    _, _, S_in = _join_plan(spec, T)
    if (C * x.element_size()) % 4:  # vo_seq_remap moves whole 4-byte words
        return F.pad(x, (0, 0, spec.pad, S_in - T - spec.pad)).reshape(1, N * S_in, C)
    return JoinSeqFn.apply(x, spec.pad, S_in)


def _split_output(yj, N, S_out, T_out):
    if (yj.shape[-1] * yj.element_size()) % 4:
        return F.pad(yj, (0, 0, 0, N * S_out - yj.shape[1])).reshape(N, S_out, -1)[:, :T_out].contiguous()
    return SplitSeqFn.apply(yj, N, S_out, T_out)


def _conv_joined(x, w, b, spec, cdt, wkey):
    T_out, S_out, _ = _join_plan(spec, x.shape[1])
    xj = _join_input(x, spec)
    yj = ConvFn.apply(xj, w, b, None, None, replace(spec, pad=0), cdt, wkey)  # slot u S_out + t <- rows u S_in + st t + k
    return _split_output(yj, x.shape[0], S_out, T_out)


def conv_layers(x, convs, fmaps=True):
    """The outputs of ``convs`` [(w, b, spec, cdt, wkey)] applied in order, as ``conv`` per layer;
    where one joined conv feeds the next, RejoinFn hands its joined output over (one remap launch
    each way instead of a split and a join).  ``fmaps`` False (the D step: only the last output
    carries a gradient, the others are returned detached): each leaky-ReLU output's mask is applied
    by the next conv's input-gradient epilogue (ConvFn in_mask / out_masked), not by a mask pass."""
    n = len(convs)
    fold = [not fmaps and i + 1 < n and convs[i][2].post == "lrelu" for i in range(n)]
    outs, pend = [], None  # pend: (yj, N, S_out, T_out) of a joined conv whose output is not split yet
    for i, (w, b, spec, cdt, wkey) in enumerate(convs):
        fl = dict(in_mask=convs[i - 1][2].post_slope if i and fold[i - 1] else None, out_masked=fold[i])
        if pend is not None:
            yj, N, S_out, T = pend
            pend = None
            C = yj.shape[-1]
            if REJOIN and _joined((N, T, C), spec) and (C * yj.element_size()) % 16 == 0:
                T_out2, S_out2, S_in2 = _join_plan(spec, T)
                y, xj = RejoinFn.apply(yj, N, S_out, T, spec.pad, S_in2)
                outs.append(y)
                pend = (ConvFn.apply(xj, w, b, None, None, replace(spec, pad=0), cdt, wkey, None, False, fl["in_mask"],
                                     fl["out_masked"]), N, S_out2, T_out2)
                continue
            x = _split_output(yj, N, S_out, T)
            outs.append(x)
        if _joined(x.shape, spec):
            T_out, S_out, _ = _join_plan(spec, x.shape[1])
            yj = ConvFn.apply(_join_input(x, spec), w, b, None, None, replace(spec, pad=0), cdt, wkey, None, False,
                              fl["in_mask"], fl["out_masked"])
            pend = (yj, x.shape[0], S_out, T_out)
        elif spec.post == "lrelu" and fmaps:  # the feature map and the next conv's input: their gradients meet in the mask pass
            x, f = ConvFn.apply(x, w, b, None, None, spec, cdt, wkey, None, True)
            outs.append(f)
        else:
            x = ConvFn.apply(x, w, b, None, None, spec, cdt, wkey, None, False, fl["in_mask"], fl["out_masked"])
            outs.append(x)
    if pend is not None:
        outs.append(_split_output(pend[0], pend[1], pend[2], pend[3]))
    if not fmaps:
        outs = [o.detach() for o in outs[:-1]] + outs[-1:]
    return outs


def _joined(shape, spec, has_res=False):
    """Whether ``conv`` runs an input of this (N, T, C) shape as one joined sequence."""
    return (FLAT_T > 0 and not has_res and spec.groups == 1 and spec.dil == 1 and spec.transposed is None
            and len(shape) == 3 and shape[0] >= 8 and out_len(spec, shape[1]) <= FLAT_T)


def conv(x, w, b, spec, cdt, res1=None, res2=None, wkey=None, link=None):
    """``wkey`` (``weight_key(module)``): reuse the packed weights while the parameters are unchanged.
    ``link``: (ResLink, role) -- see ResLink."""
    if _joined(x.shape, spec, res1 is not None or res2 is not None):
        if link is not None:
            raise ValueError("conv: a linked conv cannot run joined")
        return _conv_joined(x, w, b, spec, cdt, wkey)
    return ConvFn.apply(x, w, b, res1, res2, spec, cdt, wkey, link)


def conv_spec(shape, spec, has_res=False):
    """The spec ``conv`` hands to ConvFn for an input of this shape (joined sequences run unpadded)."""
    return replace(spec, pad=0) if _joined(shape, spec, has_res) else spec


# ----------------------------------------------------------------------------- batched packing
# After every optimizer step each conv's packed weights (forward, and the input-gradient layouts
# its backward uses) are stale: ~270 pack launches of 4-27 us per C5 step when each conv packs on
# first use.  ``prepack`` writes all of a model's packs in one vo_pack_batch launch right after its
# batched weight normalisation and records them under the same cache tags and persistent slots
# that _conv_fwd / ConvFn.backward / _dgrad look up, so those find them (a conv whose tag the plan
# missed still packs itself: the plan changes speed, never results).

def _pack_plan(w_shape, spec, cdt, ci_out, dgrad):
    """[(tag, dst shape, vo_pack_batch job fields)] of the packs one conv's forward (and with
    ``dgrad``, its backward's input gradient) looks up -- the tags and layouts of _conv_fwd /
    ConvFn.backward / _dgrad.  ``spec`` as ConvFn sees it (``conv_spec``), ci_out = its input's
    channel count."""
    G, CT = ops.PJ_GATHER, ops.PJ_CONVT

    def job(mode, swap, T, rows, width, dst_rows, ld, rpg, cpg, cig, K, tap0, tstep, src_rows):
        return dict(mode=mode, swap=swap, T=T, rows=rows, width=width, dst_rows=dst_rows, ld=ld, rpg=rpg, cpg=cpg,
                    cig=cig, K=K, tap0=tap0, tstep=tstep, src_rows=src_rows)
    out = []
    if spec.transposed is not None:
        Ci, Co, K = w_shape  # ConvTranspose1d (Ci, Co, 2s)
        s = spec.transposed[0]
        out.append(((spec, cdt, "fwd"), (2, s * Co, Ci), job(CT, 0, 2, s * Co, Ci, s * Co, Ci, s * Co, 0, Co, K, s, 0, Ci)))
        if dgrad:  # the adjoint conv's weight: w read as a (Ci, Co, K) Conv1d weight
            out.append(((spec, cdt, "dgrad_convt"), (K, Ci, Co), job(G, 0, K, Ci, Co, Ci, Co, Ci, 0, Co, K, 0, 1, Ci)))
        return out
    Co, cig, K = w_shape
    g = spec.groups
    Ci, cog = cig * g, Co // g
    if spec.plain():
        out.append(((spec, cdt, "fwd"), (K, Co, Ci), job(G, 0, K, Co, Ci, Co, Ci, Co, 0, Ci, K, 0, 1, Co)))
        if dgrad:
            out.append(((spec, cdt, "dgrad_plain"), (K, Ci, Co), job(G, 1, K, Ci, Co, Ci, Co, Ci, 0, Ci, K, K - 1, -1, Co)))
        return out
    co_rows = spec.co_pad if spec.co_pad is not None and spec.co_pad > Co else Co
    ld = Ci if spec.ci_pad is None else spec.ci_pad
    out.append(((spec, cdt, "fwd"), (K, co_rows, ld), job(G, 0, K, Co, cig, co_rows, ld, cog, cig, cig, K, 0, 1, Co)))
    if dgrad and spec.dil == 1 and not (ci_out > Ci and g != 1):
        S, co_in = spec.stride, -(-Co // 8) * 8
        for r in range(S):
            k_r = (r + spec.pad) % S
            J = len(range(k_r, K, S))
            if J == 0:
                continue
            out.append(((spec, cdt, "dgrad", r, ci_out, co_in), (J, ci_out, co_in),
                        job(G, 1, J, Ci, cog, ci_out, co_in, cig, cog, cig, K, k_r + S * (J - 1), -S, Co)))
    return out


PREPACK = os.environ.get("VO_PREPACK", "1") != "0"  # 0: every conv packs on first use (A/B)


def prepack(entries, cdt):
    """entries: [(wkey, w, spec, input shape (N, T, C), dgrad[, has residual inputs])] -- ``spec`` /
    shape as passed to ``conv`` -> every pack those convs will look up that is not cached at these
    parameter versions, in one vo_pack_batch launch (entries with a volatile key pack on use)."""
    if not PREPACK:
        return 0
    store = _CAPTURE_PACKS if torch.cuda.is_current_stream_capturing() else _PACKS
    jobs, done = [], []
    for wkey, w, spec, shape, dgrad, *res in entries:
        if volatile(wkey):
            continue
        per = store.setdefault(wkey[0], {})
        src = None
        for tag, dshape, f in _pack_plan(tuple(w.shape), conv_spec(shape, spec, bool(res and res[0])), cdt, shape[-1],
                                         dgrad):
            hit = per.get(tag)
            if hit is not None and hit[0] == wkey[1:]:
                continue
            if src is None:
                src = w.detach().float().contiguous()
            dst = _slot_fn(wkey, tag)(dshape, cdt, w.device)
            jobs.append((src, dst, f))
            done.append((per, tag, wkey[1:], dst))
    ops.pack_batch(jobs, cdt)
    for per, tag, ver, dst in done:
        per[tag] = (ver, dst)
    return len(jobs)


class WeightNormFn(torch.autograd.Function):
    """w_k = g_k v_k / ||v_k|| (torch._weight_norm(v, g, 0)) for n layers in one launch per 24 layers,
    forward and backward (vo_weight_norm / vo_weight_norm_bwd): the per-layer PyTorch kernels were
    ~270 launches per C5 step.  apply(n, v_1..v_n, g_1..g_n) -> (w_1..w_n)."""

    @staticmethod
    def forward(ctx, n, *vg):
        vs, gs = [t.detach() for t in vg[:n]], [t.detach() for t in vg[n:]]
        ctx.n = n
        ctx.save_for_backward(*vg)
        return tuple(ops.weight_norm(vs, gs))

    @staticmethod
    def backward(ctx, *dws):
        n = ctx.n
        saved = ctx.saved_tensors
        vs, gs = [t.detach() for t in saved[:n]], [t.detach() for t in saved[n:]]
        dws = [torch.zeros_like(v) if d is None else d.float().contiguous() for d, v in zip(dws, vs)]
        dvs, dgs = ops.weight_norm_bwd(vs, gs, dws)
        return (None, *dvs, *dgs)


class SpectralNormFn(torch.autograd.Function):
    """w_k = W_k / sigma_k, sigma_k = u_k . W_k v_k (u, v after the power iteration, held constant:
    torch.nn.utils.spectral_norm's autograd) for n layers in one vo_spectral_norm call.
    apply(us, vs, power, eps, W_1..W_n) -> (w_1..w_n); the u / v buffers are updated in place."""

    @staticmethod
    def forward(ctx, us, vs, power, eps, *Ws):
        ws, uo, vo, sig = ops.spectral_norm([W.detach() for W in Ws], us, vs, power, eps)
        ctx.n = len(Ws)
        ctx.save_for_backward(*Ws, *uo, *vo, *sig)
        return tuple(ws)

    @staticmethod
    def backward(ctx, *gws):
        n, sv = ctx.n, ctx.saved_tensors
        # gW = g / sigma - (sum(g W) / sigma^2) u v^T (dL/dsigma = -d / sigma^2; dsigma/dW = u v^T), every
        # layer with a gradient in one vo_spectral_norm_bwd call
        idx = [i for i in range(n) if gws[i] is not None]
        out = [None] * n
        if idx:
            Ws = [sv[i].detach() for i in idx]
            res = ops.spectral_norm_bwd([gws[i] for i in idx], Ws, [sv[n + i] for i in idx],
                                        [sv[2 * n + i] for i in idx], [sv[3 * n + i] for i in idx])
            for i, r in zip(idx, res):
                out[i] = r
        return (None, None, None, None, *out)


def spectral_norm_all(mods):
    """{module: weight} of spectral-normed convs (``weight_orig`` / ``weight_u`` / ``weight_v``, torch's
    hook: dim 0, one power iteration while the module trains), batched in one vo_spectral_norm call;
    differentiable through SpectralNormFn while autograd records.  Modules whose hook differs
    (other dim / iteration count) are left out (their hook runs per use)."""
    from torch.nn.utils.spectral_norm import SpectralNorm
    sel = []
    for m in mods:
        hook = next((h for h in m._forward_pre_hooks.values() if isinstance(h, SpectralNorm)), None)
        if hook is not None and hook.name == "weight" and hook.dim == 0 and hook.n_power_iterations == 1:
            sel.append((m, hook))
    if not sel:
        return {}
    out = {}
    for power in (True, False):
        grp = [(m, h) for m, h in sel if bool(m.training) == power]
        for eps in sorted({h.eps for _, h in grp}):
            ms = [m for m, h in grp if h.eps == eps]
            Ws = [m.weight_orig for m in ms]
            us, vs = [m.weight_u for m in ms], [m.weight_v for m in ms]
            if torch.is_grad_enabled() and any(W.requires_grad for W in Ws):
                ws = SpectralNormFn.apply(us, vs, power, eps, *Ws)
            else:
                ws = ops.spectral_norm([W.detach() for W in Ws], us, vs, power, eps)[0]
            out.update(zip(ms, ws))
    return out


# VO_BATCHED_WN=0: per-layer torch._weight_norm instead (A/B)
BATCHED_WN = os.environ.get("VO_BATCHED_WN", "1") != "0"
BATCHED_SN = os.environ.get("VO_BATCHED_SN", "1") != "0"  # 0: torch's spectral-norm hook per conv (A/B)


def weight_norm_all(mods):
    """{module: effective weight} of weight-normed convs (``weight_v`` / ``weight_g``), batched:
    differentiable through WeightNormFn while autograd records, a plain vo_weight_norm otherwise."""
    mods = [m for m in mods if hasattr(m, "weight_g")]
    if not mods:
        return {}
    if not BATCHED_WN:
        return {m: torch._weight_norm(m.weight_v, m.weight_g, 0) for m in mods}
    vs, gs = [m.weight_v for m in mods], [m.weight_g for m in mods]
    if torch.is_grad_enabled() and any(p.requires_grad for p in vs + gs):
        ws = WeightNormFn.apply(len(mods), *vs, *gs)
    else:
        ws = ops.weight_norm([v.detach() for v in vs], [g.detach() for g in gs])
    return dict(zip(mods, ws))


class PeriodFoldFn(torch.autograd.Function):
    """wav (B, T) fp32 -> (B * p, ceil(T / p), 8): reflect pad to a multiple of p, (T/p, p) view."""

    @staticmethod
    def forward(ctx, wav, period, dtype):
        ctx.shape, ctx.period = wav.shape, period
        return ops.period_fold(wav.contiguous(), period, dtype)

    @staticmethod
    def backward(ctx, g):
        B, T = ctx.shape
        return ops.period_fold_bwd(g.contiguous(), B, T, ctx.period), None, None


class WavCl8Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wav, dtype):
        return ops.wav_cl8(wav.contiguous(), dtype)

    @staticmethod
    def backward(ctx, g):
        return ops.wav_cl8_bwd(g.contiguous()), None


class AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, wav):
        ctx.T = wav.shape[1]
        return ops.avgpool_wav(wav.contiguous())

    @staticmethod
    def backward(ctx, g):
        return ops.avgpool_wav_bwd(g.float().contiguous(), ctx.T)


class GanLossFn(torch.autograd.Function):
    """scale * sum over a of |a - b| / (1 - a)^2 / a^2 (b held constant)."""

    @staticmethod
    def forward(ctx, a, b, kind, scale):
        s = ops.gan_reduce(kind, a, b)
        ctx.kind, ctx.scale = kind, scale
        ctx.save_for_backward(a, b)
        return s * scale

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = ops.gan_reduce_grad(ctx.kind, a, b, (g.float() * ctx.scale).reshape(()))
        return ga, None, None, None


# every term of a GanLossTermsFn / GanSplitTermsFn in one reduction launch pair and one gradient launch
# (vo_gan_reduce_multi / _grad_multi, bit-identical to the per-term launches); 0: per term (A/B)
GAN_MULTI = os.environ.get("VO_GAN_MULTI", "1") != "0"


def _one_dtype(ts):
    return all(t.dtype == ts[0].dtype for t in ts)


class GanLossTermsFn(torch.autograd.Function):
    """Many GAN / feature-matching terms scale_i * reduce_i(a_i, b_i) as one (n,) vector: the
    reductions accumulate into one zeroed vector and are scaled by one multiply (the per-term path
    was a zero fill, the reduction, a scalar multiply and an add per term -- 54 feature-matching
    terms per G step), and the backward runs one gradient launch per term off one scaled vector."""

    @staticmethod
    def forward(ctx, kinds, sv, *ab):
        n = len(kinds)
        a, b = ab[:n], ab[n:]
        ctx.kinds = kinds
        ctx.save_for_backward(sv, *a, *b)
        if GAN_MULTI and _one_dtype(a):
            return ops.gan_reduce_multi(kinds, a, b, sv)
        out = torch.zeros(n, dtype=torch.float32, device=a[0].device)
        for i in range(n):
            ops.gan_reduce(kinds[i], a[i], b[i], out=out[i])
        return out * sv

    @staticmethod
    def backward(ctx, g):
        sv, *ab = ctx.saved_tensors
        n = len(ctx.kinds)
        gs = g.float() * sv
        # (all terms: the scale vector as it is -- indexing it by a host list would copy from the host
        # inside graph capture)
        if GAN_MULTI and all(ctx.needs_input_grad[2:2 + n]) and _one_dtype(ab[:n]):
            gas = ops.gan_reduce_grad_multi(list(ctx.kinds), list(ab[:n]), list(ab[n:]), gs)
        else:
            gas = [ops.gan_reduce_grad(ctx.kinds[i], ab[i], ab[n + i], gs[i]) if ctx.needs_input_grad[2 + i] else None
                   for i in range(n)]
        return (None, None, *gas, *([None] * n))


_SCALES = {}  # (scales, device) -> fp32 vector (made outside graph capture, reused inside)


class GanSplitTermsFn(torch.autograd.Function):
    """The discriminator loss over score tensors that hold the real batch in their first half and
    the generated batch in their second (the D step runs both as one batch): terms
    scale * reduce(kind_first, S[:h]) for every S, then scale * reduce(kind_second, S[h:]).  Taking
    the whole S keeps the halves' slice views out of the autograd graph: their backward was a zero
    fill and a copy per half plus an add per tensor (16 + 16 + 8 launches per C5 step); here one
    gradient tensor per S is written half by half."""

    @staticmethod
    def forward(ctx, kinds, sv, *bases):
        n = len(bases)
        ctx.kinds = kinds
        ctx.save_for_backward(sv, *bases)
        if GAN_MULTI and _one_dtype(bases):
            halves = [s[: s.shape[0] // 2] for s in bases] + [s[s.shape[0] // 2:] for s in bases]
            return ops.gan_reduce_multi([kinds[0]] * n + [kinds[1]] * n, halves, [None] * (2 * n), sv)
        out = torch.zeros(2 * n, dtype=torch.float32, device=bases[0].device)
        for i, s in enumerate(bases):
            h = s.shape[0] // 2
            ops.gan_reduce(kinds[0], s[:h], None, out=out[i])
            ops.gan_reduce(kinds[1], s[h:], None, out=out[n + i])
        return out * sv

    @staticmethod
    def backward(ctx, g):
        sv, *bases = ctx.saved_tensors
        n = len(bases)
        gs = g.float() * sv
        if GAN_MULTI and all(ctx.needs_input_grad[2:2 + n]) and _one_dtype(bases):
            grads = [torch.empty_like(s, memory_format=torch.contiguous_format) for s in bases]
            hs = [s.shape[0] // 2 for s in bases]
            As = [s[:h] for s, h in zip(bases, hs)] + [s[h:] for s, h in zip(bases, hs)]
            outs = [g_[:h] for g_, h in zip(grads, hs)] + [g_[h:] for g_, h in zip(grads, hs)]
            ops.gan_reduce_grad_multi([ctx.kinds[0]] * n + [ctx.kinds[1]] * n, As, [None] * (2 * n), gs, outs=outs)
            return (None, None, *grads)
        grads = []
        for i, s in enumerate(bases):
            if not ctx.needs_input_grad[2 + i]:
                grads.append(None)
                continue
            h = s.shape[0] // 2
            gsb = torch.empty_like(s, memory_format=torch.contiguous_format)
            ops.gan_reduce_grad(ctx.kinds[0], s[:h], None, gs[i], out=gsb[:h])
            ops.gan_reduce_grad(ctx.kinds[1], s[h:], None, gs[n + i], out=gsb[h:])
            grads.append(gsb)
        return (None, None, *grads)


def _halves_of(a, b):
    """The tensor whose first / second half along dim 0 are the views a / b, else None."""
    base = a._base
    if base is None or b._base is not base or not base.is_contiguous() or base.shape[0] % 2:
        return None
    h = base.shape[0] // 2
    if a.shape[0] != h or b.shape[0] != h or a.data_ptr() != base.data_ptr() or \
            b.data_ptr() != base[h:].data_ptr() or not (a.is_contiguous() and b.is_contiguous()):
        return None
    return base


def gan_split_terms(firsts, seconds, kind_first, kind_second):
    """gan_loss_terms([(f, None, kind_first, 1 / f.numel())] + [(s, None, kind_second, 1 / s.numel())])
    -- through GanSplitTermsFn when every (f, s) pair is the two halves of one tensor."""
    bases = [_halves_of(f, s) for f, s in zip(firsts, seconds)]
    items = ([(f, None, kind_first, 1.0 / f.numel()) for f in firsts]
             + [(s, None, kind_second, 1.0 / s.numel()) for s in seconds])
    if any(bs is None for bs in bases):
        return gan_loss_terms(items)
    dev = firsts[0].device
    key = (tuple(float(it[3]) for it in items), dev)
    sv = _SCALES.get(key)
    if sv is None:
        if torch.cuda.is_current_stream_capturing():
            return gan_loss_terms(items)
        sv = _SCALES[key] = torch.tensor(key[0], dtype=torch.float32, device=dev)
    return GanSplitTermsFn.apply((kind_first, kind_second), sv, *bases)


def gan_loss_terms(items):
    """items: [(a, b or None, kind, scale)] -> (n,) fp32 tensor of scale * reduce(a, b) (b held
    constant), differentiable in each a."""
    dev = items[0][0].device
    key = (tuple(float(it[3]) for it in items), dev)
    sv = _SCALES.get(key)
    if sv is None:
        if torch.cuda.is_current_stream_capturing():  # no host -> device copy inside a capture
            return torch.stack([GanLossFn.apply(a, None if b is None else b.detach(), k, sc) for a, b, k, sc in items])
        sv = _SCALES[key] = torch.tensor(key[0], dtype=torch.float32, device=dev)
    return GanLossTermsFn.apply(tuple(it[2] for it in items), sv, *[it[0] for it in items],
                                *[None if it[1] is None else it[1].detach() for it in items])


def l1_mean(a, b):
    return GanLossFn.apply(a, b.detach(), ops.GAN_L1, 1.0 / a.numel())


def one_minus_sq_mean(a):
    return GanLossFn.apply(a, None, ops.GAN_ONE_MINUS_SQ, 1.0 / a.numel())


def sq_mean(a):
    return GanLossFn.apply(a, None, ops.GAN_SQ, 1.0 / a.numel())


class MelFn(torch.autograd.Function):
    """HiFi-GAN training log-mel of wav (B, N) (meldataset.mel_spectrogram semantics: reflect pad
    (n_fft - hop) / 2, center=False, periodic Hann, sqrt(|X|^2 + 1e-9), slaney mel, log clamp 1e-5)."""

    @staticmethod
    def forward(ctx, wav, window, fb, n_fft, hop):
        ctx.save_for_backward(wav, window, fb)
        ctx.cfg = (n_fft, hop)
        return ops.stft_mel_ex(wav.contiguous(), window, fb, n_fft=n_fft, hop=hop, n_mels=fb.shape[1],
                               pad=(n_fft - hop) // 2, mag_eps=1e-9, clip=False)

    @staticmethod
    def backward(ctx, g):
        wav, window, fb = ctx.saved_tensors
        n_fft, hop = ctx.cfg
        return (ops.stft_mel_bwd(wav.contiguous(), window, fb, g.float().contiguous(), n_fft=n_fft, hop=hop,
                                 pad=(n_fft - hop) // 2, mag_eps=1e-9), None, None, None, None)


class StftMagFn(torch.autograd.Function):
    """|STFT| (center, reflect, onesided; sqrt(max(|X|^2, eps))) of wav (B, N) -> (B, F, bins)."""

    @staticmethod
    def forward(ctx, wav, window, n_fft, hop):
        wav = wav.contiguous()
        ctx.save_for_backward(wav, window)
        ctx.cfg = (n_fft, hop)
        return ops.stft_mag(wav, window, n_fft, hop)

    @staticmethod
    def backward(ctx, g):
        wav, window = ctx.saved_tensors
        n_fft, hop = ctx.cfg
        return ops.stft_mag_bwd(wav, window, g.float().contiguous(), n_fft, hop), None, None, None


class StftLossFn(torch.autograd.Function):
    """One resolution of the multi-resolution STFT loss: (spectral convergence ||y - x||_F / ||y||_F,
    mean |log y - log x|) of magnitudes x (differentiable) and y (target)."""

    @staticmethod
    def forward(ctx, xm, ym):
        sums = ops.stft_loss_sums(xm, ym)
        ctx.save_for_backward(xm, ym, sums)
        return torch.sqrt(sums[0] / sums[1]), sums[2] / xm.numel()

    @staticmethod
    def backward(ctx, g_sc, g_mag):
        xm, ym, sums = ctx.saved_tensors
        w = torch.stack([g_sc if g_sc is not None else sums.new_zeros(()),
                         g_mag if g_mag is not None else sums.new_zeros(())])
        return ops.stft_loss_grad(xm, ym, sums, w), None
