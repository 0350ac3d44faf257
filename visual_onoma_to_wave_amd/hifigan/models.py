"""HiFi-GAN V1 generator on HIP kernels (reference: scripts/hifigan/models.py:20-174).

Parameters are registered exactly as the reference registers them (weight-normed
Conv1d / ConvTranspose1d: ``weight_g`` / ``weight_v`` + ``bias``) so the "universal"
checkpoint's 234 keys load unchanged; ``remove_weight_norm()`` folds them like the
reference.  The forward never calls the torch modules: each conv is one channels-last
implicit-GEMM MFMA launch (``vo_conv1d``) with the leaky-ReLU applied while staging
its input, the ResBlock residual / MRF sum / 1/num_kernels scale in its epilogue, and
each ConvTranspose1d upsampler in its polyphase form.
"""

import contextlib
import os
import warnings

import torch
import torch.nn as nn
from torch.nn import Conv1d, ConvTranspose1d

from .. import ops, profiling
from .._base import HipModule

LRELU_SLOPE = 0.1
# K = 3 ResBlocks as one vo_resblock3 launch (VO_RB3=0: three vo_resblock_pair launches, for A/B)
RB3_ENABLED = os.environ.get("VO_RB3", "1") != "0"
# C = 128 k = 7 / 11 pairs on fragment-ordered weights (VO_FRAG=0: the [K][Co][Ci] packs, for A/B)
FRAG_ENABLED = os.environ.get("VO_FRAG", "1") != "0"
# Conv-path MRF stages (C = 256: two conv launches per ResBlock iteration) run their ResBlock
# chains on concurrent streams (VO_MRF_STREAMS=0: one after another, for A/B)
MRF_STREAMS = os.environ.get("VO_MRF_STREAMS", "1") != "0"
_SIDE_STREAMS = {}


def _side_streams(device, n):
    """n cached side streams of ``device`` (created once: stream creation is not free)."""
    key = (str(device), n)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = [torch.cuda.Stream(device=device) for _ in range(n)]
    return _SIDE_STREAMS[key]

with warnings.catch_warnings():
    warnings.simplefilter("ignore")
    from torch.nn.utils import remove_weight_norm, weight_norm


def init_weights(m, mean=0.0, std=0.01):
    if "Conv" in m.__class__.__name__:
        m.weight.data.normal_(mean, std)


def get_padding(kernel_size, dilation=1):
    return int((kernel_size * dilation - dilation) / 2)


def _wn(conv):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return weight_norm(conv)


def _weight_and_gain(m):
    """(v, g) when weight-normed, else (weight, None)."""
    if hasattr(m, "weight_v"):
        return m.weight_v, m.weight_g
    return m.weight, None


def _pack(m, device, dtype, transposed_stride=None):
    v, g = _weight_and_gain(m)
    w = ops.pack_conv_weight(v.to(device), dtype, g=None if g is None else g.to(device),
                             transposed_stride=transposed_stride)
    return w, m.bias.detach().float().to(device).contiguous()


class ResBlock(HipModule):
    """ResBlock1: for d in dilations: x = c2(lrelu(c1_d(lrelu(x)))) + x."""

    def __init__(self, h, channels, kernel_size=3, dilation=(1, 3, 5)):
        super().__init__()
        self.h, self.channels, self.kernel_size, self.dilation = h, channels, kernel_size, tuple(dilation)
        # channel widths that run each (c1, c2) pair as one vo_resblock_pair launch (bf16 only).
        # Measured on MI355X at B=32 (k=3/7/11): C=32 0.16/0.21/0.30 ms vs 0.37/0.40/0.48 ms for
        # two conv launches; C=64 0.24/0.37/0.47 vs 0.44/0.52/0.60; C=128 0.39/0.64/0.93 vs
        # 0.66/0.80/1.03 (tools/ab_pair.py).
        self.fused_pair_channels = (32, 64, 128)
        self.convs1 = nn.ModuleList(
            _wn(Conv1d(channels, channels, kernel_size, 1, dilation=d, padding=get_padding(kernel_size, d)))
            for d in self.dilation)
        self.convs1.apply(init_weights)
        self.convs2 = nn.ModuleList(
            _wn(Conv1d(channels, channels, kernel_size, 1, dilation=1, padding=get_padding(kernel_size, 1)))
            for _ in self.dilation)
        self.convs2.apply(init_weights)

    def _build(self, device, dtype):
        packs = [(_pack(c1, device, dtype), _pack(c2, device, dtype)) for c1, c2 in zip(self.convs1, self.convs2)]
        if self.channels in (64, 128) and self.kernel_size in (7, 11) and dtype == torch.bfloat16 and FRAG_ENABLED:
            # the C = 64 / 128 pair kernel streams its weights in fragment order (vo_pack_frag)
            packs = [p + ((ops.pack_frag(p[0][0]), ops.pack_frag(p[1][0])),) for p in packs]
        return packs

    def fused(self, x):
        """True when this ResBlock runs as fused pair / block launches (else two convs per pair)."""
        return self.channels in self.fused_pair_channels and x.dtype == self.compute_dtype == torch.bfloat16

    def run(self, x, out=None, out_scale=1.0, accumulate=None, stage=None, before_last=None):
        """x (B, T, C) channels-last -> ResBlock(x) * out_scale (+ accumulate), written to out.
        ``stage`` (0..3) selects the MRF stage's own kernel instantiation and timer tag.
        ``before_last`` (conv path only) is called right before the launch that reads
        ``accumulate`` -- the MRF's concurrent chains order their accumulations there."""
        var = 0 if stage is None else stage + 1
        tag = None if stage is None else f"mrf_s{stage}"
        packs = self._packed(x.device, self._build)
        k, C = self.kernel_size, self.channels
        cur = x
        if (RB3_ENABLED and k == 3 and len(self.dilation) == 3 and C in self.fused_pair_channels
                and x.dtype == self.compute_dtype == torch.bfloat16
                and sum(d + 1 for d in self.dilation) <= 12 and max(self.dilation) <= 8):
            # k = 3: the whole ResBlock (three pairs) in one launch; x1 / x2 stay on chip
            (w1s, b1s), (w2s, b2s) = zip(*[p[0] for p in packs]), zip(*[p[1] for p in packs])
            return ops.resblock3(cur, w1s, b1s, w2s, b2s, self.dilation, LRELU_SLOPE, out=out,
                                 out_scale=out_scale, acc=accumulate, tag=tag)
        if C in self.fused_pair_channels and x.dtype == self.compute_dtype == torch.bfloat16:
            # narrow stages: one fused launch per (c1, c2) pair, the intermediate stays in LDS
            for n, (d, p) in enumerate(zip(self.dilation, packs)):
                (w1, b1), (w2, b2) = p[0], p[1]
                frag = len(p) > 2
                if frag:
                    w1, w2 = p[2]
                last = n == len(self.dilation) - 1
                cur = ops.resblock_pair(cur, w1, b1, w2, b2, k, d, LRELU_SLOPE, out=out if last else None,
                                        out_scale=out_scale if last else 1.0,
                                        acc=accumulate if last else None, tag=tag, frag=frag)
            return cur
        for n, (d, p) in enumerate(zip(self.dilation, packs)):
            (w1, b1), (w2, b2) = p[0], p[1]
            t = ops.conv1d(cur, w1, b1, Co=C, K=k, dil=d, pad=get_padding(k, d), pre_act=ops.ACT_LRELU,
                           pre_slope=LRELU_SLOPE, post_act=ops.ACT_LRELU, post_slope=LRELU_SLOPE,
                           compute_dtype=self.compute_dtype, out_dtype=x.dtype, variant=var, tag=tag)
            last = n == len(self.dilation) - 1
            if last and before_last is not None:
                before_last()
            cur = ops.conv1d(t, w2, b2, Co=C, K=k, pad=get_padding(k, 1), res1=cur,
                             out=out if last else None, out_scale=out_scale if last else 1.0,
                             res2=accumulate if last else None, compute_dtype=self.compute_dtype,
                             out_dtype=x.dtype, variant=var, tag=tag)
        return cur

    def forward(self, x):
        self._check_inference()
        xc = ops.transpose_bct(x, self.compute_dtype)
        y = self.run(xc)
        return ops.transpose_bct(y.float(), torch.float32)

    def remove_weight_norm(self):
        for m in list(self.convs1) + list(self.convs2):
            remove_weight_norm(m)


class Generator(HipModule):
    def __init__(self, h):
        super().__init__()
        self.h = h
        self.num_kernels = len(h.resblock_kernel_sizes)
        self.num_upsamples = len(h.upsample_rates)
        c0 = h.upsample_initial_channel
        self.conv_pre = _wn(Conv1d(80, c0, 7, 1, padding=3))
        self.ups = nn.ModuleList(
            _wn(ConvTranspose1d(c0 // 2 ** i, c0 // 2 ** (i + 1), k, u, padding=(k - u) // 2))
            for i, (u, k) in enumerate(zip(h.upsample_rates, h.upsample_kernel_sizes)))
        self.resblocks = nn.ModuleList(
            ResBlock(h, c0 // 2 ** (i + 1), k, d)
            for i in range(len(self.ups))
            for k, d in zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes))
        self.conv_post = _wn(Conv1d(c0 // 2 ** len(self.ups), 1, 7, 1, padding=3))
        self.ups.apply(init_weights)
        self.conv_post.apply(init_weights)

    def _build(self, device, dtype):
        ups = []
        for m, u, k in zip(self.ups, self.h.upsample_rates, self.h.upsample_kernel_sizes):
            if k != 2 * u:
                raise NotImplementedError("polyphase ConvTranspose1d needs kernel = 2 * stride")
            ups.append(_pack(m, device, dtype, transposed_stride=u) + (m.out_channels, u, (k - u) // 2))
        v, g = _weight_and_gain(self.conv_post)
        wpost = ops.pack_conv_weight(v.to(device), torch.float32, g=None if g is None else g.to(device))
        return dict(pre=_pack(self.conv_pre, device, dtype), ups=ups,
                    post=(wpost.reshape(wpost.shape[0], -1).contiguous(),
                          float(self.conv_post.bias.detach().float().cpu())))

    def run(self, mel_cl):
        """mel_cl (B, T, 80) channels-last (fp32 or compute dtype) -> wav (B, 256*T) fp32."""
        p = self._packed(mel_cl.device, self._build)
        dt = self.compute_dtype
        w, b = p["pre"]
        x = ops.conv1d(mel_cl, w, b, Co=w.shape[1], K=7, pad=3, out_dtype=dt, compute_dtype=dt)
        for i in range(self.num_upsamples):
            w, b, cout, u, pad = p["ups"][i]
            x = ops.conv1d(x, w, b, Co=u * cout, K=2, pad=1, pre_act=ops.ACT_LRELU, pre_slope=LRELU_SLOPE,
                           transposed=dict(stride=u, pad=pad, cout=cout), out_dtype=dt, compute_dtype=dt)
            x = self.mrf(i, x)
        wk, bp = p["post"]
        return ops.conv_post(x, wk, bp, slope=0.01)

    def mrf(self, i, x):
        """Multi-receptive-field fusion of upsampling stage i (hifigan/models.py:155-160):
        (sum_j ResBlock_{i,j}(x)) / num_kernels on channels-last x (B, T, C) in the compute
        dtype; the ResBlocks accumulate into one output in their epilogues."""
        xs = torch.empty_like(x)
        stage = i if self.num_upsamples == 4 else None
        timer = profiling.active()
        tag = f"mrf_s{i}"
        # the stage's ResBlock launches are consecutive: one event pair for all of them
        grp = timer.group(tag) if (stage is not None and timer is not None and timer.watching(tag)) \
            else contextlib.nullcontext()
        rbs = list(self.resblocks[i * self.num_kernels:(i + 1) * self.num_kernels])
        for rb in rbs:
            rb.compute_dtype = self.compute_dtype
        with grp:
            if MRF_STREAMS and x.is_cuda and len(rbs) > 1 and not any(rb.fused(x) for rb in rbs):
                self._mrf_concurrent(rbs, x, xs, stage)
            else:
                for j, rb in enumerate(rbs):
                    rb.run(x, out=xs, out_scale=1.0 / self.num_kernels, accumulate=xs if j > 0 else None,
                           stage=stage)
        return xs

    def _mrf_concurrent(self, rbs, x, xs, stage):
        """The MRF's ResBlock chains are independent until their sum: chain j runs on its own
        stream, and only its last launch (the one that adds into ``xs``) waits for chain j - 1's
        last launch, so the sum is formed in the same order as the sequential loop (bit-identical
        output).  The C = 256 stage's convs are non-persistent two-round launches whose
        residual / accumulator epilogues load HBM all at once; overlapping the chains lets one
        chain's epilogue traffic run under another's MFMA work."""
        main = torch.cuda.current_stream(x.device)
        side = _side_streams(x.device, len(rbs) - 1)
        chain_streams = [main] + side
        for s in side:
            s.wait_stream(main)  # x (and xs's allocation) are ordered on main
            x.record_stream(s)
            xs.record_stream(s)
        done = [None] * len(rbs)
        for j, (rb, s) in enumerate(zip(rbs, chain_streams)):
            def before_last(j=j, s=s):
                if j > 0:
                    s.wait_event(done[j - 1])
            with torch.cuda.stream(s):
                rb.run(x, out=xs, out_scale=1.0 / self.num_kernels, accumulate=xs if j > 0 else None,
                       stage=stage, before_last=before_last)
                done[j] = torch.cuda.Event()
                done[j].record(s)
        main.wait_event(done[-1])  # chain j's completion implies chains < j (their last launches)

    def train_forward(self, mel_cl):
        """Differentiable forward for HiFi-GAN training (config C5): mel_cl (B, T, 80)
        channels-last -> wav (B, 256 T) fp32.  Same HIP conv kernels as ``run`` (pre-lrelu while
        staging, residual and MRF sum in the epilogue), one launch per conv (the fused pair
        kernel has no backward), gradients through ``gan_ops.ConvFn``; the weight-norm
        reparameterisation w = g v / ||v|| of every conv runs as one batched HIP launch
        (``gan_ops.WeightNormFn``, forward and backward)."""
        from . import gan_ops as G
        dt = self.compute_dtype
        adt = torch.float32 if dt == torch.float32 else torch.bfloat16

        # every weight-normed conv's w = g v / ||v|| in one batched launch (and one in the backward),
        # then every packed weight the convs below look up in one more (gan_ops.prepack)
        W = G.weight_norm_all(list(self.modules()))

        def wgt(m):
            return W[m] if m in W else m.weight
        plan = self._train_plan(mel_cl.shape[0], mel_cl.shape[1])
        G.prepack([(G.weight_key(m), wgt(m), sp, shape, m is not self.conv_pre, res) for m, sp, shape, res in plan], dt)
        spec = {m: sp for m, sp, _, _ in plan}

        x = G.conv(mel_cl.to(adt).contiguous(), wgt(self.conv_pre), self.conv_pre.bias, spec[self.conv_pre], dt,
                   wkey=G.weight_key(self.conv_pre))
        for i in range(self.num_upsamples):
            m = self.ups[i]
            x = G.conv(x, wgt(m), m.bias, spec[m], dt, wkey=G.weight_key(m))
            xs = None
            for j in range(self.num_kernels):
                rb = self.resblocks[i * self.num_kernels + j]
                cur = x
                for n, (c1, c2) in enumerate(zip(rb.convs1, rb.convs2)):
                    # after the first pair, cur has exactly two uses (c1's input, c2's residual):
                    # their gradients meet in c1's leaky-ReLU mask pass (gan_ops.ResLink)
                    lk = G.ResLink() if n > 0 and G.RES_LINK else None
                    t = G.conv(cur, wgt(c1), c1.bias, spec[c1], dt, wkey=G.weight_key(c1),
                               link=(lk, "in") if lk else None)
                    last = n == len(rb.dilation) - 1
                    cur = G.conv(t, wgt(c2), c2.bias, spec[c2], dt, res1=cur, res2=xs if last else None,
                                 wkey=G.weight_key(c2), link=(lk, "res") if lk else None)
                xs = cur
            x = xs
        m = self.conv_post
        y = G.conv(x, wgt(m), m.bias, spec[m], dt, wkey=G.weight_key(m))
        return y[..., 0].float()

    def _train_plan(self, B, T):
        """[(module, ConvSpec, input shape (N, T, C), has residual inputs)] of ``train_forward``'s
        convs for a (B, T, 80) mel batch, in launch order."""
        from . import gan_ops as G
        plan = [(self.conv_pre, G.ConvSpec(K=7, pad=3), (B, T, self.conv_pre.in_channels), False)]
        C = self.conv_pre.out_channels
        for i, (u, k) in enumerate(zip(self.h.upsample_rates, self.h.upsample_kernel_sizes)):
            m = self.ups[i]
            sp = G.ConvSpec(K=k, pad=(k - u) // 2, pre_slope=LRELU_SLOPE, transposed=(u, (k - u) // 2))
            plan.append((m, sp, (B, T, C), False))
            T, C = G.out_len(sp, T), m.out_channels
            for j in range(self.num_kernels):
                rb = self.resblocks[i * self.num_kernels + j]
                kk = rb.kernel_size
                for n, (d, c1, c2) in enumerate(zip(rb.dilation, rb.convs1, rb.convs2)):
                    plan.append((c1, G.ConvSpec(K=kk, pad=get_padding(kk, d), dil=d, pre_slope=LRELU_SLOPE,
                                                post="lrelu", post_slope=LRELU_SLOPE), (B, T, C), False))
                    last = n == len(rb.dilation) - 1
                    plan.append((c2, G.ConvSpec(K=kk, pad=get_padding(kk, 1),
                                                out_scale=1.0 / self.num_kernels if last else 1.0), (B, T, C), True))
        plan.append((self.conv_post, G.ConvSpec(K=7, pad=3, pre_slope=0.01, post="tanh", co_pad=4), (B, T, C), False))
        return plan

    def forward(self, x):
        """x (B, 80, T) mel -> (B, 1, 256 * T) waveform (reference: models.py:149-165)."""
        self._check_inference()
        mel_cl = ops.transpose_bct(x, torch.float32)
        return self.run(mel_cl).unsqueeze(1)

    def remove_weight_norm(self):
        print("Removing weight norm...")
        for m in self.ups:
            remove_weight_norm(m)
        for rb in self.resblocks:
            rb.remove_weight_norm()
        remove_weight_norm(self.conv_pre)
        remove_weight_norm(self.conv_post)
