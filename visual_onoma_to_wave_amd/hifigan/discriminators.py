"""HiFi-GAN V1 discriminators and losses on HIP kernels (config C5).

The reference ships the generator and the training hyper-parameters only
(scripts/hifigan/models.py, scripts/hifigan/config.json); these modules follow the HiFi-GAN
V1 recipe that config belongs to, with its module / parameter names (``mpd.discriminators.N.
convs.M.weight_g`` ...), so an upstream HiFi-GAN ``do_*`` discriminator checkpoint loads:

* DiscriminatorP(period): wav reflect-padded to a multiple of p and viewed (T/p, p); five
  Conv2d (5, 1) / (3, 1) (1 -> 32 -> 128 -> 512 -> 1024, last one stride 1) + leaky ReLU 0.1,
  conv_post Conv2d (3, 1) -> 1.  Here: each period column is a sequence of a channels-last
  (B * p, T/p, C) batch and each Conv2d (k, 1) is one strided ``vo_conv1d`` launch.
* DiscriminatorS: Conv1d 1 -> 128 (15), grouped strided Conv1d (41, groups 4 / 16, strides
  2, 2, 4, 4, 1), Conv1d (5), conv_post (3); the first of the three scales spectral-normed.
  Grouped convs run as ``vo_conv1d`` groups mode over block-diagonal packed weights.
* MultiScaleDiscriminator: raw wav, AvgPool1d(4, 2, padding 2) once and twice.
* Losses: feature_loss = 2 * sum mean|f_r - f_g|; discriminator_loss = sum mean((1 - D(y))^2)
  + mean(D(G(x))^2); generator_loss = sum mean((1 - D(G(x)))^2) (fp32 ``vo_gan_reduce``).

Activations are bf16 (``compute_dtype`` float32 = exact-f32 parity mode).  Scores and
feature maps come back in this layout: MPD (B * p, H, C), MSD (B, T, C); the losses are
means, independent of it.
"""

import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import Conv1d, Conv2d

from .. import ops
from . import gan_ops as G

LRELU_SLOPE = 0.1

with warnings.catch_warnings():
    warnings.simplefilter("ignore")
    from torch.nn.utils import spectral_norm, weight_norm
    from torch.nn.utils.spectral_norm import SpectralNorm


def get_padding(kernel_size, dilation=1):
    return int((kernel_size * dilation - dilation) / 2)


def effective_weight(m):
    """The weight a weight-normed / spectral-normed conv would use in this forward (torch
    parameterisation math: w = g v / ||v||, or the power-iteration sigma in training mode)."""
    if hasattr(m, "weight_g"):
        # the same kernel as the batched training path (vo_weight_norm): the packed-weight cache is
        # keyed on parameter versions only, so every path must derive bit-identical weights
        return G.weight_norm_all([m])[m]
    for hook in m._forward_pre_hooks.values():
        if isinstance(hook, SpectralNorm):
            hook(m, None)
            return m.weight
    return m.weight


def _weight(m):
    """``effective_weight(m)``; while it needs no gradient (frozen discriminator in the G step, or
    no_grad) the value is reused across forwards at unchanged parameter versions (the G step
    runs each discriminator twice: real half without graph, generated half)."""
    wkey = G.weight_key(m)
    p = m.weight_v if hasattr(m, "weight_v") else m.weight
    if G.volatile(wkey) or (torch.is_grad_enabled() and p.requires_grad):
        return effective_weight(m)
    return G._cached(wkey, "w_eff", lambda: effective_weight(m).detach())


def _conv_w(m, w):
    return w.squeeze(-1) if w.dim() == 4 else w  # Conv2d (k, 1) weights as Conv1d


def _prepare(root, layers, dgrad_first):
    """Effective weights ``W`` of every weight-normed conv under ``root`` -- one batched launch,
    differentiable while the discriminator trains (autograd records and its parameters require
    grad), else cached at the parameters' versions (the frozen G step runs D twice) -- and every
    packed weight the convs in ``layers`` (per discriminator: [(module, spec, input shape)] in
    forward order) will look up, written by one ``gan_ops.prepack`` launch (input-gradient layouts
    for all but each discriminator's first conv, and for those too with ``dgrad_first``)."""
    mods = [m for m in root.modules() if hasattr(m, "weight_g")]
    if not mods:
        W = {}
    elif torch.is_grad_enabled() and any(m.weight_v.requires_grad for m in mods):
        W = G.weight_norm_all(mods)
    else:
        key = (root,) + tuple(v for m in mods for v in (m.weight_v._version, m.weight_g._version))
        W = G._cached(key, "W_frozen", lambda: dict(zip(mods, ops.weight_norm(
            [m.weight_v.detach() for m in mods], [m.weight_g.detach() for m in mods]))))
    if G.BATCHED_SN:  # the spectral-normed convs: one power iteration per pass, as the hook would
        W = {**W, **G.spectral_norm_all([m for m in root.modules() if hasattr(m, "weight_orig")])}
    cdt = root.compute_dtype
    G.prepack([(G.weight_key(m), _conv_w(m, W[m]), sp, shape, dgrad_first or i > 0)
               for d in layers for i, (m, sp, shape) in enumerate(d) if m in W], cdt)
    return W


def _w(m, W):
    return W[m] if W and m in W else _weight(m)


class _DiscBase(nn.Module):
    compute_dtype = torch.bfloat16

    def set_compute_dtype(self, dt):
        for m in self.modules():
            if isinstance(m, _DiscBase):
                m.compute_dtype = dt
        return self

    def _act_dtype(self):
        return torch.float32 if self.compute_dtype == torch.float32 else torch.bfloat16


class DiscriminatorP(_DiscBase):
    def __init__(self, period, kernel_size=5, stride=3, use_spectral_norm=False):
        super().__init__()
        self.period, self.kernel_size, self.stride = period, kernel_size, stride
        norm_f = spectral_norm if use_spectral_norm else weight_norm
        pad = (get_padding(5, 1), 0)
        chans = [1, 32, 128, 512, 1024]
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            self.convs = nn.ModuleList(
                [norm_f(Conv2d(chans[i], chans[i + 1], (kernel_size, 1), (stride, 1), padding=pad)) for i in range(4)]
                + [norm_f(Conv2d(1024, 1024, (kernel_size, 1), 1, padding=(2, 0)))])
            self.conv_post = norm_f(Conv2d(1024, 1, (3, 1), 1, padding=(1, 0)))

    def _specs(self):
        k, s = self.kernel_size, self.stride
        specs = [G.ConvSpec(K=k, pad=get_padding(5, 1), stride=s, post="lrelu", post_slope=LRELU_SLOPE,
                            ci_pad=8 if i == 0 else None) for i in range(4)]
        specs.append(G.ConvSpec(K=k, pad=2, post="lrelu", post_slope=LRELU_SLOPE))
        return specs, G.ConvSpec(K=3, pad=1, co_pad=8)  # 8: dY needs no channel padding in the backward

    def _layers(self, B, T):
        """[(module, spec, input shape (N, T, C))] of ``forward``'s convs for a (B, T) wav batch."""
        N, H, C = B * self.period, -(-T // self.period), 8
        specs, post = self._specs()
        out = []
        for m, sp in zip(list(self.convs) + [self.conv_post], specs + [post]):
            out.append((m, sp, (N, H, C)))
            H, C = G.out_len(sp, H), m.out_channels
        return out

    def forward(self, wav, W=None, fmaps=True):
        """wav (B, T) fp32 -> (score (B * p, H'), fmaps [(B * p, H_l, C_l)]); ``fmaps`` False: the feature
        maps come back detached (the D step), which lets each layer's leaky-ReLU backward ride in the next
        conv's input-gradient epilogue (gan_ops.conv_layers).  ``W``: effective
        weights batched (and the convs' weights packed) by the caller (``_prepare``)."""
        cdt, adt = self.compute_dtype, self._act_dtype()
        layers = self._layers(*wav.shape)
        if W is None:
            W = _prepare(self, [layers], wav.requires_grad)
        x = G.PeriodFoldFn.apply(wav, self.period, adt)
        # squeeze, not [..., 0]: its adjoint is a view of the 3-D weight gradient (select's was a zero
        # fill and a copy per conv and D step)
        fmap = G.conv_layers(x, [(_w(m, W).squeeze(-1), m.bias, sp, cdt, G.weight_key(m)) for m, sp, _ in layers],
                             fmaps)
        score = fmap[-1][..., 0].contiguous()
        fmap[-1] = score
        return score, fmap


class MultiPeriodDiscriminator(_DiscBase):
    def __init__(self, periods=(2, 3, 5, 7, 11)):
        super().__init__()
        self.discriminators = nn.ModuleList(DiscriminatorP(p) for p in periods)

    def prepare(self, wav, dgrad_first=None):
        """``_prepare`` over every period's convs for a (B, T) wav batch -> W."""
        layers = [d._layers(*wav.shape) for d in self.discriminators]
        return _prepare(self, layers, wav.requires_grad if dgrad_first is None else dgrad_first)

    def forward(self, y, y_hat, fmaps=True):
        """Reference call convention: (y_d_rs, y_d_gs, fmap_rs, fmap_gs).  y and y_hat run as one
        batch (one launch per layer for both)."""
        B = y.shape[0]
        both = torch.cat([y, y_hat], 0)
        W = self.prepare(both)
        rs, gs, frs, fgs = [], [], [], []
        for d in self.discriminators:
            p = d.period
            s, fm = d(both, W, fmaps)
            rs.append(s[: B * p])
            gs.append(s[B * p:])
            frs.append([f[: B * p] for f in fm])
            fgs.append([f[B * p:] for f in fm])
        return rs, gs, frs, fgs


class DiscriminatorS(_DiscBase):
    def __init__(self, use_spectral_norm=False):
        super().__init__()
        norm_f = spectral_norm if use_spectral_norm else weight_norm
        cfg = [(1, 128, 15, 1, 1, 7), (128, 128, 41, 2, 4, 20), (128, 256, 41, 2, 16, 20), (256, 512, 41, 4, 16, 20),
               (512, 1024, 41, 4, 16, 20), (1024, 1024, 41, 1, 16, 20), (1024, 1024, 5, 1, 1, 2)]
        self.cfg = cfg
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            self.convs = nn.ModuleList(norm_f(Conv1d(ci, co, k, s, groups=g, padding=p)) for ci, co, k, s, g, p in cfg)
            self.conv_post = norm_f(Conv1d(1024, 1, 3, 1, padding=1))

    def _layers(self, B, T):
        """[(module, spec, input shape (N, T, C))] of ``forward``'s convs for a (B, T) wav batch."""
        out, C = [], 8
        for m, (ci, co, k, s, g, p) in zip(self.convs, self.cfg):
            sp = G.ConvSpec(K=k, pad=p, stride=s, groups=g, post="lrelu", post_slope=LRELU_SLOPE,
                            ci_pad=8 if ci == 1 else None)
            out.append((m, sp, (B, T, C)))
            T, C = G.out_len(sp, T), co
        out.append((self.conv_post, G.ConvSpec(K=3, pad=1, co_pad=8), (B, T, C)))
        return out

    def forward(self, wav, W=None, fmaps=True):
        """wav (B, T) fp32 -> (score (B, T'), fmaps [(B, T_l, C_l)])."""
        cdt, adt = self.compute_dtype, self._act_dtype()
        layers = self._layers(*wav.shape)
        if W is None:
            W = _prepare(self, [layers], wav.requires_grad)
        x = G.WavCl8Fn.apply(wav, adt)
        fmap = G.conv_layers(x, [(_w(m, W), m.bias, sp, cdt, G.weight_key(m)) for m, sp, _ in layers], fmaps)
        score = fmap[-1][..., 0].contiguous()
        fmap[-1] = score
        return score, fmap


class MultiScaleDiscriminator(_DiscBase):
    def __init__(self):
        super().__init__()
        self.discriminators = nn.ModuleList(
            [DiscriminatorS(use_spectral_norm=True), DiscriminatorS(), DiscriminatorS()])

    def prepare(self, wav, dgrad_first=None):
        """``_prepare`` over the three scales' convs for a (B, T) wav batch -> W."""
        B, T = wav.shape
        layers = []
        for i, d in enumerate(self.discriminators):
            if i:
                T = T // 2 + 1  # AvgPool1d(4, 2, padding 2)
            layers.append(d._layers(B, T))
        return _prepare(self, layers, wav.requires_grad if dgrad_first is None else dgrad_first)

    def forward(self, y, y_hat, fmaps=True):
        B = y.shape[0]
        x = torch.cat([y, y_hat], 0)
        W = self.prepare(x)
        rs, gs, frs, fgs = [], [], [], []
        for i, d in enumerate(self.discriminators):
            if i != 0:
                x = G.AvgPoolFn.apply(x)
            s, fm = d(x, W, fmaps)
            rs.append(s[:B])
            gs.append(s[B:])
            frs.append([f[:B] for f in fm])
            fgs.append([f[B:] for f in fm])
        return rs, gs, frs, fgs


def feature_loss(fmap_r, fmap_g):
    """2 * sum over discriminators and layers of mean|f_r - f_g| (f_r held constant): one
    ``gan_loss_terms`` vector for every layer."""
    items = [(gl, rl, ops.GAN_L1, 2.0 / gl.numel()) for dr, dg in zip(fmap_r, fmap_g) for rl, gl in zip(dr, dg)]
    return G.gan_loss_terms(items).sum()


def discriminator_loss(disc_real_outputs, disc_generated_outputs):
    """(sum of mean((1 - D(y))^2) + mean(D(G(x))^2), [real terms], [generated terms])."""
    n = len(disc_real_outputs)
    t = G.gan_split_terms(disc_real_outputs, disc_generated_outputs, ops.GAN_ONE_MINUS_SQ, ops.GAN_SQ)
    return t.sum(), list(t[:n].unbind()), list(t[n:].unbind())


def generator_loss(disc_outputs):
    """(sum of mean((1 - D(G(x)))^2), [terms])."""
    t = G.gan_loss_terms([(dg, None, ops.GAN_ONE_MINUS_SQ, 1.0 / dg.numel()) for dg in disc_outputs])
    return t.sum(), list(t.unbind())


class MelLoss(nn.Module):
    """HiFi-GAN training mel (meldataset.mel_spectrogram with fmax_for_loss) on vo_stft_mel_ex."""

    def __init__(self, n_fft=1024, num_mels=80, sampling_rate=22050, hop_size=256, win_size=1024, fmin=0,
                 fmax=None):
        super().__init__()
        from ..audio import librosa_mel
        if win_size != n_fft:
            raise NotImplementedError("win_size != n_fft")
        self.n_fft, self.hop = n_fft, hop_size
        fb = librosa_mel(sampling_rate, n_fft, num_mels, fmin, fmax)  # (n_mels, n_fft/2 + 1)
        self.register_buffer("fb", torch.from_numpy(fb).t().contiguous(), persistent=False)
        self.register_buffer("window", torch.hann_window(win_size), persistent=False)

    def mel(self, wav):
        return G.MelFn.apply(wav, self.window, self.fb, self.n_fft, self.hop)

    def forward(self, wav_hat, mel_target):
        return G.l1_mean(self.mel(wav_hat), mel_target)


class MultiResolutionSTFTLoss(nn.Module):
    """Auxiliary multi-resolution STFT loss (BASELINE.json config C5; Parallel WaveGAN,
    Yamamoto et al. 2020): per resolution (n_fft, hop, win) the spectral convergence and the mean
    log-magnitude L1 of |STFT| (hann window of win samples zero-padded to n_fft, center=True),
    each averaged over the resolutions.  Forward, backward and reductions on HIP."""

    def __init__(self, fft_sizes=(1024, 2048, 512), hop_sizes=(120, 240, 50), win_lengths=(600, 1200, 240)):
        super().__init__()
        self.res = list(zip(fft_sizes, hop_sizes, win_lengths))
        for i, (n, _, w) in enumerate(self.res):
            win = torch.zeros(n)
            left = (n - w) // 2
            win[left: left + w] = torch.hann_window(w)
            self.register_buffer(f"window{i}", win, persistent=False)

    def forward(self, wav_hat, wav):
        """(sc, mag) of wav_hat (B, N) against wav (B, N)."""
        sc = mag = 0.0
        for i, (n, hop, _) in enumerate(self.res):
            window = getattr(self, f"window{i}")
            xm = G.StftMagFn.apply(wav_hat, window, n, hop)
            with torch.no_grad():
                ym = ops.stft_mag(wav.contiguous(), window, n, hop)
            s, m = G.StftLossFn.apply(xm, ym)
            sc = sc + s
            mag = mag + m
        return sc / len(self.res), mag / len(self.res)
