"""HiFi-GAN V1 training step (config C5) with data parallelism.

Hyper-parameters come from the reference's scripts/hifigan/config.json (batch 16 per GPU,
segment 8192, AdamW lr 2e-4, betas (0.8, 0.99), per-epoch ExponentialLR 0.999, fmax_for_loss
null); the step follows the HiFi-GAN V1 recipe that config belongs to:

  D step: L_D = sum_{MPD, MSD} [mean((1 - D(y))^2) + mean(D(G(x).detach())^2)]
  G step: L_G = sum adv mean((1 - D(G(x)))^2) + 2 sum_l mean|D_l(y) - D_l(G(x))| + 45 L1(mel)
          [+ stft_loss_weight (spectral convergence + log |STFT| L1) of the multi-resolution STFT
           loss (BASELINE.json config C5's "multi-res STFT loss"; off by default = HiFi-GAN V1)]

Multi-GPU: one process per GPU; generator and discriminator gradients are averaged by two
bucketed RCCL all-reduces (``train.GradBucketer``) launched from backward hooks, so each
overlaps the rest of its backward.  In the G step the discriminators are frozen (their
gradients would be discarded by the next D step's zero_grad) and run on the real batch
under no_grad: one backward through D on the generated half only.
"""

import itertools

import torch

from .. import _base, optim
from ..train import GradBucketer, TrainState, _capture_ctx, _check_graph_runtime, _warmup_ctx
from .discriminators import (MelLoss, MultiPeriodDiscriminator, MultiResolutionSTFTLoss, MultiScaleDiscriminator,
                             discriminator_loss, feature_loss, generator_loss)


def _single(disc, wav, grad):
    """(scores, fmaps) of a Multi*Discriminator on one batch."""
    scores, fmaps = [], []
    ctx = torch.enable_grad() if grad else torch.no_grad()
    with ctx:
        # frozen D: one weight-norm and one packing launch for the real and the generated pass
        # together (both at these parameter versions; the generated pass's backward needs the
        # input-gradient layouts of every conv)
        W = disc.prepare(wav, dgrad_first=True)
        x = wav
        for i, d in enumerate(disc.discriminators):
            if isinstance(disc, MultiScaleDiscriminator) and i:
                from . import gan_ops
                x = gan_ops.AvgPoolFn.apply(x)
            s, f = d(x, W)
            scores.append(s)
            fmaps.append(f)
    return scores, fmaps


class HifiGanTrainer:
    """``graphed=True``: ``step_graphed`` replays the whole step (both optimiser steps and, with
    ``distributed=True``, both bucketed RCCL all-reduces included) as one HIP graph captured
    after eager warm-up steps on a side stream whose effects are undone before the first replay
    -- the step launches ~4.6k kernels, and the eager loop is host-launch-bound.  AdamW then runs
    with ``capturable=True`` and device-tensor learning rates, so ``end_epoch``'s ExponentialLR
    decay is written into the captured step without re-capturing."""

    def __init__(self, generator, h, mpd=None, msd=None, distributed=False, device=None, graphed=False,
                 comm_dtype=None, capturable=None, stft_loss_weight=0.0):
        self.generator = generator
        device = device or next(generator.parameters()).device
        self.mpd = (mpd or MultiPeriodDiscriminator()).to(device)
        self.msd = (msd or MultiScaleDiscriminator()).to(device)
        self.h = h
        self.graphed = graphed
        self._graph = None
        if graphed:
            _check_graph_runtime()
        # capturable AdamW (device-tensor step counts and learning rates) is required for the graph
        # and may be chosen for eager steps too (capturable=True: the same update arithmetic)
        cap = graphed if capturable is None else bool(capturable)
        if graphed and not cap:
            raise ValueError("graphed training needs the capturable optimizer")
        lr = (lambda: torch.tensor(float(h.learning_rate), device=device)) if cap else (lambda: h.learning_rate)
        # AdamW (torch's defaults: weight decay 0.01, eps 1e-8) as multi-tensor HIP launches on the GPU
        adamw = optim.AdamW if torch.device(device).type == "cuda" else torch.optim.AdamW
        self.optim_g = adamw(generator.parameters(), lr(), betas=[h.adam_b1, h.adam_b2], capturable=cap)
        self.optim_d = adamw(itertools.chain(self.msd.parameters(), self.mpd.parameters()),
                             lr(), betas=[h.adam_b1, h.adam_b2], capturable=cap)
        self.sched_g = torch.optim.lr_scheduler.ExponentialLR(self.optim_g, gamma=h.lr_decay)
        self.sched_d = torch.optim.lr_scheduler.ExponentialLR(self.optim_d, gamma=h.lr_decay)
        self.mel_loss = MelLoss(h.n_fft, h.num_mels, h.sampling_rate, h.hop_size, h.win_size, h.fmin,
                                h.fmax_for_loss).to(device)
        self.stft_loss_weight = float(stft_loss_weight)
        self.stft_loss = MultiResolutionSTFTLoss().to(device) if self.stft_loss_weight else None
        self.bk_g = self.bk_d = None
        if distributed:
            self.bk_g = GradBucketer(list(generator.parameters()), comm_dtype=comm_dtype)
            self.bk_d = GradBucketer(list(self.msd.parameters()) + list(self.mpd.parameters()), comm_dtype=comm_dtype)
            self.bk_g.broadcast_parameters(generator)
            self.bk_d.broadcast_parameters(self.mpd)
            self.bk_d.broadcast_parameters(self.msd)

    def set_compute_dtype(self, dt):
        self.generator.set_compute_dtype(dt)
        self.mpd.set_compute_dtype(dt)
        self.msd.set_compute_dtype(dt)
        return self

    def _d_params(self):
        return itertools.chain(self.mpd.parameters(), self.msd.parameters())

    def step(self, x_mel_cl, y):
        """x_mel_cl (B, frames, 80) generator input mel (channels-last), y (B, 256 frames) fp32
        target segment -> dict of fp32 loss tensors (device scalars, no host sync)."""
        self.generator.train()
        self.mpd.train()
        self.msd.train()
        y_g_hat = self.generator.train_forward(x_mel_cl)
        with torch.no_grad():
            y_mel = self.mel_loss.mel(y)

        # discriminators: real and generated halves as one batch per layer
        for p in self._d_params():
            p.requires_grad_(True)
        self.optim_d.zero_grad(set_to_none=True)
        yd = y_g_hat.detach()
        # fmaps=False: the feature maps carry no gradient here, so each layer's leaky-ReLU backward
        # rides in the next conv's input-gradient epilogue (gan_ops.conv_layers)
        r, g, _, _ = self.mpd(y, yd, fmaps=False)
        loss_disc_f, _, _ = discriminator_loss(r, g)
        r, g, _, _ = self.msd(y, yd, fmaps=False)
        loss_disc_s, _, _ = discriminator_loss(r, g)
        loss_disc_all = loss_disc_s + loss_disc_f
        loss_disc_all.backward()
        if self.bk_d is not None:
            self.bk_d.finish()
        self.optim_d.step()

        # generator: D frozen, real features without graph
        for p in self._d_params():
            p.requires_grad_(False)
        self.optim_g.zero_grad(set_to_none=True)
        loss_mel = self.mel_loss(y_g_hat, y_mel) * 45
        _, fr_f = _single(self.mpd, y, False)
        _, fr_s = _single(self.msd, y, False)
        g_f, fg_f = _single(self.mpd, y_g_hat, True)
        g_s, fg_s = _single(self.msd, y_g_hat, True)
        loss_fm = feature_loss(fr_f, fg_f) + feature_loss(fr_s, fg_s)
        loss_adv = generator_loss(g_f)[0] + generator_loss(g_s)[0]
        loss_gen_all = loss_adv + loss_fm + loss_mel
        extra = {}
        if self.stft_loss is not None:
            sc, mag = self.stft_loss(y_g_hat, y)
            loss_stft = (sc + mag) * self.stft_loss_weight
            loss_gen_all = loss_gen_all + loss_stft
            extra["stft"] = loss_stft.detach()
        loss_gen_all.backward()
        if self.bk_g is not None:
            self.bk_g.finish()
        self.optim_g.step()
        for p in self._d_params():
            p.requires_grad_(True)
        return dict(disc=loss_disc_all.detach(), gen=loss_gen_all.detach(), mel=loss_mel.detach(),
                    fm=loss_fm.detach(), adv=loss_adv.detach(), **extra)

    def step_graphed(self, x_mel_cl, y, warmup=3):
        """``step`` as one HIP-graph replay (captured on the first call, after ``warmup`` eager
        steps on a side stream whose updates are then undone).  Inputs are copied into the
        graph's static buffers; the returned loss tensors are the graph's (overwritten by the next
        replay).  No host synchronisation."""
        from . import gan_ops
        if not self.graphed:
            raise RuntimeError("HifiGanTrainer: construct with graphed=True to replay steps as a HIP graph")
        if self._graph is None:
            self._x, self._y = x_mel_cl.clone(), y.clone()
            snap = TrainState([self.generator, self.mpd, self.msd], [self.optim_g, self.optim_d])
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side), _warmup_ctx([self.bk_g, self.bk_d]):
                for _ in range(warmup):
                    self.step(self._x, self._y)
            torch.cuda.current_stream().wait_stream(side)
            gan_ops.reset_pack_cache()
            graph = torch.cuda.CUDAGraph()
            with _capture_ctx([self.bk_g, self.bk_d]), torch.cuda.graph(graph):
                self._out = self.step(self._x, self._y)
            snap.restore()
            gan_ops.reset_pack_cache()
            _base.invalidate_packs(self.generator, self.mpd, self.msd)
            self._graph = graph
        self._x.copy_(x_mel_cl)
        self._y.copy_(y)
        self._graph.replay()
        gan_ops.reset_pack_cache()  # replays move the parameters without bumping their versions
        _base.invalidate_packs(self.generator, self.mpd, self.msd)
        return self._out

    def end_epoch(self):
        """Per-epoch ExponentialLR decay (scripts/hifigan/config.json lr_decay); with graphed=True
        the learning rates are device tensors the captured AdamW steps read."""
        self.sched_g.step()
        self.sched_d.step()
