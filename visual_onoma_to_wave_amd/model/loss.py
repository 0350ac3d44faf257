"""FastSpeech2 loss (reference: scripts/model/loss.py:7-87).

Masked L1 on the mel and PostNet mel, MSE on log(d + 1) durations, MSE on energy (and
kurtosis when conditioned); returns the reference's 6-tuple (total, mel, postnet_mel,
energy, kurtosis, duration).  The reductions run as PyTorch-ROCm ops on the device (a few
kB of scalars per step).
"""

import torch
import torch.nn as nn


def _masked_mean(x, mask):
    m = mask.to(x.dtype)
    return (x * m).sum() / m.sum()


class FastSpeech2Loss(nn.Module):
    def __init__(self):
        super().__init__()

    def forward(self, inputs, predictions):
        (mel_t, _mel_lens, _max_mel_len, e_t, k_t, d_t, _images, _ev) = inputs[5:]
        (mel_p, post_p, e_p, k_p, logd_p, _, src_masks, mel_masks, _, _) = predictions
        src_m = ~src_masks
        mel_m = ~mel_masks
        logd_t = torch.log(d_t.float() + 1).detach()
        mel_t = mel_t[:, : mel_m.shape[1], :].detach()
        mm = mel_m[..., None].expand_as(mel_p)
        mel_loss = _masked_mean((mel_p - mel_t).abs(), mm)
        post_loss = _masked_mean((post_p - mel_t).abs(), mm)
        zero = torch.zeros((), device=mel_p.device)
        e_loss = _masked_mean((e_p - e_t.detach()) ** 2, src_m) if e_t is not None else zero
        k_loss = _masked_mean((k_p - k_t.detach()) ** 2, src_m) if (k_t is not None and k_p is not None) else zero
        d_loss = _masked_mean((logd_p - logd_t) ** 2, src_m)
        total = mel_loss + post_loss + d_loss + e_loss + k_loss
        return total, mel_loss, post_loss, e_loss, k_loss, d_loss
