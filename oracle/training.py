"""ORACLE (test infrastructure only) -- FastSpeech2 loss and LR schedule restated."""

import numpy as np
import torch


def fastspeech2_loss(inputs, predictions):
    """FastSpeech2Loss.forward, scripts/model/loss.py:15-87 -> 6-tuple
    (total, mel, postnet_mel, energy, kurtosis, duration)."""
    (mel_t, _mel_lens, _max_mel_len, e_t, k_t, d_t, _images, _ev) = inputs[5:]
    (mel_p, post_p, e_p, k_p, logd_p, _, src_masks, mel_masks, _, _) = predictions
    src_m = ~src_masks
    mel_m = ~mel_masks
    logd_t = torch.log(d_t.float() + 1)
    mel_t = mel_t[:, : mel_m.shape[1], :]
    mel_loss = (mel_p.masked_select(mel_m[..., None]) -
                mel_t.masked_select(mel_m[..., None])).abs().mean()
    post_loss = (post_p.masked_select(mel_m[..., None]) -
                 mel_t.masked_select(mel_m[..., None])).abs().mean()
    if e_t is not None:
        e_loss = ((e_p.masked_select(src_m) - e_t.masked_select(src_m)) ** 2).mean()
    else:
        e_loss = torch.tensor(0.0)
    k_loss = torch.tensor(0.0)
    d_loss = ((logd_p.masked_select(src_m) - logd_t.masked_select(src_m)) ** 2).mean()
    total = mel_loss + post_loss + d_loss + e_loss + k_loss
    return total, mel_loss, post_loss, e_loss, k_loss, d_loss


def lr_at(step, init_lr=1e-3, warmup=4000, anneal_steps=(300000, 400000, 500000), rate=0.3):
    """ScheduledOptim._get_lr_scale/_update_learning_rate, scripts/model/optimizer.py:33-51,
    evaluated for the step counter value AFTER the increment."""
    lr = np.min([np.power(step, -0.5), np.power(warmup, -1.5) * step])
    for s in anneal_steps:
        if step > s:
            lr = lr * rate
    return init_lr * lr
