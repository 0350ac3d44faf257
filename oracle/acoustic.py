"""ORACLE (test infrastructure only) -- acoustic model restated on the CPU.

Pure functions over a reference-layout state dict ``sd`` ({key: torch.Tensor}),
fp32 PyTorch-CPU ops for the dense math and numpy for the index math.  Citations
are reference file:line (``scripts/...``).
"""

import math

import numpy as np
import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- helpers

def sinusoid_table(n_position, d_hid):
    """scripts/transformer/Models.py:13-33 -- computed in float64, cast to fp32."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    j = np.arange(d_hid)
    angle = pos / np.power(10000, 2 * (j // 2) / d_hid)
    tab = angle.copy()
    tab[:, 0::2] = np.sin(angle[:, 0::2])
    tab[:, 1::2] = np.cos(angle[:, 1::2])
    return torch.from_numpy(tab.astype(np.float32))


def mask_from_lengths(lengths, max_len=None):
    """scripts/utils/tools.py:164-171 -- True marks padding."""
    lengths = torch.as_tensor(lengths)
    if max_len is None:
        max_len = int(lengths.max().item())
    ids = torch.arange(max_len)[None, :]
    return ids >= lengths[:, None]


def energy_bins(stats_energy, n_bins=256, log=False):
    """scripts/model/modules.py:32-50 -- linspace(min, max, n_bins-1) (fp32 linspace)."""
    lo, hi = stats_energy[0], stats_energy[1]
    if log:
        return torch.exp(torch.linspace(np.log(lo), np.log(hi), n_bins - 1))
    return torch.linspace(lo, hi, n_bins - 1)


def bucketize(values, bins):
    """torch.bucketize(right=False) as used at scripts/model/modules.py:56,62:
    index i with bins[i-1] < v <= bins[i]  ==  number of bins strictly below v."""
    v = np.asarray(values, dtype=np.float32)
    b = np.asarray(bins, dtype=np.float32)
    return np.searchsorted(b, v, side="left").astype(np.int64)


def length_regulate(x, durations, max_len=None):
    """LengthRegulator.LR/expand, scripts/model/modules.py:132-159 + pad, utils/tools.py:669-687.

    Row j of batch b is repeated max(int(d[b, j]), 0) times (int() truncates toward
    zero); rows are concatenated, then zero-padded (or CROPPED, if the expanded
    length exceeds max_len: F.pad with a negative amount) to max_len, or to the
    longest expansion when max_len is None.  Returns (out, mel_len int64, index)
    where index[b, t] is the source token of frame t (-1 on padding).
    """
    x = torch.as_tensor(x)
    d = np.asarray(durations, dtype=np.float32)
    B, T = d.shape
    reps = np.maximum(np.trunc(d).astype(np.int64), 0)
    mel_len = reps.sum(axis=1)
    L = int(max_len) if max_len is not None else int(mel_len.max())
    index = np.full((B, L), -1, dtype=np.int64)
    for b in range(B):
        src = np.repeat(np.arange(T), reps[b])[:L]
        index[b, : len(src)] = src
    out = torch.zeros((B, L) + tuple(x.shape[2:]), dtype=x.dtype)
    for b in range(B):
        valid = index[b] >= 0
        out[b, torch.from_numpy(valid)] = x[b, torch.from_numpy(index[b][valid])]
    return out, torch.from_numpy(mel_len), index


def conv1d_bct(x_btc, w, b, pad, dilation=1):
    """Conv1d applied to a (B, T, C) tensor the way the reference transposes around it."""
    y = F.conv1d(x_btc.transpose(1, 2), w, b, padding=pad, dilation=dilation)
    return y.transpose(1, 2)


def layer_norm(x, sd, p, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def linear(x, sd, p):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"])


def batch_norm_eval(x, sd, p, eps=1e-5, training=False):
    """BatchNorm; training=True normalises with batch statistics (train-mode forward) without
    touching the running stats of ``sd``."""
    if training:
        return F.batch_norm(x, None, None, sd[p + ".weight"], sd[p + ".bias"], True, 0.0, eps)
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], False, 0.0, eps)


# ----------------------------------------------------------------------------- modules

def vfe(sd, images, p="encoder.VisualFeatureExtractor", slice_w=102, stride=1, n_conv=3, training=False):
    """VisualFeatureExtractor.forward, scripts/model/visual_feature_extractor.py:60-83.

    Slices i*W .. i*W + W*stride of the image width, for i < (width - (stride//2)*W*2)/W,
    then per slice 3 x [Conv2d 3x3 pad 1 -> BatchNorm2d(eval) -> ReLU], flatten
    (h*w), Linear(2448 -> 256) + ReLU.
    """
    B, C, H, W = images.shape
    n = int((W - (stride // 2) * slice_w * 2) / slice_w)
    sl = torch.stack([images[:, :, :, i * slice_w: i * slice_w + slice_w * stride]
                      for i in range(n)], dim=1)
    x = sl.reshape(B * n, C, H, slice_w * stride)
    for i in range(n_conv):
        x = F.conv2d(x, sd[f"{p}.embedder.{3 * i}.weight"], sd[f"{p}.embedder.{3 * i}.bias"],
                     padding=1)
        x = batch_norm_eval(x, sd, f"{p}.embedder.{3 * i + 1}", training=training)
        x = F.relu(x)
    x = x.reshape(B * n, -1)
    x = F.relu(linear(x, sd, f"{p}.bridge.0"))
    return x.reshape(B, n, -1)


def mha(sd, p, x, key_pad_mask, n_head=2):
    """MultiHeadAttention.forward (scripts/transformer/SubLayers.py:29-57) +
    ScaledDotProductAttention (scripts/transformer/Modules.py:14-25).
    Heads are batched head-major (n*b); masked keys get -inf before softmax(dim=2);
    post-LN over fc(out) + residual.  Returns (out, attn probs (n*b, L, L))."""
    B, L, D = x.shape
    dk = D // n_head
    q = linear(x, sd, p + ".w_qs").view(B, L, n_head, dk).permute(2, 0, 1, 3).reshape(-1, L, dk)
    k = linear(x, sd, p + ".w_ks").view(B, L, n_head, dk).permute(2, 0, 1, 3).reshape(-1, L, dk)
    v = linear(x, sd, p + ".w_vs").view(B, L, n_head, dk).permute(2, 0, 1, 3).reshape(-1, L, dk)
    m = key_pad_mask[:, None, :].expand(-1, L, -1).repeat(n_head, 1, 1)
    s = torch.bmm(q, k.transpose(1, 2)) / float(np.power(dk, 0.5))
    s = s.masked_fill(m, -np.inf)
    a = torch.softmax(s, dim=2)
    o = torch.bmm(a, v).view(n_head, B, L, dk).permute(1, 2, 0, 3).reshape(B, L, -1)
    o = linear(o, sd, p + ".fc")
    return layer_norm(o + x, sd, p + ".layer_norm"), a


def pwffn(sd, p, x, k1=9, k2=1):
    """PositionwiseFeedForward.forward, scripts/transformer/SubLayers.py:85-93."""
    h = F.relu(conv1d_bct(x, sd[p + ".w_1.weight"], sd[p + ".w_1.bias"], (k1 - 1) // 2))
    h = conv1d_bct(h, sd[p + ".w_2.weight"], sd[p + ".w_2.bias"], (k2 - 1) // 2)
    return layer_norm(h + x, sd, p + ".layer_norm")


def fft_block(sd, p, x, pad_mask):
    """FFTBlock.forward, scripts/transformer/Layers.py:21-30."""
    y, attn = mha(sd, p + ".slf_attn", x, pad_mask)
    y = y.masked_fill(pad_mask[..., None], 0)
    y = pwffn(sd, p + ".pos_ffn", y)
    return y.masked_fill(pad_mask[..., None], 0), attn


def encoder(sd, images, src_mask, n_layers=4, training=False):
    """Encoder.forward (use_image branch), scripts/transformer/Models.py:99-126."""
    B, T = src_mask.shape
    x = vfe(sd, images, training=training) + sd["encoder.position_enc"][:, :T, :]
    for i in range(n_layers):
        x, _ = fft_block(sd, f"encoder.layer_stack.{i}", x, src_mask)
    return x


def decoder(sd, x, mel_mask, n_layers=6, max_seq_len=1000, training=False):
    """Decoder.forward, scripts/transformer/Models.py:165-197."""
    B, L, D = x.shape
    if not training and L > max_seq_len:
        x = x + sinusoid_table(L, D)[None, :L]
    else:
        L = min(L, max_seq_len)
        x = x[:, :L] + sd["decoder.position_enc"][:, :L, :]
        mel_mask = mel_mask[:, :L]
    for i in range(n_layers):
        x, _ = fft_block(sd, f"decoder.layer_stack.{i}", x, mel_mask)
    return x, mel_mask


def variance_predictor(sd, p, x, pad_mask, k=3):
    """VariancePredictor.forward + Conv, scripts/model/modules.py:161-259."""
    h = conv1d_bct(x, sd[p + ".conv_layer.conv1d_1.conv.weight"],
                   sd[p + ".conv_layer.conv1d_1.conv.bias"], (k - 1) // 2)
    h = layer_norm(F.relu(h), sd, p + ".conv_layer.layer_norm_1")
    h = conv1d_bct(h, sd[p + ".conv_layer.conv1d_2.conv.weight"],
                   sd[p + ".conv_layer.conv1d_2.conv.bias"], 1)
    h = layer_norm(F.relu(h), sd, p + ".conv_layer.layer_norm_2")
    out = linear(h, sd, p + ".linear_layer").squeeze(-1)
    if pad_mask is not None:
        out = out.masked_fill(pad_mask, 0.0)
    return out


def variance_adaptor(sd, x, src_mask, mel_mask, max_len, e_target, d_target,
                     e_control, d_control, energy_stats):
    """VarianceAdaptor.forward, scripts/model/modules.py:79-124 (energy on, kurtosis off)."""
    p = "variance_adaptor"
    log_d = variance_predictor(sd, p + ".duration_predictor", x, src_mask)
    e_pred = variance_predictor(sd, p + ".energy_predictor", x, src_mask)
    bins = sd[p + ".energy_bins"]
    if e_target is not None:
        idx = bucketize(e_target, bins)
    else:
        e_mean, e_std = energy_stats[2], energy_stats[3]
        e_pred = e_pred * e_std + e_mean
        e_pred = e_pred * e_control
        e_pred = (e_pred - e_mean) / e_std
        idx = bucketize(e_pred, bins)
    x = x + sd[p + ".energy_embedding.weight"][torch.from_numpy(idx)]
    if d_target is not None:
        x, mel_len, index = length_regulate(x, d_target, max_len)
        d_rounded = torch.as_tensor(d_target)
    else:
        d_rounded = torch.clamp(torch.round(torch.exp(log_d) - 1) * d_control, min=0)
        x, mel_len, index = length_regulate(x, d_rounded, max_len)
        mel_mask = mask_from_lengths(mel_len)
    return x, e_pred, log_d, d_rounded, mel_len, mel_mask, idx, index


def postnet(sd, x, n=5, k=5, training=False):
    """PostNet.forward, scripts/transformer/Layers.py:129-137 (dropout off; BatchNorm with batch
    statistics when training)."""
    y = x.transpose(1, 2)
    for i in range(n):
        p = f"postnet.convolutions.{i}"
        y = F.conv1d(y, sd[p + ".0.conv.weight"], sd[p + ".0.conv.bias"], padding=(k - 1) // 2)
        y = batch_norm_eval(y, sd, p + ".1", training=training)
        if i < n - 1:
            y = torch.tanh(y)
    return y.transpose(1, 2)


def vtts_forward(sd, audiotypes, texts, src_lens, max_src_len, mels=None, mel_lens=None,
                 max_mel_len=None, e_targets=None, k_targets=None, d_targets=None,
                 images=None, event_image_features=None, use_image=True, e_control=1.0,
                 d_control=1.0, energy_stats=None, training=False, bf16_back=False):
    """vTTS.forward, scripts/model/vtts.py:47-119 -> the reference's 10-tuple.

    ``bf16_back``: the decoder, mel_linear and PostNet at bf16 -- the reference's own arithmetic at the
    precision split of the HIP path's "mixed" mode; its distance from the fp32 result is the bf16
    tolerance bar of the parity tests.  True / "autocast": CPU bf16 autocast; "operands": bf16 operands
    of every contraction, fp32 accumulation and fp32 everywhere else (oracle/bf16.py)."""
    assert use_image, "only the visual-text input path is on the hot path"
    src_masks = mask_from_lengths(src_lens, max_src_len)
    mel_masks = mask_from_lengths(mel_lens, max_mel_len) if mels is not None else None
    x = encoder(sd, images, src_masks, training=training)
    x = x + sd["audiotype_emb.weight"][audiotypes][:, None, :]
    x, e_pred, log_d, d_rounded, mel_lens_o, mel_masks, _, _ = variance_adaptor(
        sd, x, src_masks, mel_masks, max_mel_len, e_targets, d_targets, e_control, d_control,
        energy_stats)
    import contextlib
    import sys

    from .bf16 import bf16_operands
    ctx = (bf16_operands(sys.modules[__name__]) if bf16_back == "operands" else
           torch.autocast("cpu", dtype=torch.bfloat16, enabled=bool(bf16_back)) if bf16_back else contextlib.nullcontext())
    with ctx:
        x, mel_masks = decoder(sd, x, mel_masks, training=training)
        mel = linear(x, sd, "mel_linear")
        post = postnet(sd, mel, training=training) + mel
    mel, post = mel.float(), post.float()
    return (mel, post, e_pred, None, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_lens_o)


def complete_state_dict(arrays, stats_energy):
    """Generated arrays + the init-time tensors the modules compute themselves."""
    sd = {k: torch.from_numpy(np.array(v)) for k, v in arrays.items()}
    pe = sinusoid_table(1001, 256)[None]
    sd["encoder.position_enc"] = pe
    sd["decoder.position_enc"] = pe.clone()
    sd["variance_adaptor.energy_bins"] = energy_bins(stats_energy)
    return sd
