"""Variance adaptor on HIP kernels.

VarianceAdaptor   <- scripts/model/modules.py:16-124
LengthRegulator   <- scripts/model/modules.py:126-159 (+ utils/tools.py:669-687 pad)
VariancePredictor <- scripts/model/modules.py:161-213
Conv              <- scripts/model/modules.py:216-259

The adaptor keeps the reference's decisions (bucketize of the energy, rounding of the
predicted durations) in fp32 inside the head kernel; the LengthRegulator runs as one
device-side scan + gather, so the only host synchronisation left is reading the total
mel length when the caller does not give ``max_len`` (the output shape depends on it).
"""

import json
import os
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn

import torch.nn.functional as F

from .. import autograd as AG
from .. import ops
from .._base import HipModule
from ..transformer.SubLayers import lens_from_mask


class Conv(nn.Module):
    """Parameter holder: ``conv`` = nn.Conv1d applied to (B, T, C) activations."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=0, dilation=1,
                 bias=True, w_init="linear"):
        super().__init__()
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                              padding=padding, dilation=dilation, bias=bias)


class VariancePredictor(HipModule):
    def __init__(self, model_config):
        super().__init__()
        d_in = model_config["transformer"]["encoder_hidden"]
        vp = model_config["variance_predictor"]
        f, k = vp["filter_size"], vp["kernel_size"]
        self.input_size, self.filter_size, self.kernel, self.conv_output_size = d_in, f, k, f
        self.dropout = vp["dropout"]
        self.conv_layer = nn.Sequential(OrderedDict([
            ("conv1d_1", Conv(d_in, f, kernel_size=k, padding=(k - 1) // 2)),
            ("relu_1", nn.ReLU()),
            ("layer_norm_1", nn.LayerNorm(f)),
            ("dropout_1", nn.Dropout(self.dropout)),
            ("conv1d_2", Conv(f, f, kernel_size=k, padding=1)),
            ("relu_2", nn.ReLU()),
            ("layer_norm_2", nn.LayerNorm(f)),
            ("dropout_2", nn.Dropout(self.dropout)),
        ]))
        self.linear_layer = nn.Linear(f, 1)

    def _build(self, device, dtype):
        c = self.conv_layer

        def f32(t):
            return t.detach().float().to(device).contiguous()

        return dict(
            w1=ops.pack_conv_weight(c.conv1d_1.conv.weight.to(device), dtype), b1=f32(c.conv1d_1.conv.bias),
            g1=f32(c.layer_norm_1.weight), be1=f32(c.layer_norm_1.bias),
            w2=ops.pack_conv_weight(c.conv1d_2.conv.weight.to(device), dtype), b2=f32(c.conv1d_2.conv.bias),
            g2=f32(c.layer_norm_2.weight), be2=f32(c.layer_norm_2.bias),
            lw=f32(self.linear_layer.weight.reshape(-1)), lb=float(self.linear_layer.bias.detach().float().cpu()),
        )

    def hidden(self, x):
        """conv -> relu -> LN -> conv -> relu -> LN over (B, T, D) -> (B, T, filter)."""
        p = self._packed(x.device, self._build)
        k = self.kernel
        h = ops.conv1d(x, p["w1"], p["b1"], Co=self.filter_size, K=k, pad=(k - 1) // 2,
                       post_act=ops.ACT_RELU, compute_dtype=self.compute_dtype, out_dtype=self.compute_dtype)
        h = ops.layernorm(h, p["g1"], p["be1"])
        h = ops.conv1d(h, p["w2"], p["b2"], Co=self.filter_size, K=k, pad=1, post_act=ops.ACT_RELU,
                       compute_dtype=self.compute_dtype, out_dtype=self.compute_dtype)
        return ops.layernorm(h, p["g2"], p["be2"]), p

    def train_run(self, x, mask):
        c, cd, k = self.conv_layer, self.contract_dtype, self.kernel
        h = AG.conv1d(x, c.conv1d_1.conv.weight, c.conv1d_1.conv.bias, K=k, pad=(k - 1) // 2, relu=True,
                      compute_dtype=cd)
        h = AG.dropout(AG.layernorm(h, None, c.layer_norm_1.weight, c.layer_norm_1.bias), self.dropout)
        h = AG.conv1d(h, c.conv1d_2.conv.weight, c.conv1d_2.conv.bias, K=k, pad=1, relu=True, compute_dtype=cd)
        h = AG.dropout(AG.layernorm(h, None, c.layer_norm_2.weight, c.layer_norm_2.bias), self.dropout)
        out = F.linear(h.float(), self.linear_layer.weight, self.linear_layer.bias).squeeze(-1)
        return out.masked_fill(mask, 0.0) if mask is not None else out

    def forward(self, encoder_output, mask):
        self._check_inference()
        x = encoder_output.to(self.compute_dtype).contiguous()
        h, p = self.hidden(x)
        lens = lens_from_mask(mask) if mask is not None else None
        pred, _ = ops.duration_head(h, p["lw"], p["lb"], lens, want_round=False)
        return pred


class LengthRegulator(nn.Module):
    def LR(self, x, duration, max_len, out_dtype=None):
        if max_len is None:
            mel_len, _ = ops.lr_lengths(duration)
            max_len = int(mel_len.cpu().max()) if mel_len.numel() else 0
        out, mel_len, _ = ops.length_regulate(x.contiguous(), duration, int(max_len), out_dtype=out_dtype)
        return out, mel_len

    def forward(self, x, duration, max_len):
        return self.LR(x, duration, max_len)


class VarianceAdaptor(HipModule):
    def __init__(self, preprocess_config, model_config):
        super().__init__()
        ve = model_config["variance_embedding"]
        self.duration_predictor = VariancePredictor(model_config)
        self.length_regulator = LengthRegulator()
        self.is_energy, self.is_kurtosis = ve["is_energy_condition"], ve["is_kurtosis_condition"]
        if self.is_kurtosis:
            self.kurtosis_predictor = VariancePredictor(model_config)
        if self.is_energy:
            self.energy_predictor = VariancePredictor(model_config)
        for q in (ve["kurtosis_quantization"], ve["energy_quantization"]):
            if q not in ("linear", "log"):
                raise AssertionError(f"quantization {q!r} must be 'linear' or 'log'")
        n_bins = ve["n_bins"]
        with open(os.path.join(preprocess_config["path"]["preprocessed"], "stats.json")) as f:
            stats = json.load(f)
        e_min, e_max, self.energy_mean, self.energy_std = stats["energy"]
        k_min, k_max, self.kurtosis_mean, self.kurtosis_std = stats["kurtosis"]
        d = model_config["transformer"]["encoder_hidden"]

        def bins(lo, hi, mode):
            if mode == "log":
                return torch.exp(torch.linspace(np.log(lo), np.log(hi), n_bins - 1))
            return torch.linspace(lo, hi, n_bins - 1)

        # parameter order follows the reference state dict (kurt_bins, kurt_embedding, energy_*)
        self.kurt_bins = nn.Parameter(bins(k_min, k_max, ve["kurtosis_quantization"]), requires_grad=False)
        self.kurt_embedding = nn.Embedding(n_bins, d)
        self.energy_bins = nn.Parameter(bins(e_min, e_max, ve["energy_quantization"]), requires_grad=False)
        self.energy_embedding = nn.Embedding(n_bins, d)

    def set_compute_dtype(self, dtype, f32_split=False):
        return super().set_compute_dtype(dtype, f32_split)

    def run(self, x, src_lens, max_len=None, e_target=None, k_target=None, d_target=None, e_control=1.0,
            d_control=1.0, out_dtype=None):
        """x (B, T, D) in the compute dtype; src_lens (B,) int32.  x is updated in place
        (energy / kurtosis embedding add) before the length regulator."""
        hd, pd = self.duration_predictor.hidden(x)
        log_d, d_round = ops.duration_head(hd, pd["lw"], pd["lb"], src_lens, d_control=d_control,
                                           want_round=d_target is None)
        e_pred = k_pred = None
        if self.is_energy:
            he, pe = self.energy_predictor.hidden(x)
            e_pred, _ = ops.energy_head(
                he, pe["lw"], pe["lb"], src_lens, x, self.energy_bins.detach().float().contiguous(),
                self.energy_embedding.weight.detach().float().contiguous(), target=e_target,
                mean=self.energy_mean, std=self.energy_std, control=e_control)
        if self.is_kurtosis:
            hk, pk = self.kurtosis_predictor.hidden(x)
            k_pred, _ = ops.energy_head(
                hk, pk["lw"], pk["lb"], src_lens, x, self.kurt_bins.detach().float().contiguous(),
                self.kurt_embedding.weight.detach().float().contiguous(), target=k_target,
                mean=self.kurtosis_mean, std=self.kurtosis_std, control=1.0)
        dur = d_target if d_target is not None else d_round
        out, mel_len = self.length_regulator.LR(x, dur, max_len, out_dtype=out_dtype)
        mel_mask = mel_lens32 = None
        if d_target is None:
            mel_mask, mel_lens32 = ops.mask_from_lengths(mel_len, out.shape[1])
        d_rounded = d_target if d_target is not None else d_round
        return out, e_pred, k_pred, log_d, d_rounded, mel_len, mel_mask, mel_lens32

    def train_run(self, x, src_mask, src_lens, mel_mask, max_len, e_target, k_target, d_target, out_dtype):
        """Teacher-forced training forward (scripts/model/modules.py:79-108)."""
        if d_target is None:
            raise ValueError("training needs duration targets (teacher forcing), as in the reference")
        log_d = self.duration_predictor.train_run(x, src_mask)
        e_pred = k_pred = None
        if self.is_energy:
            e_pred = self.energy_predictor.train_run(x, src_mask)
            x = AG.bucket_embed(x, self.energy_embedding, e_target, self.energy_bins)
        if self.is_kurtosis:
            k_pred = self.kurtosis_predictor.train_run(x, src_mask)
            x = AG.bucket_embed(x, self.kurt_embedding, k_target, self.kurt_bins)
        if max_len is None:
            mel_len, _ = ops.lr_lengths(d_target)
            max_len = int(mel_len.cpu().max())
        out, mel_len = AG.length_regulate(x, d_target, max_len, out_dtype=out_dtype)
        return out, e_pred, k_pred, log_d, d_target, mel_len, mel_mask

    def forward(self, x, src_mask, mel_mask=None, max_len=None, energy_target=None, kurtosis_target=None,
                duration_target=None, e_control=1.0, d_control=1.0):
        self._check_inference()
        x = x.to(self.compute_dtype).contiguous().clone()
        out, e, k, log_d, d_r, mel_len, mm, _ = self.run(
            x, lens_from_mask(src_mask), max_len, energy_target, kurtosis_target, duration_target,
            e_control, d_control)
        return out, e, k, log_d, d_r, mel_len, (mm if duration_target is None else mel_mask)
