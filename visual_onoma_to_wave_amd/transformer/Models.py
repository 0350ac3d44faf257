"""Encoder / Decoder stacks on HIP kernels.

get_sinusoid_encoding_table <- scripts/transformer/Models.py:13-33 (float64 -> fp32, so the
                               frozen ``position_enc`` parameter is bit-identical)
Encoder <- scripts/transformer/Models.py:36-126 (visual-glyph branch: VFE + PE -> 4 FFT blocks)
Decoder <- scripts/transformer/Models.py:129-197 (PE add, max_seq_len truncation, 6 FFT blocks)
"""

import json
import os

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .._base import HipModule
from ..utils.symbols import get_symbols
from . import Constants
from .Layers import FFTBlock
from .SubLayers import lens_from_mask


def get_sinusoid_encoding_table(n_position, d_hid, padding_idx=None):
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    exponent = 2 * (np.arange(d_hid) // 2) / d_hid
    table = pos / np.power(10000, exponent)[None, :]
    table[:, 0::2] = np.sin(table[:, 0::2])
    table[:, 1::2] = np.cos(table[:, 1::2])
    if padding_idx is not None:
        table[padding_idx] = 0.0
    return torch.FloatTensor(table)


def _fft_stack(cfg, prefix, n_layers):
    t = cfg["transformer"]
    d_model = t[prefix + "_hidden"]
    n_head = t[prefix + "_head"]
    d_k = d_model // n_head
    return nn.ModuleList(
        FFTBlock(d_model, n_head, d_k, d_k, t["conv_filter_size"], t["conv_kernel_size"],
                 dropout=t[prefix + "_dropout"])
        for _ in range(n_layers))


class Encoder(HipModule):
    def __init__(self, preprocess_config, model_config):
        super().__init__()
        from ..model.visual_feature_extractor import VisualFeatureExtractor

        t = model_config["transformer"]
        self.input_type = preprocess_config["input_type"]
        self.max_seq_len = model_config["max_seq_len"]
        self.d_model = t["encoder_hidden"]
        n_vocab = len(get_symbols(preprocess_config["path"]["preprocessed"])) + 1
        if self.input_type == "visual-text":
            with open(os.path.join(preprocess_config["path"]["preprocessed"], "visual_text.json")) as f:
                vt = json.load(f)
            vfe = model_config["visual_feature_extractor"]
            self.VisualFeatureExtractor = VisualFeatureExtractor(
                load_scale=preprocess_config["visual_text"]["scale_in_training"],
                slice_width=vt["max_pixelsize"][0], slice_height=vt["height"][0],
                embed_dim=self.d_model, embed_normalize=True, bridge_relu=True,
                kernel_size=vfe["conv_kernel_size"], num_convolutions=vfe["layer_num"],
                stride=preprocess_config["visual_text"]["stride"])
        self.src_word_emb = nn.Embedding(n_vocab, self.d_model, padding_idx=Constants.PAD)
        self.position_enc = nn.Parameter(
            get_sinusoid_encoding_table(self.max_seq_len + 1, self.d_model).unsqueeze(0),
            requires_grad=False)
        self.layer_stack = _fft_stack(model_config, "encoder", t["encoder_layer"])

    def run(self, src_seq, lens, images=None, use_image=True):
        """-> (B, T, D) in the compute dtype; lens (B,) int32."""
        B, T = src_seq.shape
        pe = self.position_enc.detach()[0].float().contiguous()
        if use_image:
            x = self.VisualFeatureExtractor.run(images, out_dtype=self.compute_dtype)
            if x.shape[1] != T:
                raise ValueError(f"image holds {x.shape[1]} glyph slices but max_src_len is {T}")
            ops.add_pos_class(x, pe=pe)
        else:
            x = torch.zeros((B, T, self.d_model), dtype=self.compute_dtype, device=src_seq.device)
            ops.add_pos_class(x, pe=pe, cls=self.src_word_emb.weight.detach().float().contiguous(),
                              cls_idx=src_seq.contiguous(), per_token=True)
        for layer in self.layer_stack:
            x = layer.run(x, lens)
        return x

    def train_run(self, src_seq, lens, images=None, use_image=True):
        B, T = src_seq.shape
        pe = self.position_enc[0, :T].to(self.compute_dtype)
        if use_image:
            x = self.VisualFeatureExtractor.train_run(images, self.compute_dtype)
        else:
            x = self.src_word_emb(src_seq).to(self.compute_dtype)
        x = (x + pe[None]).contiguous()
        for layer in self.layer_stack:
            x, _ = layer.train_run(x, lens)
        return x

    def forward(self, src_seq, mask, return_attns=False, images=None, use_image=True):
        self._check_inference()
        return self.run(src_seq, lens_from_mask(mask), images, use_image)


class Decoder(HipModule):
    def __init__(self, config):
        super().__init__()
        t = config["transformer"]
        self.max_seq_len = config["max_seq_len"]
        self.d_model = t["decoder_hidden"]
        self.position_enc = nn.Parameter(
            get_sinusoid_encoding_table(self.max_seq_len + 1, self.d_model).unsqueeze(0),
            requires_grad=False)
        self.layer_stack = _fft_stack(config, "decoder", t["decoder_layer"])
        for layer in self.layer_stack:  # bench.py's C2 roofline: the decoder FFN's k = 9 conv
            layer.pos_ffn.timer_tag = "dec_ffn_w1"

    ln_bf16_copy = True  # mixed precision: LayerNorms hand the next conv a bf16 copy (bit-identical; A/B)

    def run(self, x, mask, lens):
        """x (B, T, D) compute dtype (consumed in place for the PE add) -> (out, mask)."""
        B, T, D = x.shape
        if not self.training and T > self.max_seq_len:
            pe = get_sinusoid_encoding_table(T, D).to(x.device).contiguous()
        else:
            T = min(T, self.max_seq_len)
            pe = self.position_enc.detach()[0].float().contiguous()
            if x.shape[1] != T:
                x = x[:, :T].contiguous()
            mask = mask[:, :T]  # lens past T mask nothing inside [0, T): no clamp needed
        ops.add_pos_class(x, pe=pe)
        # mixed precision (fp32 residual stream, bf16 convs): each LayerNorm also writes the bf16
        # copy the next conv reads (vo_layernorm_dual), the last one only the fp32 output
        dual = self.ln_bf16_copy and x.dtype == torch.float32 and self.compute_dtype == torch.bfloat16
        x16 = None
        n = len(self.layer_stack)
        for i, layer in enumerate(self.layer_stack):
            if dual and i + 1 < n:
                x, x16 = layer.run(x, lens, x16=x16, want16=True)
            else:
                x = layer.run(x, lens, x16=x16)
        return x, mask

    def train_run(self, x, mask, lens):
        B, T, D = x.shape
        T = min(T, self.max_seq_len)
        x = (x[:, :T] + self.position_enc[0, :T].to(x.dtype)[None]).contiguous()
        mask = mask[:, :T]
        x16 = None
        for layer in self.layer_stack:
            x, x16 = layer.train_run(x, lens, x16)
        # mixed: the fp32 stream's bf16 copy is what mel_linear reads (its forward operand and saved input)
        return (x16 if x16 is not None else x), mask

    def forward(self, enc_seq, mask, return_attns=False):
        self._check_inference()
        x = enc_seq.to(self.compute_dtype).contiguous().clone()
        return self.run(x, mask, lens_from_mask(mask))
