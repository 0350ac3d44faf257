"""vTTS acoustic model on HIP kernels (reference: scripts/model/vtts.py:10-119).

forward() keeps the reference's positional signature and 10-tuple result, so
``model(*(batch[1:]), use_image)`` from prediction.ipynb / 04_train.py works unchanged.
"""

import json
import os

import torch
import torch.nn as nn

from .. import ops
from .._base import HipModule
from ..transformer import Decoder, Encoder, PostNet
from .modules import VarianceAdaptor

PRECISIONS = ("mixed", "fp32", "bf16")


class vTTS(HipModule):
    def __init__(self, preprocess_config, model_config, train_config):
        super().__init__()
        self.model_config = model_config
        self.encoder = Encoder(preprocess_config, model_config)
        self.variance_adaptor = VarianceAdaptor(preprocess_config, model_config)
        self.decoder = Decoder(model_config)
        self.mel_linear = nn.Linear(model_config["transformer"]["decoder_hidden"],
                                    preprocess_config["audio"]["mel"]["n_mel_channels"])
        self.postnet = PostNet()
        self.audiotype_emb = None
        if model_config["multi_audiotype"]:
            with open(os.path.join(preprocess_config["path"]["preprocessed"], "audiotype.json")) as f:
                n_types = len(json.load(f))
            self.audiotype_emb = nn.Embedding(n_types, model_config["transformer"]["encoder_hidden"])
        self.set_precision("mixed")

    def set_precision(self, mode, f32_split=True):
        """'mixed' (default): encoder + variance adaptor fp32, decoder / PostNet bf16;
        'fp32': everything exact-f32 MFMA; 'bf16': everything bf16 MFMA.
        f32_split (mixed only): the training step's fp32 contractions (encoder, variance predictors) as
        split-bf16 (ops.F32X3: three bf16 MFMAs per product, ~1e-5 relative per product) instead of exact
        f32 MFMA; inference stays exact fp32."""
        if mode not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}")
        front = torch.bfloat16 if mode == "bf16" else torch.float32
        back = torch.float32 if mode == "fp32" else torch.bfloat16
        self.precision = mode
        self.compute_dtype = back
        # the decoder's residual stream (LengthRegulator output, LayerNorm outputs): fp32 unless
        # everything is bf16 -- bf16 autocast of the reference keeps LayerNorm (and so the
        # residual adds) in fp32, and a bf16 stream doubled the mixed mode's drift from fp32
        self.stream_dtype = torch.bfloat16 if mode == "bf16" else torch.float32
        split = f32_split and mode == "mixed"
        self.f32_split = split
        self.encoder.set_compute_dtype(front, f32_split=split)
        self.variance_adaptor.set_compute_dtype(front, f32_split=split)
        self.decoder.set_compute_dtype(back)
        self.postnet.set_compute_dtype(back)
        return self

    def _build(self, device, dtype):
        return dict(wmel=ops.pack_conv_weight(self.mel_linear.weight.to(device)[:, :, None], dtype),
                    bmel=self.mel_linear.bias.detach().float().to(device).contiguous())

    def forward(self, audiotypes, texts, src_lens, max_src_len, mels=None, mel_lens=None, max_mel_len=None,
                e_targets=None, k_targets=None, d_targets=None, images=None, event_image_features=None,
                use_image=True, e_control=1.0, d_control=1.0):
        if self._training_path():
            return self._train_forward(audiotypes, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len,
                                       e_targets, k_targets, d_targets, images, use_image)
        src_masks, src_l32 = ops.mask_from_lengths(src_lens, max_src_len)
        mel_masks = mel_l32 = None
        if mels is not None:
            mel_masks, mel_l32 = ops.mask_from_lengths(mel_lens, max_mel_len)
        x = self.encoder.run(texts, src_l32, images=images, use_image=use_image)
        if self.audiotype_emb is not None:
            ops.add_pos_class(x, cls=self.audiotype_emb.weight.detach().float().contiguous(),
                              cls_idx=audiotypes)
        (x, e_pred, k_pred, log_d, d_rounded, mel_len, va_mask, va_l32) = self.variance_adaptor.run(
            x, src_l32, max_mel_len, e_targets, k_targets, d_targets, e_control, d_control,
            out_dtype=self.stream_dtype)
        if d_targets is None:
            mel_masks, mel_l32 = va_mask, va_l32
        if mel_masks is None:
            raise ValueError("teacher-forced calls (d_targets given) need mels / mel_lens / max_mel_len "
                             "to build the decoder mask, as in the reference")
        x, mel_masks = self.decoder.run(x, mel_masks, mel_l32)
        p = self._packed(x.device, self._build)
        mel = ops.conv1d(x, p["wmel"], p["bmel"], Co=self.mel_linear.out_features, K=1,
                         out_dtype=torch.float32, compute_dtype=self.compute_dtype)
        post = self.postnet.run(mel, residual=mel, out_dtype=torch.float32)
        return (mel, post, e_pred, k_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_len)

    def _train_forward(self, audiotypes, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len, e_targets,
                       k_targets, d_targets, images, use_image):
        """Training step forward (dropout and BatchNorm batch statistics active; autograd records
        HIP-forward ops, see visual_onoma_to_wave_amd.autograd)."""
        from .. import autograd as AG
        AG.begin_dropout_step(texts.device)  # one device seed for every dropout site of this step
        src_masks, src_l32 = ops.mask_from_lengths(src_lens, max_src_len)
        if mels is None:
            raise ValueError("training needs mels / mel_lens / max_mel_len (teacher forcing)")
        mel_masks, mel_l32 = ops.mask_from_lengths(mel_lens, max_mel_len)
        x = self.encoder.train_run(texts, src_l32, images=images, use_image=use_image)
        if self.audiotype_emb is not None:
            x = x + self.audiotype_emb(audiotypes).to(x.dtype)[:, None, :]
        x, e_pred, k_pred, log_d, d_rounded, mel_len, mel_masks = self.variance_adaptor.train_run(
            x, src_masks, src_l32, mel_masks, max_mel_len, e_targets, k_targets, d_targets,
            out_dtype=self.stream_dtype)
        x, mel_masks = self.decoder.train_run(x, mel_masks, mel_l32)
        mel = AG.linear(x, self.mel_linear.weight, self.mel_linear.bias, compute_dtype=self.compute_dtype,
                        out_dtype=torch.float32)
        post = self.postnet.train_run(mel) + mel
        return (mel, post, e_pred, k_pred, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_len)
