"""FastSpeech2 loss (reference: scripts/model/loss.py:7-87) -- placeholder until the
training path lands; see visual_onoma_to_wave_amd.train."""

import torch.nn as nn


class FastSpeech2Loss(nn.Module):
    def forward(self, inputs, predictions):
        raise NotImplementedError("FastSpeech2Loss lands with the training path")
