"""Factories and the vocoder wrapper -- the drop-in boundary callers use
(reference: scripts/utils/model.py:10-98).

get_model(restore_step, configs, device, train=False)
get_vocoder(config, device)
vocoder_infer(mels, vocoder, model_config, preprocess_config, lengths=None, Normalize=True)
"""

import json
import os

import numpy as np
import torch

from .. import hifigan
from ..model import ScheduledOptim, vTTS

_PKG_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def get_model(restore_step, configs, device, train=False):
    preprocess_config, model_config, train_config = configs
    model = vTTS(preprocess_config, model_config, train_config).to(device)
    ckpt = None
    if restore_step:
        path = os.path.join(train_config["path"]["ckpt_path"], f"{restore_step}.pth.tar")
        ckpt = torch.load(path, map_location=device, weights_only=True)
        model.load_state_dict(ckpt["model"])
    if train:
        optim = ScheduledOptim(model, train_config, model_config, restore_step)
        if restore_step:
            optim.load_state_dict(ckpt["optimizer"])
        model.train()
        return model, optim
    model.eval()
    model.requires_grad_ = False
    return model


def get_param_num(model):
    return sum(p.numel() for p in model.parameters())


def _hifigan_config():
    for path in ("scripts/hifigan/config.json", os.path.join(_PKG_DATA, "hifigan_config.json")):
        if os.path.exists(path):
            with open(path) as f:
                return json.load(f)
    raise FileNotFoundError("hifigan config.json not found")


def get_vocoder(config, device, checkpoint=None):
    """HiFi-GAN generator with weight norm folded.  ``checkpoint`` overrides the
    reference's cwd-relative ``scripts/hifigan/generator_<speaker>.pth.tar``; the MelGAN
    branch of the reference is a remote torch.hub fetch and is not available offline."""
    name, speaker = config["vocoder"]["model"], config["vocoder"]["speaker"]
    if name != "HiFi-GAN":
        raise NotImplementedError(f"vocoder {name!r}: only HiFi-GAN is on the HIP path (MelGAN is a "
                                  "remote torch.hub model)")
    vocoder = hifigan.Generator(hifigan.AttrDict(_hifigan_config()))
    path = checkpoint or {"LJSpeech": "scripts/hifigan/generator_LJSpeech.pth.tar",
                          "universal": "scripts/hifigan/generator_universal.pth.tar"}[speaker]
    # a missing checkpoint raises, as torch.load does in the reference (utils/model.py:64-67):
    # never synthesise with random weights
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    vocoder.load_state_dict(ckpt["generator"])
    vocoder.eval()
    vocoder.remove_weight_norm()
    return vocoder.to(device)


def vocoder_infer(mels, vocoder, model_config, preprocess_config, lengths=None, Normalize=True):
    name = model_config["vocoder"]["model"]
    with torch.no_grad():
        if name != "HiFi-GAN":
            raise NotImplementedError(name)
        wavs = vocoder(mels).squeeze(1)
    wavs = wavs.cpu().numpy()
    if Normalize:
        # the reference reads preprocess_config["preprocessing"]["audio"]["max_wav_value"]
        # (a key the ICASSP config does not have); accept both layouts
        audio = preprocess_config.get("preprocessing", preprocess_config)["audio"]
        wavs = (wavs * audio["max_wav_value"]).astype("int16")
    wavs = [w for w in wavs]
    if lengths is not None:
        for i in range(len(mels)):
            wavs[i] = wavs[i][: lengths[i]]
    return wavs


def __getattr__(name):
    """Names the build does not provide come from the caller's own ``scripts/utils/model.py``
    (see ``compat``)."""
    from .. import compat
    return compat.caller_attr("utils.model", name)
