"""Batch / mask / padding helpers on the path (reference: scripts/utils/tools.py).

to_device              <- tools.py:22-72   (the host -> device crossing of a 13-item batch; glyph
                          batches are laid out on the GPU, dataset.GlyphBatch / vo_glyph_batch)
get_mask_from_lengths  <- tools.py:164-171 (HIP kernel; True = padding)
expand                 <- tools.py:173-177
pad_1D / pad_2D / pad_2D_gray_image <- tools.py:585-635 (host-side collate padding)
pad                    <- tools.py:669-687
"""

import numpy as np
import torch

from .. import ops

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _to_tensor_image(im):
    """torchvision ToTensor for an 'L' image / uint8 (H, W) array -> (1, H, W) float / 255."""
    a = np.asarray(im)
    if a.ndim == 2:
        a = a[None]
    elif a.ndim == 3:
        a = a.transpose(2, 0, 1)
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.float().div_(255.0) if t.dtype == torch.uint8 else t.float()


def _images_to_device(images, device):
    """Glyph batches are laid out on the GPU (vo_glyph_batch: per-character centring, white
    padding and ToTensor in one launch); an already padded (B, H, W) uint8 batch (the
    reference's pad_2D_gray_image output) gets the device ToTensor only."""
    from ..dataset import GlyphBatch
    if isinstance(images, GlyphBatch):
        return images.to(device)
    dev = torch.device(device)
    if dev.type == "cuda":
        arr = [np.asarray(im) for im in images]
        if all(a.dtype == np.uint8 and a.ndim == 2 for a in arr):
            return ops.glyph_batch(arr, None, 0, 0, dev)
    return torch.stack([_to_tensor_image(im) for im in images]).to(device)


def to_device(data, device):
    (ids, audiotypes, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len, energies,
     kurtosises, durations, images, event_image_features) = data
    audiotypes = torch.from_numpy(audiotypes).long().to(device)
    src_lens = torch.from_numpy(src_lens).to(device)
    if mels is not None:
        mels = torch.from_numpy(mels).float().to(device)
    if mel_lens is not None:
        mel_lens = torch.from_numpy(mel_lens).float().to(device)
    if energies is not None:
        energies = torch.from_numpy(energies).float().to(device)
    if kurtosises is not None:
        kurtosises = torch.from_numpy(kurtosises).float().to(device)
    if durations is not None:
        durations = torch.from_numpy(durations).float().to(device)
    if images is not None:
        images = _images_to_device(images, device)
    if event_image_features is not None and event_image_features[0] is not None:
        event_image_features = torch.from_numpy(event_image_features).float().to(device)
    else:
        event_image_features = None
    texts = torch.from_numpy(texts).to(device)
    return (ids, audiotypes, texts, src_lens, max_src_len, mels, mel_lens, max_mel_len, energies,
            kurtosises, durations, images, event_image_features)


def get_mask_from_lengths(lengths, max_len=None):
    if max_len is None:
        max_len = int(lengths.detach().cpu().max()) if lengths.numel() else 0
    if not lengths.is_cuda:
        ids = torch.arange(0, max_len, device=lengths.device)[None, :]
        return ids >= lengths[:, None]
    mask, _ = ops.mask_from_lengths(lengths.contiguous(), int(max_len))
    return mask


def expand(values, durations):
    out = []
    for v, d in zip(values, durations):
        out += [v] * max(0, int(d))
    return np.array(out)


def pad_1D(inputs, PAD=0):
    max_len = max(len(x) for x in inputs)
    return np.stack([np.pad(x, (0, max_len - x.shape[0]), mode="constant", constant_values=PAD)
                     for x in inputs])


def pad_2D(inputs, maxlen=None):
    max_len = maxlen or max(np.shape(x)[0] for x in inputs)
    out = []
    for x in inputs:
        if np.shape(x)[0] > max_len:
            raise ValueError("not max_len")
        s = np.shape(x)[1]
        out.append(np.pad(x, (0, max_len - np.shape(x)[0]), mode="constant", constant_values=0)[:, :s])
    return np.stack(out)


def pad_2D_gray_image(inputs, width, stride):
    max_len = max(np.shape(x)[1] for x in inputs)
    margin = (stride // 2) * width
    return np.stack([np.pad(x, [(0, 0), (margin, margin + max_len - np.shape(x)[1])], mode="constant",
                            constant_values=255) for x in inputs])


def pad(input_ele, mel_max_length=None):
    """Host helper kept for API parity; on the device path the LengthRegulator kernel pads."""
    max_len = mel_max_length or max(x.size(0) for x in input_ele)
    out = []
    for x in input_ele:
        n = x.size(0)
        y = x.new_zeros((max_len,) + tuple(x.shape[1:]))
        y[: min(n, max_len)] = x[: min(n, max_len)]
        out.append(y)
    return torch.stack(out)


def __getattr__(name):
    """Names off the synthesis path (``log``, ``synth_one_sample``, ``plot_mel`` ...,
    ``tools.py:140-241,541-582``) come from the caller's own ``scripts/utils/tools.py``
    (see ``compat``)."""
    from .. import compat
    return compat.caller_attr("utils.tools", name)
