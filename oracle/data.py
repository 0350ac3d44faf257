"""ORACLE (test infrastructure only) -- the reference's glyph batch layout restated in numpy.

character_padding  <- Dataset.character_padding_forinput, scripts/dataset.py:71-92
pad_2D_gray_image  <- scripts/utils/tools.py:616-635
to_tensor          <- transforms.ToTensor in to_device, scripts/utils/tools.py:18-20,50-51
(cv2.hconcat of equal-height uint8 arrays == np.concatenate(axis=1).)  Pinned by construction
against the reference's own numpy calls; the reference itself cannot run here (cv2 absent).
"""

import numpy as np


def character_padding(img, img_length, width):
    cols, w = [], 0
    for L in img_length:
        L = int(L)
        ext = img[:, w:w + L]
        pleft = int(int((width - L) / 2) + (width - L) % 2)
        pright = int((width - L) / 2)
        cols.append(np.pad(ext, [(0, 0), (pleft, pright)], mode="constant", constant_values=255))
        w += L
    return np.concatenate(cols, axis=1)


def pad_2D_gray_image(inputs, width, stride):
    max_len = max(np.shape(x)[1] for x in inputs)
    out = np.stack([np.pad(x, [(0, 0), (0, max_len - np.shape(x)[1])], mode="constant", constant_values=255)
                    for x in inputs])
    each = (stride // 2) * width
    return np.stack([np.pad(x, [(0, 0), (each, each)], mode="constant", constant_values=255) for x in out])


def to_tensor(batch):
    """(B, H, W) uint8 -> (B, 1, H, W) float32 / 255 (torchvision ToTensor: float division)."""
    return (batch.astype(np.float32) / np.float32(255.0))[:, None]


def glyph_batch(strips, widths, width, stride):
    return to_tensor(pad_2D_gray_image([character_padding(s, w, width) for s, w in zip(strips, widths)], width,
                                       stride))
