"""Training input pipeline: the Dataset / collate_fn mirror of
scripts/dataset.py on a synthetic preprocessed directory, and the on-GPU glyph layout
(vo_glyph_batch) bit-exact against the reference's numpy layout (oracle/data.py)."""

import json
import os

import numpy as np
import pytest
import torch

from helpers import configs


def _make_corpus(root, n=10, seed=0, cell=102, H=24):
    from PIL import Image
    rng = np.random.default_rng(seed)
    p = root
    chars = "アイウエオカキクケコ"
    lines = []
    for d in ("mel", "energy", "duration", "image/width", "image/png"):
        os.makedirs(os.path.join(p, d, "bells5"), exist_ok=True)
    for i in range(n):
        L = int(rng.integers(2, 7))
        text = "".join(rng.choice(list(chars), L))
        widths = rng.integers(30, cell + 1, L).astype(np.int32)
        strip = rng.integers(0, 256, (H, int(widths.sum()))).astype(np.uint8)
        dur = rng.integers(1, 6, L)
        T = int(dur.sum())
        name = f"utt{i:03d}"
        np.save(os.path.join(p, "mel", "bells5", name + ".npy"), rng.standard_normal((T, 80)).astype(np.float32))
        np.save(os.path.join(p, "energy", "bells5", name + ".npy"), rng.standard_normal(L).astype(np.float32))
        np.save(os.path.join(p, "duration", "bells5", name + ".npy"), dur)
        np.save(os.path.join(p, "image", "width", "bells5", name + ".npy"), widths)
        Image.fromarray(strip, "L").save(os.path.join(p, "image", "png", "bells5", name + ".png"))
        lines.append(f"{name}|bells5|24|ipaexg|{text}")
    for f in ("train.txt", "val.txt", "test.txt"):
        with open(os.path.join(p, f), "w", encoding="utf-8") as fh:
            fh.write("\n".join(lines) + "\n")
    with open(os.path.join(p, "visual_text.json"), "w") as fh:
        json.dump({"max_pixelsize": [cell], "height": [H]}, fh)
    with open(os.path.join(p, "audiotype.json"), "w") as fh:
        json.dump({"bells5": 9}, fh)


def _dataset(tmp_path, batch=4):
    from visual_onoma_to_wave_amd.dataset import Dataset
    _make_corpus(str(tmp_path))
    pc, mc, tc = configs()
    pc = dict(pc, path=dict(pc["path"], preprocessed=str(tmp_path)))
    tc = dict(tc, optimizer=dict(tc["optimizer"], batch_size=batch))
    return Dataset("train.txt", pc, tc, mc, sort=True, drop_last=False)


def test_dataset_collate_mirrors_reference(tmp_path):
    from oracle import data as O
    from visual_onoma_to_wave_amd.dataset import GlyphBatch
    ds = _dataset(tmp_path)
    items = [ds[i] for i in range(len(ds))]
    batches = ds.collate_fn(items)
    assert [len(b[0]) for b in batches] == [4, 4, 2]  # batch_size groups + tail (drop_last=False)
    for b in batches:
        (ids, at, texts, src_lens, max_src, mels, mel_lens, max_mel, e, k, d, images, ev) = b
        assert list(src_lens) == sorted(src_lens, reverse=True)  # sort=True: longest first
        assert texts.shape == (len(ids), max_src) and mels.shape == (len(ids), max_mel, 80)
        assert isinstance(images, GlyphBatch) and len(images) == len(ids)
        ref = O.glyph_batch(images.strips, images.char_widths, 102, 1)
        assert ref.shape == (len(ids), 1, 24, 102 * max_src)
        assert (at == 9).all() and k is None


@pytest.mark.gpu
def test_glyph_batch_on_gpu_bit_exact(tmp_path):
    from oracle import data as O
    from visual_onoma_to_wave_amd.utils.tools import to_device
    ds = _dataset(tmp_path)
    for b in ds.collate_fn([ds[i] for i in range(len(ds))]):
        ref = O.glyph_batch(b[11].strips, b[11].char_widths, 102, 1)
        out = to_device(b, torch.device("cuda"))
        assert out[11].shape == ref.shape
        assert np.array_equal(out[11].cpu().numpy(), ref)
    # margins (stride 3 -> one cell each side) and already-padded uint8 batches
    g = b[11]
    g.stride = 3
    assert np.array_equal(g.to("cuda").cpu().numpy(), O.glyph_batch(g.strips, g.char_widths, 102, 3))
    padded = O.pad_2D_gray_image([O.character_padding(s, w, 102) for s, w in zip(g.strips, g.char_widths)], 102, 1)
    out = to_device(b[:11] + (list(padded), b[12]), torch.device("cuda"))
    assert np.array_equal(out[11].cpu().numpy(), O.to_tensor(padded))
