"""Synthetic inputs for the visual-onomatopoeia -> waveform path.

There is no corpus and no pretrained checkpoint offline, so benchmarks and tests
run on procedurally drawn glyph strips of the exact shape the reference feeds the
model (``prediction.ipynb`` cell 5 / ``scripts/dataset.py:71-92``):

* one 24 x 102 gray-scale cell per character, white background (uint8 255),
  black strokes, about 12.5 % ink (the training-sample png in ``sample/``);
* converted the way ``torchvision.transforms.ToTensor`` converts an "L" image
  (``scripts/utils/tools.py:18-19,51``): float32 = uint8 / 255, shape
  (B, 1, 24, 102 * T);
* durations from a seeded multinomial with every d >= 1 and a fixed row sum, so
  the mel length is fixed;
* mel spectrograms ~ clamp(N(-5, 2), log(1e-5), 2.5) (natural-log mels, the
  range ``preprocessor.py:323-337`` produces).
"""

import numpy as np

CELL_H = 24
CELL_W = 102


def glyph_cells(rng, n_cells, ink=0.125):
    """Draw ``n_cells`` 24x102 uint8 glyph cells (255 = paper, 0 = ink)."""
    cells = np.full((n_cells, CELL_H, CELL_W), 255, dtype=np.uint8)
    yy, xx = np.mgrid[0:CELL_H, 0:CELL_W]
    for c in range(n_cells):
        cell = cells[c]
        # a glyph occupies a roughly square box centred in the 102-px cell
        gw = int(rng.integers(14, 30))
        x0 = (CELL_W - gw) // 2 + int(rng.integers(-6, 7))
        target = ink * CELL_H * CELL_W * rng.uniform(0.6, 1.4)
        n_ink = 0
        for _ in range(64):
            if n_ink >= target:
                break
            kind = rng.integers(0, 3)
            t = int(rng.integers(2, 4))  # stroke thickness
            if kind == 0:  # horizontal stroke
                y = int(rng.integers(2, CELL_H - 2 - t))
                xa = x0 + int(rng.integers(0, gw // 2))
                xb = min(CELL_W, xa + int(rng.integers(gw // 3, gw)))
                m = (yy >= y) & (yy < y + t) & (xx >= xa) & (xx < xb)
            elif kind == 1:  # vertical stroke
                x = x0 + int(rng.integers(0, max(1, gw - t)))
                ya = int(rng.integers(1, CELL_H // 2))
                yb = min(CELL_H, ya + int(rng.integers(CELL_H // 3, CELL_H - 2)))
                m = (xx >= x) & (xx < x + t) & (yy >= ya) & (yy < yb)
            else:  # diagonal stroke
                xa = x0 + int(rng.integers(0, gw // 2))
                slope = rng.uniform(-1.2, 1.2)
                ya = rng.uniform(4, CELL_H - 4)
                m = (np.abs((yy - ya) - slope * (xx - xa)) < t * 0.6) & (xx >= xa) & (
                    xx < xa + gw // 2)
            # anti-aliased edge values like a rendered font
            val = rng.integers(0, 40)
            cell[m] = np.minimum(cell[m], val)
            n_ink = int((cell < 128).sum())
    return cells


def glyph_images(rng, batch, n_chars):
    """(B, 1, 24, 102*T) float32 in [0, 1] (white = 1.0)."""
    cells = glyph_cells(rng, batch * n_chars)
    img = cells.reshape(batch, n_chars, CELL_H, CELL_W).transpose(0, 2, 1, 3)
    img = img.reshape(batch, 1, CELL_H, n_chars * CELL_W)
    return (img.astype(np.float32) / np.float32(255.0))


def durations(rng, batch, n_src, total, src_lens=None):
    """Integer durations (B, n_src) float32, each >= 1 on valid tokens, row sum = total."""
    d = np.zeros((batch, n_src), dtype=np.float32)
    for b in range(batch):
        n = n_src if src_lens is None else int(src_lens[b])
        extra = rng.multinomial(total - n, np.ones(n) / n)
        d[b, :n] = 1 + extra
    return d


def mels(rng, batch, n_frames, n_mels=80, channels_last=False):
    """Log-mel spectrograms ~ clamp(N(-5, 2), log(1e-5), 2.5)."""
    m = rng.normal(-5.0, 2.0, size=(batch, n_mels, n_frames)).astype(np.float32)
    m = np.clip(m, np.float32(np.log(1e-5)), np.float32(2.5))
    return m.transpose(0, 2, 1).copy() if channels_last else m


def acoustic_batch(seed, batch, n_src, n_mel, ragged=False):
    """A teacher-forced acoustic batch in the positional order of ``vTTS.forward``.

    Returns a dict with numpy arrays: audiotypes, texts, src_lens, max_src_len,
    mels, mel_lens, max_mel_len, e_targets, d_targets, images.
    """
    rng = np.random.default_rng(seed)
    if ragged:
        src_lens = rng.integers(max(1, n_src // 3), n_src + 1, size=batch)
        src_lens[0] = n_src
    else:
        src_lens = np.full(batch, n_src)
    src_lens = src_lens.astype(np.int64)
    imgs = glyph_images(rng, batch, n_src)
    # padded characters are white (pad_2D_gray_image pads with 255)
    for b in range(batch):
        imgs[b, :, :, int(src_lens[b]) * CELL_W:] = 1.0
    d = durations(rng, batch, n_src, n_mel, src_lens)
    texts = rng.integers(1, 73, size=(batch, n_src)).astype(np.int64)
    for b in range(batch):
        texts[b, int(src_lens[b]):] = 0
    e = rng.normal(0.0, 1.0, size=(batch, n_src)).astype(np.float32)
    for b in range(batch):
        e[b, int(src_lens[b]):] = 0.0
    return dict(
        audiotypes=rng.integers(0, 10, size=batch).astype(np.int64),
        texts=texts,
        src_lens=src_lens,
        max_src_len=int(n_src),
        mels=mels(rng, batch, n_mel, channels_last=True),
        mel_lens=np.full(batch, n_mel, dtype=np.float32),
        max_mel_len=int(n_mel),
        e_targets=e,
        d_targets=d,
        images=imgs,
    )
